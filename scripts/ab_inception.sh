# A/B of the InceptionV3 shard forward (scripts/bench_family.py --workload inceptionv3):
# branch convs one launch each (STAGES=0) vs the grouped stage launches with the automatic
# tile and forced tiles, ROUNDS interleaved rounds on one box -> gpurun_out/inc_ab.txt
ROUNDS=${ROUNDS:-2}
VARIANTS=${VARIANTS:-"0:-1 1:-1 1:18 1:17 1:20"}
mkdir -p gpurun_out
for r in $(seq "$ROUNDS"); do
  for v in $VARIANTS; do
    st=${v%%:*}; tile=${v##*:}
    line=$(TCAM_INCEPTION_STAGES=$st TCAM_INCEPTION_STAGE_TILE=$tile timeout -k 10 240 \
           python scripts/bench_family.py --workload inceptionv3 2>>gpurun_out/inc_ab.err) \
      || { echo "variant $v failed"; exit 1; }
    echo "round $r stages=$st tile=$tile $line" | tee -a gpurun_out/inc_ab.txt | cut -c1-300
  done
done
