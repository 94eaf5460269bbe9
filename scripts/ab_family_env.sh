# A/B of environment settings in the InceptionV3 family bench, ROUNDS interleaved rounds
#   VARIANTS="base=X=0 heads=TCAM_CONV_TILE_MAP=1024x6912=31" bash scripts/ab_family_env.sh
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
out=gpurun_out/ab_family_env.txt
for r in $(seq "$ROUNDS"); do
  for v in $VARIANTS; do
    name=${v%%=*}; kv=${v#*=}
    line=$(env "$kv" timeout -k 10 200 python scripts/bench_family.py --workload inceptionv3 --steps 30 --warmup 3 \
           2>>gpurun_out/ab_family_env.err) || { echo "variant $v failed"; exit 1; }
    echo "$r $name $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["frames_per_s"], d["roofline"]["frac"])')" | tee -a "$out"
  done
done
