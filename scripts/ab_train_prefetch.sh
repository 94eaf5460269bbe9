# Next-batch encoder forward prefetched on a side stream vs not, in the training bench (fp32-accurate and AMP),
# ROUNDS interleaved rounds -> gpurun_out/ab_train_prefetch.txt (heartbeat file)
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
out=gpurun_out/ab_train_prefetch.txt
for r in $(seq "$ROUNDS"); do
  for amp in "" "--amp"; do
    for v in 1 0; do
      line=$(TCAM_ENC_PREFETCH=$v timeout -k 10 300 python scripts/bench_train.py --steps 5 --warmup 2 $amp \
             2>>gpurun_out/ab_train_prefetch.err) || { echo "prefetch=$v $amp failed"; exit 1; }
      echo "$r prefetch=$v ${amp:-fp32acc} $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$out"
    done
  done
done
