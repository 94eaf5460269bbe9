# fp32-accurate training step with the fused layer-1 bottleneck on / off (its frozen encoder
# runs the f16x3 plan), two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/train_fused_ab.txt
for r in 1 2; do
for v in 0 1; do
  TCAM_FUSED_L1=$v timeout -k 10 300 python scripts/bench_train.py --steps 5 --warmup 2 > gpurun_out/tf_one.json 2> gpurun_out/tf.err || { tail -5 gpurun_out/tf.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/tf_one.json')); print('TCAM_FUSED_L1=$v', d['value'], d['ms_per_step'])" >> gpurun_out/train_fused_ab.txt
done
done
cat gpurun_out/train_fused_ab.txt
