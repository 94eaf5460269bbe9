# AMP fused layer-1 bottleneck: parity tests, then the AMP training step on / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bottleneck.py tests/test_gpu_amp.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/amp_fused_tests.log 2>&1
rc=$?; tail -3 gpurun_out/amp_fused_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/amp_fused_ab.txt
for r in 1 2; do
for v in 0 1; do
  TCAM_FUSED_L1=$v timeout -k 10 300 python scripts/bench_train.py --amp --steps 6 --warmup 2 > gpurun_out/af_one.json 2> gpurun_out/af.err || { tail -5 gpurun_out/af.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/af_one.json')); print('amp TCAM_FUSED_L1=$v', d['value'], d['ms_per_step'])" >> gpurun_out/amp_fused_ab.txt
done
done
cat gpurun_out/amp_fused_ab.txt
