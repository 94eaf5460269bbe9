# Headline with the fused layer-1 bottleneck on / off (TCAM_FUSED_L1), two interleaved rounds,
# then the ResNet50 parity suites with the fusion on.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/fused_ab.txt
for v in 0 1 0 1; do
  TCAM_FUSED_L1=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-alt \
    > gpurun_out/fused_ab_one.json 2> gpurun_out/fused_ab.err || { tail -5 gpurun_out/fused_ab.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/fused_ab_one.json')); print('TCAM_FUSED_L1=$v', d['value'], d['roofline']['frac'])" >> gpurun_out/fused_ab.txt
done
cat gpurun_out/fused_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_gpu_bottleneck.py -m gpu -x -q \
  --timeout 170 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fused_tests.log; exit $rc
