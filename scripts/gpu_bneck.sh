# Fused layer-1 bottleneck: parity tests, then its time against the unfused convs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bottleneck.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/bneck_tests.log 2>&1
rc=$?; tail -15 gpurun_out/bneck_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/bench_bneck.py > gpurun_out/bneck_bench.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bneck_bench.txt; exit $rc
