# Fused layer-1 bottleneck: parity tests for both tile shapes, then its time against the
# unfused convs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 7 14; do
  TCAM_BNECK_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_bottleneck.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/bneck_tests_$t.log 2>&1
  rc=$?; echo "tile $t"; tail -3 gpurun_out/bneck_tests_$t.log; [ $rc -eq 0 ] || exit $rc
done
: > gpurun_out/bneck_bench.txt
for t in 14 7 14 7; do
  echo "TCAM_BNECK_TILE=$t" >> gpurun_out/bneck_bench.txt
  TCAM_BNECK_TILE=$t timeout -k 10 200 python scripts/bench_bneck.py >> gpurun_out/bneck_bench.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/bneck_bench.txt
