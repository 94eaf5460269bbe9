set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bottleneck.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bneck_xcd_tests.log 2>&1
rc=$?; tail -1 gpurun_out/bneck_xcd_tests.log; [ $rc -eq 0 ] || exit $rc
{ for v in 0 1 0 1; do echo "TCAM_BNECK_XCD=$v"; TCAM_BNECK_XCD=$v timeout -k 10 200 python scripts/bench_bneck.py || exit $?; done;
  for v in 0 1; do echo "TCAM_BNECK_XCD=$v phases"; TCAM_BNECK_XCD=$v PHASES=1 timeout -k 10 200 python scripts/bench_bneck.py || exit $?; done; } > gpurun_out/bneck_xcd.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bneck_xcd.txt; exit $rc
