set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{ for t in 14 7; do for xb in 2; do echo "TCAM_BNECK_TILE=$t XB=$xb"; TCAM_BNECK_XB=$xb TCAM_BNECK_TILE=$t PHASES=1 timeout -k 10 200 python scripts/bench_bneck.py || exit $?; done; done; } > gpurun_out/bneck_ph.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bneck_ph.txt; [ $rc -eq 0 ] || exit $rc
for t in 7 14; do for xb in 2; do
  TCAM_BNECK_XB=$xb TCAM_BNECK_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_bottleneck.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/bneck_tests_$t.log 2>&1
  rc=$?; echo "tile $t xb $xb: $(tail -1 gpurun_out/bneck_tests_$t.log)"; [ $rc -eq 0 ] || exit $rc
done; done
