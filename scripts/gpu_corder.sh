set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matches_fp64" > gpurun_out/corder_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/corder_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
for dbg in 4 0; do
  DBG=$dbg TILES=${TILES:-14,10} timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/corder_$dbg.txt 2>&1
  rc=$?; echo "dbg=$dbg rc=$rc"; cat gpurun_out/corder_$dbg.txt; [ $rc -eq 0 ] || exit $rc
done
