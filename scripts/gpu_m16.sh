set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matches_fp64" > gpurun_out/m16_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/m16_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
TILES=${TILES:-4,17,3,18,0,19,1,20,2,21,10,15,11,14} timeout -k 10 400 python -u scripts/tune_conv_x6.py > gpurun_out/m16_tune.txt 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/m16_tune.txt
