set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matches_fp64 and (-23- or -24- or -25- or -26- or -27-)" > gpurun_out/lw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/lw_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
ONLY=l2.c1,l2.c2,d1.c1,l3.c1,l4.c1,l4.c3 TILES=10,15,25,26,14,23 REPS=10 timeout -k 10 200 python -u scripts/tune_conv_x6.py > gpurun_out/lw_tune2.txt 2>&1
echo "tune rc=$?"; cat gpurun_out/lw_tune2.txt
