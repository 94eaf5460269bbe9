set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matches_fp64 and (-22- or -14-)" > gpurun_out/il_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/il_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
ONLY=l3.c1,l3.c2,l4.c1,l4.c2,l4.c3,l4.c3ds,d0.c1 TILES=14,22 REPS=10 timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/il_tune.txt 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/il_tune.txt
