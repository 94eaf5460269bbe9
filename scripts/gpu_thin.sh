set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_model.py tests/test_gpu_family.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/thin_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/thin_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
ONLY=l1.c2,d2.c1,d3.c1,d3.c2,d4.c1,d4.c2 TILES=-1,1,4,17,20,23 timeout -k 10 200 python -u scripts/tune_conv_x6.py > gpurun_out/thin_tune.txt 2>&1
echo "tune rc=$?"; cat gpurun_out/thin_tune.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/thin_bench.json 2>/dev/null
echo "bench rc=$?"; cut -c1-300 gpurun_out/thin_bench.json
