set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x6chk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/x6chk_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
TILES=${TILES:-14,10} timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/x6chk_tune.txt 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/x6chk_tune.txt; fatal $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/x6chk_bench.json 2> gpurun_out/x6chk_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/x6chk_bench.json
