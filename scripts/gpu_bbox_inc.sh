set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/inc_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/inc_tests.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/bench_bbox.py > gpurun_out/inc_bbox.log 2>&1
echo "bbox rc=$?"; grep -v amdgpu gpurun_out/inc_bbox.log
timeout -k 10 300 python scripts/diag_bbox_cost.py > gpurun_out/inc_diag.txt 2>&1
echo "diag rc=$?"; grep round gpurun_out/inc_diag.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/inc_bench.json 2>/dev/null
echo "bench rc=$?"; cut -c1-250 gpurun_out/inc_bench.json
