set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_family.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/grow_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/grow_tests.log)"; fatal $rc; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/grow_tests.log | head; exit $rc; }
timeout -k 10 200 python scripts/diag_inc_phases.py 2>&1 | grep -v amdgpu.ids; fatal $?
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/grow_bench.json 2>/dev/null
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/grow_bench.json)"
