set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
for nt in 512 1024; do
TCAM_BBOX_INC_NT=$nt timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/nt_$nt.log 2>&1
rc=$?; echo "nt=$nt tests rc=$rc $(tail -1 gpurun_out/nt_$nt.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
TCAM_BBOX_INC_NT=$nt timeout -k 10 200 python scripts/diag_inc_phases.py 2>&1 | grep -E "bbox_levels|max WG"; fatal $?
TCAM_BBOX_INC_NT=$nt timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/nt_bench_$nt.json 2>/dev/null
rc=$?; echo "nt=$nt bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/nt_bench_$nt.json)"; fatal $rc
done
