set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
for c in 1 2 3 4; do
TCAM_BBOX_INC_CHUNKS=$c timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k bbox > gpurun_out/inc_c$c.log 2>&1
rc=$?; echo "chunks=$c tests rc=$rc $(tail -1 gpurun_out/inc_c$c.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
TCAM_BBOX_INC_CHUNKS=$c timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/inc_bench_c$c.json 2>/dev/null
rc=$?; echo "chunks=$c bench rc=$rc $(cut -c1-200 gpurun_out/inc_bench_c$c.json | grep -o '"value": [0-9.]*')"; fatal $rc
done
