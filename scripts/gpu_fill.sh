set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/bench_bbox.py > gpurun_out/bbox_bench.txt 2>&1 || { tail gpurun_out/bbox_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bbox_bench.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_boxv2.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_fill.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fill.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-alt > gpurun_out/fill_bench_$r.json 2> gpurun_out/fill_bench_$r.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fill_bench_$r.json'));print('bench', d['value'], d['roofline']['frac'])"
done
