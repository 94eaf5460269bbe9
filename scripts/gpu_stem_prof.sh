set -o pipefail
mkdir -p gpurun_out/prof_stem
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_f16.py -m gpu -q -x -k "stem" --timeout 170 --timeout-method thread > gpurun_out/pytest_stem.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_stem.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stem -o stem -- python3 scripts/layer_times.py r50 > gpurun_out/prof_stem/lt.log 2>&1 || exit $?
grep -E "stem|from_nchw" gpurun_out/prof_stem/stem_kernel_stats.csv | cut -c1-250
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-alt > gpurun_out/bench_stem$i.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_stem$i.json'));print(d['value'], d['roofline']['frac'], d['roofline']['achieved'])"
TCAM_STEM_DIRECT=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-alt > gpurun_out/bench_nostem$i.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_nostem$i.json'));print('generic stem', d['value'], d['roofline']['frac'], d['roofline']['achieved'])"
done
