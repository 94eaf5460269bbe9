# Drain of the last clip's bbox sweep on 1 vs 4 level ranges per frame (TCAM_BBOX_DRAIN_CHUNKS),
# at the driver's 20 steps and at 100, interleaved; then the bbox / evaluator GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_boxv2.py tests/test_gpu_fullsize.py -m gpu -x -q \
  --timeout 170 --timeout-method thread > gpurun_out/drain_tests.log 2>&1
rc=$?; tail -2 gpurun_out/drain_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/drain_ab.txt
for r in 1 2 3; do
for c in 1 4; do
  TCAM_BBOX_DRAIN_CHUNKS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt \
    > gpurun_out/drain_one.json 2> gpurun_out/drain.err || { tail -5 gpurun_out/drain.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/drain_one.json')); print('drain_chunks=$c steps=20', d['value'])" >> gpurun_out/drain_ab.txt
done
done
for c in 1 4; do
  TCAM_BBOX_DRAIN_CHUNKS=$c timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-alt \
    > gpurun_out/drain_one.json 2> gpurun_out/drain.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/drain_one.json')); print('drain_chunks=$c steps=100', d['value'])" >> gpurun_out/drain_ab.txt
done
cat gpurun_out/drain_ab.txt
