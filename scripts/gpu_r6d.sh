# round 6: training step after a CRF change (CRF on), plus the CRF-using GPU tests
set -o pipefail
mkdir -p gpurun_out/r6d
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crf.py tests/test_gpu_crf_scale.py $(ls tests/test_gpu_*train*.py tests/test_gpu_loss*.py 2>/dev/null) > gpurun_out/r6d/tests.log 2>&1 || { tail -30 gpurun_out/r6d/tests.log; exit 1; }
tail -2 gpurun_out/r6d/tests.log
for a in "" "--amp"; do
  timeout -k 10 300 python scripts/bench_train.py --steps 6 --warmup 2 $a > gpurun_out/r6d/train.json 2>gpurun_out/r6d/train.err || exit $?
  echo "$a $(python -c 'import json;d=json.load(open("gpurun_out/r6d/train.json"));print(d["value"],d["ms_per_step"],d["losses_last"])')"
done
