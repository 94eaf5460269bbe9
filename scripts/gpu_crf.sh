set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_crf.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_crf.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_crf.log
if [ $rc -eq 0 ]; then
  timeout -k 10 180 python scripts/bench_crf.py > gpurun_out/bench_crf.log 2>&1; echo "bench rc=$?"; cat gpurun_out/bench_crf.log
fi
