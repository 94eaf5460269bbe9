set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  TCAM_DUMP_LAUNCHES=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>gpurun_out/bench.err
  echo "bench rc=$?"
  cat gpurun_out/bench.log; grep launch gpurun_out/bench.err
fi
