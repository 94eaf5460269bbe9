set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_model.py -x -q > gpurun_out/test_model.log 2>&1 &&
TCAM_DUMP_LAUNCHES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-budget 3 --no-alt > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/test_model.log; cat gpurun_out/bench.json; exit $rc
