set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_conv_x6.py > gpurun_out/tune_x6.log 2>&1 &&
timeout -k 10 400 python -m pytest tests/test_gpu_x6.py -x -q > gpurun_out/test_x6.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/tune_x6.log; tail -30 gpurun_out/test_x6.log; exit $rc
