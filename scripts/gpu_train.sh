set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_train.log
