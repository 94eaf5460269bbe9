set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_conv_x6.py > gpurun_out/tune_x6.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/tune_x6.log; exit $rc
