set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python scripts/tune_conv.py > gpurun_out/tune.log 2>&1
echo "rc=$?"; cat gpurun_out/tune.log
