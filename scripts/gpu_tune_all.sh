set -o pipefail
mkdir -p gpurun_out
REPS=5 timeout -k 10 600 python -u scripts/tune_conv_x6.py > gpurun_out/tune_all_r1.txt 2>&1
echo "tune rc=$?"; grep -v amdgpu gpurun_out/tune_all_r1.txt | cut -c1-75
