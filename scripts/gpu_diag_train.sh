set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
TCAM_X6_NOLW=0 timeout -k 10 200 python -u scripts/diag_train_seeds.py > gpurun_out/diag_seeds0.log 2>&1; rc=$?; cat gpurun_out/diag_seeds0.log | tail -6; fatal $rc
TCAM_X6_NOLW=2 timeout -k 10 200 python -u scripts/diag_train_seeds.py > gpurun_out/diag_seeds2.log 2>&1; rc=$?; cat gpurun_out/diag_seeds2.log | tail -6; fatal $rc
