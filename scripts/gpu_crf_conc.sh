set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_crf.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/crf_conc.log 2>&1
rc=$?; echo "crf tests rc=$rc"; tail -3 gpurun_out/crf_conc.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_family_bench.sh
