set -o pipefail
mkdir -p gpurun_out/bprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bprof -o run -- python3 scripts/bench_bbox.py > gpurun_out/bbox.log 2>&1
echo "rc=$?"; grep bbox_levels gpurun_out/bbox.log
