set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -x -q -k "bbox or box" > gpurun_out/test_bbox.log 2>&1 &&
timeout -k 10 300 python scripts/bench_bbox.py > gpurun_out/bench_bbox.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 gpurun_out/test_bbox.log; cat gpurun_out/bench_bbox.log | grep -v amdgpu.ids; exit $rc
