set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -k "prefetched_encoder_overflow" -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_r5b0.log 2>&1; tail -3 gpurun_out/pytest_r5b0.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread --deselect tests/test_gpu_train.py::test_prefetched_encoder_overflow_belongs_to_its_own_step > gpurun_out/pytest_r5b.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r5b.log
timeout -k 10 200 python -u scripts/bench_bbox.py > gpurun_out/bbox_bench.txt 2>&1; tail -6 gpurun_out/bbox_bench.txt
exit $rc
