set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_family.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "bbox or family or pool or rect or resize" > gpurun_out/pytest_fam.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_fam.log
[ $rc -eq 0 ] && bash scripts/gpu_family_bench.sh
