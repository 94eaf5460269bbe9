# A/B of the 256x192 tile (37) on InceptionV3 (SPG heads) and the f16 tile tests for it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{ for v in 0 1 0 1; do
    echo "TCAM_CONV_T192=$v"
    TCAM_CONV_T192=$v timeout -k 10 200 python scripts/bench_family.py --workload inceptionv3 --steps 20 || exit $?
  done; } > gpurun_out/t192_ab.txt 2>&1 || { tail -5 gpurun_out/t192_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t192_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_f16.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "37" > gpurun_out/t192_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t192_tests.log; exit $rc
