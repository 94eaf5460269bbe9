# A/B of the AMP (FmtH1) 256x256 rings: 3 stages (t31) vs 4 stages (t38 32x32x16, t39 16x16x32)
# at the training step's 256 frames, then the AMP tile tests for the new ids.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FMT=amp FRAMES=256 ROUNDS=5 REPS=5 ONLY=${ONLY:-l4.c1,l4.c2,l4.c3ds,d0.c1,l3.c1,l3.c2,l4.c3} \
  VARIANTS=auto,t31,t39,t40,t41 timeout -k 10 400 python scripts/ab_f16.py > gpurun_out/amp_ring.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/amp_ring.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_amp.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "39 or 40 or 41" > gpurun_out/amp_ring_tests.log 2>&1
rc=$?; tail -3 gpurun_out/amp_ring_tests.log; exit $rc
