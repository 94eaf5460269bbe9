# AMP training step with / without the fragment-prefetch 256x256 tile (TCAM_AMP_FP), two
# interleaved rounds, then tests/test_gpu_amp.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/amp_step_ab.txt
for v in 0 1 0 1; do
  echo "TCAM_AMP_FP=$v" >> gpurun_out/amp_step_ab.txt
  TCAM_AMP_FP=$v timeout -k 10 300 python scripts/bench_train.py --amp --steps 6 --warmup 2 \
    >> gpurun_out/amp_step_ab.txt 2> gpurun_out/amp_step_ab.err || { tail -5 gpurun_out/amp_step_ab.err; exit 1; }
done
cut -c1-200 gpurun_out/amp_step_ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_amp.py -m gpu -x -q --timeout 170 --timeout-method thread \
  > gpurun_out/amp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/amp_tests.log; exit $rc
