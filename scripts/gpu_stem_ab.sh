# Persistent vs one-tile-per-block stem: tests, per-kernel time (rocprofv3 over layer_times),
# and the pipelined headline A/B -> gpurun_out/prof_stem*/, gpurun_out/ab_env.txt
set -o pipefail
mkdir -p gpurun_out/prof_stem_p gpurun_out/prof_stem_o
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_f16.py tests/test_gpu_fullsize.py -m gpu -q -x -k "stem or r50" --timeout 170 --timeout-method thread > gpurun_out/pytest_stem.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_stem.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stem_p -o stem -- python3 scripts/layer_times.py r50 > gpurun_out/prof_stem_p/lt.log 2>&1 || exit $?
TCAM_STEM_ONE_TILE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stem_o -o stem -- python3 scripts/layer_times.py r50 > gpurun_out/prof_stem_o/lt.log 2>&1 || exit $?
grep -h stem gpurun_out/prof_stem_p/stem_kernel_stats.csv gpurun_out/prof_stem_o/stem_kernel_stats.csv | cut -c1-200
rm -f gpurun_out/ab_env.txt
ROUNDS=2 VARIANTS="persist=TCAM_STEM_ONE_TILE=0 onetile=TCAM_STEM_ONE_TILE=1" bash scripts/ab_envbench.sh
