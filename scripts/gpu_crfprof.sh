# rocprofv3 kernel stats of the CRF filter bench (32 frames 224^2, K = 2)
set -o pipefail
mkdir -p gpurun_out/prof_crf
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_crf.py > gpurun_out/bench_crf.json 2> gpurun_out/bench_crf.err || exit $?
cat gpurun_out/bench_crf.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_crf -o crf \
  -- python3 scripts/bench_crf.py > gpurun_out/prof_crf/crf.log 2>&1 || exit $?
