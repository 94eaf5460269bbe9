set -o pipefail
mkdir -p gpurun_out/prof_family
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_family.py > gpurun_out/bench_family.log 2> gpurun_out/bench_family.err
echo "bench rc=$?"; cat gpurun_out/bench_family.log; tail -3 gpurun_out/bench_family.err
timeout -k 10 300 python scripts/bench_frames.py > gpurun_out/bench_frames.log 2> gpurun_out/bench_frames.err
echo "frames rc=$?"; cat gpurun_out/bench_frames.log; tail -3 gpurun_out/bench_frames.err
