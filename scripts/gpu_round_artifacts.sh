set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
# stop the whole call after a fault / abort / segfault / time limit (no further GPU steps)
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; fatal $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.log; fatal $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt --fwd-streams 1 > gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
