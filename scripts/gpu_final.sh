# Round artifacts in one call: GPU tests, smoke, PMC traffic passes (-> perfdata json the
# bench reports as roofline.traffic), the bench line, and the rocprofv3 kernel stats of the
# same bench with one forward stream (the stream the roofline pass times on).
set -o pipefail
mkdir -p gpurun_out/prof gpurun_out/pmc_traffic
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; fatal $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_traffic -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --fwd-streams 1 > gpurun_out/pmc_traffic/fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; fatal $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_traffic -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --fwd-streams 1 > gpurun_out/pmc_traffic/write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; fatal $rc
python scripts/pmc_traffic.py && cp tcam_wsol_video_amd/perfdata/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.log; fatal $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt --fwd-streams 1 > gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"; tail -1 gpurun_out/prof_bench.log | cut -c1-300
