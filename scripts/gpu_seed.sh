set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_seed.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_seed.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Mismatch" gpurun_out/pytest_seed.log | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_seed.py > gpurun_out/bench_seed.json 2> gpurun_out/bench_seed.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_seed.json; tail -5 gpurun_out/bench_seed.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_seed -o seed -- python3 $GRAFT_REPO_ROOT/scripts/bench_seed.py > $GRAFT_REPO_ROOT/gpurun_out/prof_seed.log 2>&1
echo "prof rc=$?"
