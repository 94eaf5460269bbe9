set -o pipefail
mkdir -p gpurun_out/prof_train
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_train.log | tail -30; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_train.py --steps 5 --warmup 2 > gpurun_out/bench_train.log 2> gpurun_out/bench_train.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_train.log; tail -3 gpurun_out/bench_train.err; fatal $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o train -- python3 scripts/bench_train.py --steps 2 --warmup 1 > gpurun_out/prof_train.log 2>&1
echo "prof rc=$?"
