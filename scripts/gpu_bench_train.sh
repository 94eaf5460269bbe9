set -o pipefail
mkdir -p gpurun_out/prof_train
export TMPDIR=/tmp
timeout -k 10 400 python scripts/bench_train.py --steps 5 --warmup 2 > gpurun_out/bench_train.log 2> gpurun_out/bench_train.err
echo "bench rc=$?"; cat gpurun_out/bench_train.log; tail -3 gpurun_out/bench_train.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o train -- python3 scripts/bench_train.py --steps 2 --warmup 1 > gpurun_out/prof_train.log 2>&1
echo "prof rc=$?"
