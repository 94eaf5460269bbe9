set -o pipefail
mkdir -p gpurun_out/prof_train
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 300 python scripts/bench_family.py > gpurun_out/bench_family.log 2> gpurun_out/bench_family.err
rc=$?; echo "family rc=$rc"; cut -c1-200 gpurun_out/bench_family.log; fatal $rc
timeout -k 10 400 python scripts/bench_train.py --steps 5 --warmup 2 > gpurun_out/bench_train.log 2> gpurun_out/bench_train.err
rc=$?; echo "train rc=$rc"; cut -c1-200 gpurun_out/bench_train.log; fatal $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o train -- python3 scripts/bench_train.py --steps 2 --warmup 1 > gpurun_out/prof_train.log 2>&1
echo "prof rc=$?"
