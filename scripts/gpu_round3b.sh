# one GPU call: the AMP tests with their printed errors, the full -m gpu suite, smoke, the
# headline bench, the fp32-accurate and AMP training benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_amp.py -m gpu -q -s -k "oracle or close" --timeout 170 --timeout-method thread > gpurun_out/pytest_amp_s.log 2>&1 || exit $?
grep -E "amp seeds|passed|failed" gpurun_out/pytest_amp_s.log
bash scripts/gpu.sh tests smoke bench || exit $?
timeout -k 10 400 python scripts/bench_train.py --steps 5 --warmup 2 > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || exit $?
cat gpurun_out/bench_train.json
timeout -k 10 400 python scripts/bench_train.py --steps 5 --warmup 2 --amp > gpurun_out/bench_train_amp.json 2> gpurun_out/bench_train_amp.err || exit $?
cat gpurun_out/bench_train_amp.json
