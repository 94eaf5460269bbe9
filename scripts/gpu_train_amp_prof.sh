# AMP training step: bench line + rocprofv3 kernel stats (gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out/prof_amp
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_train.py --amp --steps 5 --warmup 2 > gpurun_out/bench_train_amp.json \
  2> gpurun_out/bench_train_amp.err || { tail -5 gpurun_out/bench_train_amp.err; exit 1; }
cat gpurun_out/bench_train_amp.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_amp -o amp \
  -- python3 scripts/bench_train.py --amp --steps 2 --warmup 1 > gpurun_out/prof_amp/amp.log 2>&1
