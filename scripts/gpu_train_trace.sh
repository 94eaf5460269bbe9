# TCAM training step (configs[2], 256 frames): bench lines + kernel traces for the per-stream
# CU-time breakdown (scripts/stream_breakdown.py).  gpurun from the repo root.
set -o pipefail
mkdir -p gpurun_out/trace_train
export TMPDIR=/tmp
for p in ${PRECS:-amp f16x3}; do
  a=""; [ "$p" = amp ] && a="--amp"
  timeout -k 10 300 python scripts/bench_train.py $a --steps 8 --warmup 2 > "gpurun_out/trace_train/bench_$p.json" \
    2> "gpurun_out/trace_train/bench_$p.err" || exit $?
  cat "gpurun_out/trace_train/bench_$p.json" | cut -c1-300
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_train -o "$p" \
    -- python3 scripts/bench_train.py $a --steps 3 --warmup 1 > "gpurun_out/trace_train/$p.log" 2>&1 || exit $?
done
