# TCAM decoder training step (256 frames), both precisions, + a kernel profile of the f16x3 step
set -o pipefail
mkdir -p gpurun_out/trq
export TMPDIR=/tmp
for prec in "" "--amp"; do
  timeout -k 10 300 python scripts/bench_train.py --steps 6 --warmup 2 $prec > gpurun_out/trq/t.json 2> gpurun_out/trq/t.err || exit $?
  echo "prec=${prec:-f16x3} $(python -c 'import json;d=json.load(open("gpurun_out/trq/t.json"));print(d["value"],d["ms_per_step"])')" | tee -a gpurun_out/trq/summary.txt
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trq -o f16x3 \
    -- python3 scripts/bench_train.py --steps 3 --warmup 1 > gpurun_out/trq/prof.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trq -o amp \
    -- python3 scripts/bench_train.py --steps 3 --warmup 1 --amp > gpurun_out/trq/prof_amp.log 2>&1 || exit $?
