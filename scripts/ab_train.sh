# A/B of the fp32-accurate training step: 3x3 weight gradients on x6 (TCAM_WGRAD=x6) vs
# f16x3 (default), alternating on one box.  gpurun -- 'bash scripts/ab_train.sh [rounds]'
# Output: gpurun_out/ab_train.txt; every step has its own time limit, stops at first failure.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_train.txt
: > "$out"
for r in $(seq "${1:-2}"); do
  for v in x6 f16x3; do
    line=$(TCAM_WGRAD=$v timeout -k 10 300 python scripts/bench_train.py --steps 6 --warmup 2 \
           2> gpurun_out/ab_train.err) || { echo "train $v failed"; exit 1; }
    echo "$r $v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["losses_last"])')" | tee -a "$out"
  done
done
