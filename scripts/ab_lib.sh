# A/B of two builds of libtcam_hip.so on one GPU box (run through gpurun from the repo root):
#   gpurun -- 'bash scripts/ab_lib.sh [rounds]'
# B = tcam_wsol_video_amd/libtcam_hip_base.so (e.g. built from the previous commit),
# A = the in-tree libtcam_hip.so.  Alternates the headline bench (no CPU baseline, no fp32
# line) and, when ONLY is set, scripts/ab_x6.py per-layer timings; every step has its own
# time limit and the script stops at the first failure.  Output: gpurun_out/ab_lib.txt
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=tcam_wsol_video_amd/libtcam_hip_base.so
ROUNDS=${1:-2}
out=gpurun_out/ab_lib.txt
: > "$out"
for r in $(seq "$ROUNDS"); do
  for v in base new; do
    if [ "$v" = base ]; then lp=$BASE; else lp=""; fi
    line=$(TCAM_LIB_PATH=$lp timeout -k 10 300 python bench.py --steps 40 --warmup 3 \
           --no-cpu-baseline --no-alt 2> gpurun_out/ab_bench.err) || { echo "bench $v failed"; exit 1; }
    echo "$r $v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')" | tee -a "$out"
    if [ -n "${ONLY:-}" ]; then
      TCAM_LIB_PATH=$lp AB=${AB:-8} ROUNDS=3 timeout -k 10 300 python scripts/ab_x6.py \
        2>&1 | sed "s/^/$r $v /" | tee -a "$out" || exit 1
    fi
  done
done
