# Headline with the fused layer-1 bottleneck off / 14x14 tiles / 14x7 tiles, two interleaved
# rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/fused_ab.txt
for r in 1 2; do
for v in off 7; do
  if [ $v = off ]; then F=0; T=14; else F=1; T=$v; fi
  TCAM_FUSED_L1=$F TCAM_BNECK_TILE=$T timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-alt \
    > gpurun_out/fused_ab_one.json 2> gpurun_out/fused_ab.err || { tail -5 gpurun_out/fused_ab.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/fused_ab_one.json')); print('fused=$v', d['value'], d['roofline']['frac'])" >> gpurun_out/fused_ab.txt
done
done
cat gpurun_out/fused_ab.txt
