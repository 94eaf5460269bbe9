set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/xcd_bench_ab.txt
for r in 1 2 3; do
for v in 0 1; do
  TCAM_BNECK_XCD=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-alt > gpurun_out/xb_one.json 2> gpurun_out/xb.err || { tail -5 gpurun_out/xb.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/xb_one.json')); print('TCAM_BNECK_XCD=$v', d['value'], d['roofline']['frac'])" >> gpurun_out/xcd_bench_ab.txt
done
done
cat gpurun_out/xcd_bench_ab.txt
