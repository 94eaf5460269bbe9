# Round 5: fragment-prefetch tiles (35 / 36) — bit-identity vs tiles 30 / 26, per-layer A/B,
# then the headline bench with TCAM_CONV_FP=0 / 1 interleaved (one box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_f16.py -k "fragment_prefetch" -x -q --timeout 120 --timeout-method thread > gpurun_out/fp_bitid.log 2>&1 || { tail -20 gpurun_out/fp_bitid.log; exit 1; }
tail -2 gpurun_out/fp_bitid.log
PREC=f16x3 TILES=30,35,26,36 REPS=10 ONLY=d0.c1,l4.c2,l3.c2,l4.c1,l4.c3ds,l4.c3,l3.c1,d1.c1 timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/fp_tune.txt 2>&1 || { tail -20 gpurun_out/fp_tune.txt; exit 1; }
cat gpurun_out/fp_tune.txt
for r in 1 2; do
  for fp in 0 1; do
    TCAM_CONV_FP=$fp timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-alt > gpurun_out/fp_bench_${fp}_${r}.json 2> gpurun_out/fp_bench_${fp}_${r}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/fp_bench_${fp}_${r}.json'));print('FP=$fp', d['value'], d['roofline']['frac'])"
  done
done
