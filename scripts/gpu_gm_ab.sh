# Round 5: m-band tile order (TCAM_CONV_GM) — per-launch table and headline bench, one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for gm in 0 4 2; do
  TCAM_CONV_GM=$gm timeout -k 10 200 python -u scripts/layer_times.py r50 > gpurun_out/gm_layers_$gm.txt 2>&1 || { tail gpurun_out/gm_layers_$gm.txt; exit 1; }
  echo "GM=$gm"; head -12 gpurun_out/gm_layers_$gm.txt | grep -v amdgpu.ids
done
for r in 1 2; do
  for gm in 0 4 2; do
    TCAM_CONV_GM=$gm timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-alt > gpurun_out/gm_bench_${gm}_${r}.json 2> gpurun_out/gm_bench_${gm}_${r}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/gm_bench_${gm}_${r}.json'));print('GM=$gm', d['value'], d['roofline']['frac'])"
  done
done
