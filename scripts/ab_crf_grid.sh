# CRF per-vertex grid: fixed 2048 blocks vs sized by the entry count -> gpurun_out/ab_crf_grid.txt
out=gpurun_out/ab_crf_grid.txt
for r in 1 2 3; do
  for v in 2048 0; do
    line=$(TCAM_CRF_PERSIST=$v timeout -k 10 120 python scripts/bench_crf.py 2>/dev/null) || exit 1
    echo "$r persist=$v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_call"], d.get("bitexact_vs_reference"))')" | tee -a "$out"
  done
done
