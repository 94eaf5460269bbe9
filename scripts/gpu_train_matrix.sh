# Training-step matrix on one box: precision x (encoder prefetch on/off) x (CRF on/off)
# gpurun -- 'bash scripts/gpu_train_matrix.sh'   -> gpurun_out/train_matrix.txt
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/train_matrix.txt
: > "$out"
for prec in "" "--amp"; do
  for pf in 1 0; do
    for crf in "" "--no-crf"; do
      TCAM_ENC_PREFETCH=$pf timeout -k 10 300 python scripts/bench_train.py --steps 6 --warmup 2 $prec $crf \
        > gpurun_out/tm.json 2> gpurun_out/tm.err || { echo "failed: $prec $pf $crf"; exit 1; }
      echo "prec=${prec:-f16x3} prefetch=$pf crf=${crf:-on} $(python -c 'import json;d=json.load(open("gpurun_out/tm.json"));print(d["value"],d["ms_per_step"])')" | tee -a "$out"
    done
  done
done
