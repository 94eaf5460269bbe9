# Short-run headline (the driver's 20 steps) with 1 / 2 level ranges per frame in the bbox sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/chunks_ab.txt
for r in 1 2 3; do
for c in 1 2; do
  TCAM_BBOX_INC_CHUNKS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt \
    > gpurun_out/chunks_one.json 2> gpurun_out/chunks.err || { tail -5 gpurun_out/chunks.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/chunks_one.json')); print('chunks=$c steps=20', d['value'])" >> gpurun_out/chunks_ab.txt
done
done
for c in 1 2; do
  TCAM_BBOX_INC_CHUNKS=$c timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-alt \
    > gpurun_out/chunks_one.json 2> gpurun_out/chunks.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/chunks_one.json')); print('chunks=$c steps=100', d['value'])" >> gpurun_out/chunks_ab.txt
done
cat gpurun_out/chunks_ab.txt
