# InceptionV3 shard rate vs forward streams (2/3/4), one box; plus the headline's side rates
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/inc_streams.txt
: > "$out"
for ns in 2 3 4 2; do
  TCAM_FAMILY_FWD_STREAMS=$ns timeout -k 10 300 python scripts/bench_family.py --workload inceptionv3 > gpurun_out/inc.jsonl 2> gpurun_out/inc.err || exit 1
  echo "streams=$ns $(python -c 'import json;d=json.loads(open("gpurun_out/inc.jsonl").readline());print(d["frames_per_s"], d["roofline"]["frac"])')" | tee -a "$out"
done
