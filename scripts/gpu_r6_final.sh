# round 6 final evidence: headline bench (driver's command), its kernel stats, family benches
set -o pipefail
mkdir -p gpurun_out/r6f
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6f/bench20.json 2> gpurun_out/r6f/bench20.err || exit $?
tail -1 gpurun_out/r6f/bench20.json | cut -c1-200
timeout -k 10 400 python bench.py --gpus 1 --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r6f/bench100.json 2> gpurun_out/r6f/bench100.err || exit $?
tail -1 gpurun_out/r6f/bench100.json | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f/prof -o bench \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > gpurun_out/r6f/prof.log 2>&1 || exit $?
timeout -k 10 400 python scripts/bench_family.py > gpurun_out/r6f/family.jsonl 2> gpurun_out/r6f/family.err || exit $?
python -c "
import json
for l in open('gpurun_out/r6f/family.jsonl'):
    d=json.loads(l); print(d['workload'][:50], d['frames_per_s'], d['roofline']['frac'])
"
