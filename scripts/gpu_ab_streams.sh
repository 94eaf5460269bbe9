set -o pipefail
mkdir -p gpurun_out
for n in 1 2 3; do
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-alt --fwd-streams $n > gpurun_out/ab_$n.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1]);print($n, d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
