set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/timer_ab.txt
for r in 1 2 3; do
for v in window off all; do
  extra=""; [ $v = off ] && extra="--no-roofline-timer"; [ $v = all ] && extra="--timer-window 0"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt $extra > gpurun_out/timer_one.json 2> gpurun_out/timer.err || { tail -5 gpurun_out/timer.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/timer_one.json')); r=d.get('roofline') or {}; print('timer=$v', d['value'], r.get('frac'), r.get('avg_launch_ms'), r.get('conv_busy_ms_per_step'), r.get('launches_per_step'))" >> gpurun_out/timer_ab.txt
done
done
cat gpurun_out/timer_ab.txt
