set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
for s in 1 2 3 4; do
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-alt --fwd-streams $s > gpurun_out/streams_$s.json 2>/dev/null
rc=$?; echo "streams=$s rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/streams_$s.json)"; fatal $rc
done
