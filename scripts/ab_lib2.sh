# Like ab_lib.sh, with a heartbeat file (gpurun kills a call that writes nothing for 180 s; a
# fresh box's first bench can take that long before its one JSON line)
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
BASE=tcam_wsol_video_amd/libtcam_hip_base.so
ROUNDS=${1:-2}
out=gpurun_out/ab_lib.txt
: > "$out"
for r in $(seq "$ROUNDS"); do
  for v in new base; do
    if [ "$v" = base ]; then lp=$BASE; else lp=""; fi
    line=$(TCAM_LIB_PATH=$lp timeout -k 10 300 python bench.py --steps 40 --warmup 3 \
           --no-cpu-baseline --no-alt 2> gpurun_out/ab_bench_$v.err) || { echo "bench $v failed rc=$?" | tee -a "$out"; exit 1; }
    echo "$r $v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')" | tee -a "$out"
  done
done
