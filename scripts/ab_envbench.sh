# A/B of environment settings inside the pipelined headline bench, ROUNDS interleaved rounds on
# one box, with a heartbeat file -> gpurun_out/ab_env.txt
#   VARIANTS="base=X=0 nt=TCAM_X6_DEBUG=64" bash scripts/ab_envbench.sh
ROUNDS=${ROUNDS:-3}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
out=gpurun_out/ab_env.txt
for r in $(seq "$ROUNDS"); do
  for v in $VARIANTS; do
    name=${v%%=*}; kv=${v#*=}
    line=$(env "$kv" timeout -k 10 240 python bench.py --steps 60 --warmup 3 --no-cpu-baseline \
           --no-alt 2>>gpurun_out/ab_env.err) || { echo "variant $v failed"; exit 1; }
    echo "$r $name $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')" | tee -a "$out"
  done
done
