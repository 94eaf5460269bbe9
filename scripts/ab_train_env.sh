# A/B of environment settings on the training step (scripts/bench_train.py), interleaved,
# with a heartbeat -> gpurun_out/ab_train_env.txt
#   VARIANTS="base=X=0 pipe=TCAM_WGRAD_PIPE=1" ARGS="--amp" bash scripts/ab_train_env.sh
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
out=gpurun_out/ab_train_env.txt
for r in $(seq "$ROUNDS"); do
  for v in $VARIANTS; do
    name=${v%%=*}; kv=${v#*=}
    line=$(env "$kv" timeout -k 10 300 python scripts/bench_train.py $ARGS 2>>gpurun_out/ab_train_env.err) \
      || { echo "variant $v failed"; exit 1; }
    echo "$r $name $ARGS $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$out"
  done
done
