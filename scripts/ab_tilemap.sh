# A/B of per-shape tile choices inside the pipelined headline bench (TCAM_CONV_TILE_MAP,
# "<Cout>x<K>=<id>,..."), ROUNDS interleaved rounds on one box -> gpurun_out/ab_tilemap.txt
#   VARIANTS="base= l4c3t18=2048x512=18" bash scripts/ab_tilemap.sh
ROUNDS=${ROUNDS:-3}
VARIANTS=${VARIANTS:-"base= l4c3t18=2048x512=18"}
mkdir -p gpurun_out
out=gpurun_out/ab_tilemap.txt
for r in $(seq "$ROUNDS"); do
  for v in $VARIANTS; do
    name=${v%%=*}; map=${v#*=}
    line=$(TCAM_CONV_TILE_MAP=$map timeout -k 10 240 python bench.py --steps 60 --warmup 3 \
           --no-cpu-baseline --no-alt 2>>gpurun_out/ab_tilemap.err) || { echo "variant $v failed"; exit 1; }
    echo "$r $name $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')" | tee -a "$out"
  done
done
