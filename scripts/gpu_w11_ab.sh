# A/B: wgrad11 block target (split count) on the stage-1 step, interleaved
set -o pipefail
d=gpurun_out/w11ab; mkdir -p $d
for r in 1 2; do
  for t in 1024 512 256; do
    for a in "" "--amp"; do
      TCAM_W11_BLOCKS=$t timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 $a > $d/b.json 2> $d/b.err || exit $?
      python -c 'import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d["train_prec"],d["value"],d["ms_per_step"])' $d/b.json $t | tee -a $d/summary.txt
    done
  done
done
