# A/B: wgrad11's split reduction fused into the kernel (last block per tile) vs the reduce kernel
set -o pipefail
d=gpurun_out/w11f; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_enc_train.py tests/test_gpu_ddp_train.py > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -2 $d/tests.log
for r in 1 2; do
  for f in 0 1; do
    for a in "" "--amp"; do
      TCAM_W11_FUSED=$f timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 $a > $d/b.json 2> $d/b.err || exit $?
      python -c 'import json,sys;d=json.load(open(sys.argv[1]));print("fused="+sys.argv[2], d["train_prec"],d["value"],d["ms_per_step"])' $d/b.json $f | tee -a $d/summary.txt
    done
  done
done
