# stage-1 step: encoder-training tests, both benches, kernel profiles of both precisions
set -o pipefail
d=gpurun_out/${OUTDIR:-stdcl2}
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_enc_train.py tests/test_gpu_ddp_train.py ${EXTRA_TESTS} > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -2 $d/tests.log
for a in "" "--amp"; do
  timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 $a > $d/b.json 2> $d/b.err || exit $?
  python -c 'import json,sys;d=json.load(open(sys.argv[1]));print(d["train_prec"],d["value"],d["ms_per_step"],d["roofline"]["frac"])' $d/b.json | tee -a $d/summary.txt
  cp $d/b.json $d/bench${a:-_f16x3}.json
done
for p in f16x3 amp; do
  a=""; [ $p = amp ] && a="--amp"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o $p \
    -- python3 scripts/bench_stdcl.py --steps 3 --warmup 1 $a > $d/prof_$p.log 2>&1 || exit $?
done
