# training kernels: their tests, the stage-1 bench (both precisions), the TCAM step bench
set -o pipefail
d=gpurun_out/${OUTDIR:-tall}
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_enc_train.py tests/test_gpu_ddp_train.py tests/test_gpu_train.py tests/test_gpu_amp.py \
  tests/test_gpu_autograd.py > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -2 $d/tests.log
for a in "" "--amp"; do
  timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 $a > $d/b.json 2> $d/b.err || exit $?
  python -c 'import json,sys;d=json.load(open(sys.argv[1]));print("stage1",d["train_prec"],d["value"],d["ms_per_step"],d["roofline"]["frac"])' $d/b.json | tee -a $d/summary.txt
  cp $d/b.json $d/stdcl${a:-_f16x3}.json
done
for a in "" "--amp"; do
  timeout -k 10 300 python scripts/bench_train.py --steps 6 --warmup 2 $a > $d/t.json 2> $d/t.err || exit $?
  python -c 'import json,sys;d=json.load(open(sys.argv[1]));print("tcam",sys.argv[2],d["value"],d["ms_per_step"])' $d/t.json "${a:-f16x3}" | tee -a $d/summary.txt
  cp $d/t.json $d/train${a:-_f16x3}.json
done
