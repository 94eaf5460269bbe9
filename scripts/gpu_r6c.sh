# round 6: CRF lattice without the global sort — parity, CRF profile, training diagnostics
set -o pipefail
mkdir -p gpurun_out/r6c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_crf.py tests/test_gpu_crf_scale.py > gpurun_out/r6c/crf_tests.log 2>&1 || { tail -30 gpurun_out/r6c/crf_tests.log; exit 1; }
tail -2 gpurun_out/r6c/crf_tests.log
bash scripts/gpu_crfprof.sh || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ddp_train.py > gpurun_out/r6c/ddp.log 2>&1 || { tail -30 gpurun_out/r6c/ddp.log; exit 1; }
tail -2 gpurun_out/r6c/ddp.log
for a in "" "--no-crf" "--amp" "--amp --no-crf"; do
  timeout -k 10 300 python scripts/bench_train.py --steps 6 --warmup 2 $a > gpurun_out/r6c/train.json 2>gpurun_out/r6c/train.err || exit $?
  echo "$a $(python -c 'import json;d=json.load(open("gpurun_out/r6c/train.json"));print(d["value"],d["ms_per_step"])')"
done
