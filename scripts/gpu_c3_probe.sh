# Round 5: where the residual 1x1 (c3) launches spend their time — tile shapes and the
# debug switches (8 = no epilogue, 2 = no K-loop global loads after the first step,
# 16 = no residual prefetch), then the pending GPU test files.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PREC=f16x3 TILES=18,30,31,32,33,34 REPS=10 ONLY=l3.c3,l4.c3,l4.c3ds timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/c3_tiles.txt 2>&1 || { tail gpurun_out/c3_tiles.txt; exit 1; }
cat gpurun_out/c3_tiles.txt
for d in 8 2 16; do
  PREC=f16x3 DBG=$d TILES=18,30 REPS=10 ONLY=l3.c3,l4.c3 timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/c3_dbg$d.txt 2>&1 || { tail gpurun_out/c3_dbg$d.txt; exit 1; }
  echo "DBG=$d"; cat gpurun_out/c3_dbg$d.txt
done
PREC=f16x3 TILES=35 REPS=10 ONLY=d0.c1,l4.c2,l3.c2 timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/fp_prio0.txt 2>&1 && PREC=f16x3 DBG=512 TILES=35 REPS=10 ONLY=d0.c1,l4.c2,l3.c2 timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/fp_prio1.txt 2>&1 || exit 1
echo prio0; cat gpurun_out/fp_prio0.txt; echo prio1; cat gpurun_out/fp_prio1.txt
timeout -k 10 1100 python -u -m pytest tests/test_gpu_boxv2.py tests/test_gpu_entrypoints.py tests/test_gpu_train.py tests/test_gpu_ddp_train.py tests/test_gpu_parallel.py tests/test_gpu_model.py tests/test_gpu_autograd.py tests/test_gpu_f16.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_r5a.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r5a.log; exit $rc
