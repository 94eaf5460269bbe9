# BN kernels over coalesced 2-D grids: the training tests, then the stage-1 bench + profile
set -o pipefail
mkdir -p gpurun_out/bn_co
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_enc_train.py tests/test_gpu_train.py tests/test_gpu_amp.py tests/test_gpu_ddp_train.py \
  > gpurun_out/bn_co/tests.log 2>&1 || { tail -30 gpurun_out/bn_co/tests.log; exit 1; }
tail -3 gpurun_out/bn_co/tests.log
timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 > gpurun_out/bn_co/stdcl_f16x3.json 2> gpurun_out/bn_co/stdcl_f16x3.err || exit $?
cat gpurun_out/bn_co/stdcl_f16x3.json
timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 --amp > gpurun_out/bn_co/stdcl_amp.json 2> gpurun_out/bn_co/stdcl_amp.err || exit $?
cat gpurun_out/bn_co/stdcl_amp.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bn_co -o f16x3 \
    -- python3 scripts/bench_stdcl.py --steps 3 --warmup 1 > gpurun_out/bn_co/prof.log 2>&1 || exit $?
