set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_x6.py tests/test_gpu_model.py -x -q > gpurun_out/test_model.log 2>&1 &&
TILES=auto timeout -k 10 400 python scripts/tune_conv_x6.py > gpurun_out/tune_x6.log 2>&1 &&
TCAM_DUMP_LAUNCHES=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-budget 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "rc=$rc"; tail -15 gpurun_out/test_model.log; cat gpurun_out/tune_x6.log;  cat gpurun_out/bench.json; grep launch gpurun_out/bench.err | head -80; exit $rc
