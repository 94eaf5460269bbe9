set -o pipefail
mkdir -p gpurun_out
TCAM_DUMP_LAUNCHES=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>gpurun_out/bench.err
echo "bench rc=$?"
cat gpurun_out/bench.log; grep launch gpurun_out/bench.err
