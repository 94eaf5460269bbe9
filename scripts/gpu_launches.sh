set -o pipefail
mkdir -p gpurun_out
TCAM_DUMP_LAUNCHES=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/launch_bench.json 2> gpurun_out/launch_dump.txt
echo "rc=$?"; grep "launch" gpurun_out/launch_dump.txt | head -80
