set -o pipefail
mkdir -p gpurun_out/prof_crf
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_crf -o crf -- python3 scripts/bench_crf.py > gpurun_out/prof_crf.log 2>&1
echo "prof rc=$?"
f=$(find gpurun_out/prof_crf -name "*kernel_stats.csv" | head -1); cut -d, -f1-4,7 "$f" | head -30
