# HBM traffic of the dominant kernel family (conv_x6) per launch, from PMC counters
# (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in separate passes; gfx950's
# FETCH_SIZE counts half the bytes of 16-B/lane streaming reads -> doubled).
set -o pipefail
mkdir -p gpurun_out/pmc_traffic
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_traffic -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/pmc_traffic/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_traffic -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/pmc_traffic/write.log 2>&1
echo "pmc rc=$?"
find gpurun_out/pmc_traffic -name "*counter_collection*" | head
