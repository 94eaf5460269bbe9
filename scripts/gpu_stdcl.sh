# Stage-1 (STD_CL) training bench + kernel profile (run through gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out/prof_stdcl
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 > gpurun_out/stdcl_f16x3.json 2> gpurun_out/stdcl_f16x3.err || exit $?
cat gpurun_out/stdcl_f16x3.json
timeout -k 10 300 python scripts/bench_stdcl.py --steps 10 --warmup 3 --amp > gpurun_out/stdcl_amp.json 2> gpurun_out/stdcl_amp.err || exit $?
cat gpurun_out/stdcl_amp.json
for p in ${PROF:-f16x3}; do
  a=""; [ "$p" = amp ] && a="--amp"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stdcl -o "$p" \
    -- python3 scripts/bench_stdcl.py --steps 3 --warmup 1 $a > "gpurun_out/prof_stdcl/$p.log" 2>&1 || exit $?
done
