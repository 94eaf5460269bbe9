set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
for dbg in 0 2; do
  DBG=$dbg ONLY=l4.c2,l3.c2,d0.c1 TILES=14,22 REPS=10 timeout -k 10 200 python -u scripts/tune_conv_x6.py > gpurun_out/dbg_$dbg.txt 2>&1
  echo "dbg=$dbg rc=$?"; cat gpurun_out/dbg_$dbg.txt
done
export ONLY=l4.c2 TILES=14 REPS=3 SK=0
for dbg in 0 2; do
DBG=$dbg timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc2 -o d$dbg -- python3 scripts/tune_conv_x6.py > gpurun_out/pmc2/d$dbg.log 2>&1
echo "pmc dbg=$dbg rc=$?"
done
