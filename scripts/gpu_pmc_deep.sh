# PMC passes over single deep f16x3 conv layers (scripts/ab_f16.py, auto tile):
#   bash scripts/gpu_pmc_deep.sh   -> gpurun_out/pmc_deep/<pass>.csv (+ .log)
# one rocprofv3 run per counter set (SQ <= 8, GRBM <= 2 per pass)
set -o pipefail
mkdir -p gpurun_out/pmc_deep
export TMPDIR=/tmp ONLY=${ONLY:-l4.c2,d0.c1,l4.c3} VARIANTS=auto ROUNDS=2 REPS=4
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
            "SQ_INSTS_MFMA SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/pmc_deep \
    -o "pass$i" -- python3 scripts/ab_f16.py > "gpurun_out/pmc_deep/pass$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -3 "gpurun_out/pmc_deep/pass$i.log"; }
done
ls gpurun_out/pmc_deep
