set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
export ONLY=${ONLY:-l4.c2} TILES=${TILES:-11,14} REPS=3 SK=0
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc -o x1 -- python3 scripts/tune_conv_x6.py > gpurun_out/pmc/x1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc -o x2 -- python3 scripts/tune_conv_x6.py > gpurun_out/pmc/x2.log 2>&1
echo rc=$?
ls -R gpurun_out/pmc | head -30
