set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
export ONLY=l4.c2 TILES=0,6 REPS=3
timeout -k 10 300 python scripts/tune_conv.py
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc -o p1 -- python3 scripts/tune_conv.py > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc -o p2 -- python3 scripts/tune_conv.py > /dev/null 2>&1
echo rc=$?
ls gpurun_out/pmc
