# Per-phase time of the sorted-list level sweep on the bench clip's CAMs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TCAM_LEVEL_VARIANT=0 timeout -k 10 200 python scripts/diag_inc_phases.py > gpurun_out/phases.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/phases.txt; exit $rc
