set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{ for st in 0 8 15 0 8 15; do echo "TCAM_BNECK_STAGGER=$st"; TCAM_BNECK_STAGGER=$st timeout -k 10 200 python scripts/bench_bneck.py || exit $?; done;
  for st in 0 12; do echo "TCAM_BNECK_STAGGER=$st phases"; TCAM_BNECK_STAGGER=$st PHASES=1 timeout -k 10 200 python scripts/bench_bneck.py || exit $?; done; } > gpurun_out/bneck_stagger.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bneck_stagger.txt; exit $rc
