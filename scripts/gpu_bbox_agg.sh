# bbox level sweep with / without per-wave combining (TCAM_BBOX_AGG): phase profile, cost to the
# pipelined bench, bench lines, then the bbox GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{ for v in 0 1; do
    echo "== TCAM_BBOX_AGG=$v"
    TCAM_BBOX_AGG=$v timeout -k 10 200 python scripts/diag_inc_phases.py || exit $?
  done
  for v in 0 1; do
    echo "== TCAM_BBOX_AGG=$v cost"
    TCAM_BBOX_AGG=$v timeout -k 10 200 python scripts/diag_bbox_cost.py || exit $?
  done; } > gpurun_out/bbox_agg.txt 2>&1 || { tail -5 gpurun_out/bbox_agg.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bbox_agg.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_boxv2.py tests/test_gpu_model.py -m gpu -x -q \
  --timeout 170 --timeout-method thread -k "bbox or box or cam" > gpurun_out/bbox_agg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bbox_agg_tests.log; exit $rc
