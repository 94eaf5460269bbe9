# GPU-box driver (run through gpurun from the repo root):
#   gpurun --timeout 900 -- 'bash scripts/gpu.sh <step> [<step> ...]'
# Steps run in order and the script stops at the first failure (every GPU step has its
# own time limit; a fault, abort or time limit ends the call).  Outputs go to gpurun_out/.
#
#   tests                pytest -m gpu ($PYTEST_FILES, default tests/; $PYTEST_K: -k filter)
#   smoke                __graft_entry__.smoke()
#   bench                bench.py headline line (N=1)            -> gpurun_out/bench.json
#   prof                 rocprofv3 --kernel-trace --stats of the exact headline command
#                        (2 forward streams)                     -> gpurun_out/prof/
#   pmc                  PMC passes over the headline command: FETCH_SIZE, WRITE_SIZE,
#                        MFMA busy / GRBM_GUI_ACTIVE             -> gpurun_out/pmc/
#   traffic              pmc + scripts/pmc_traffic.py -> perfdata/pmc_traffic.json
#   family               scripts/bench_family.py (VGG16+CRF, InceptionV3 shard)
#   train                scripts/bench_train.py + its rocprof stats
#   crf | seed | frames | jpeg | e2e  the per-component benches (e2e: CAM+bbox from JPEG files)
#   jpegprof             rocprofv3 --kernel-trace --stats of scripts/bench_jpeg.py -> gpurun_out/prof_jpeg/
#   layererr             scripts/layer_error.py (per-layer error of x6 / f16x3 vs fp64) -> gpurun_out/layer_error.txt
#   layers               scripts/layer_times.py r50 (per-launch conv times) -> gpurun_out/layer_times.txt
#   incphases            scripts/diag_inc_phases.py for the incremental and the sorted-list sweeps
#   bboxprof             rocprofv3 --kernel-trace --stats of scripts/bench_bbox.py -> gpurun_out/prof_bbox/
#   bboxcost             scripts/diag_bbox_cost.py (headline loop with / without the bbox stage)
#   tune                 scripts/tune_conv_x6.py (per-layer tile timings)
#   ab                   scripts/ab_x6.py (debug-flag A/B of the x6 conv, one process; $AB, $ONLY)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline --no-alt"}
stop() { echo "step $1 failed rc=$2"; exit "$2"; }

run_step() {
  case "$1" in
  tests)
    kargs=(); [ -n "${PYTEST_K:-}" ] && kargs=(-k "$PYTEST_K")
    timeout -k 10 1150 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 170 \
      --timeout-method thread "${kargs[@]}" > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; tail -5 gpurun_out/pytest_gpu.log; return $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; tail -2 gpurun_out/smoke.log; return $rc ;;
  bench)
    timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
    rc=$?; cat gpurun_out/bench.json; return $rc ;;
  prof)
    mkdir -p gpurun_out/prof
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
      -- python3 bench.py $BENCH_ARGS > gpurun_out/prof/bench.log 2>&1
    rc=$?; tail -1 gpurun_out/prof/bench.log | cut -c1-400; return $rc ;;
  pmc)
    mkdir -p gpurun_out/pmc
    for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
      name=$(echo "$pass" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
      timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/pmc \
        -o "$name" -- python3 bench.py $BENCH_ARGS > "gpurun_out/pmc/$name.log" 2>&1 || return $?
    done ;;
  traffic)
    run_step pmc || return $?
    python scripts/pmc_traffic.py && cp tcam_wsol_video_amd/perfdata/pmc_traffic.json gpurun_out/ ;;
  family)
    timeout -k 10 400 python scripts/bench_family.py > gpurun_out/bench_family.jsonl 2> gpurun_out/bench_family.err
    rc=$?; cat gpurun_out/bench_family.jsonl; return $rc ;;
  train)
    mkdir -p gpurun_out/prof_train
    timeout -k 10 400 python scripts/bench_train.py --steps 5 --warmup 2 > gpurun_out/bench_train.json \
      2> gpurun_out/bench_train.err || return $?
    cat gpurun_out/bench_train.json
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o train \
      -- python3 scripts/bench_train.py --steps 2 --warmup 1 > gpurun_out/prof_train/train.log 2>&1 ;;
  crf|seed|frames|jpeg|e2e)
    timeout -k 10 300 python "scripts/bench_$1.py" > "gpurun_out/bench_$1.json" 2> "gpurun_out/bench_$1.err"
    rc=$?; cat "gpurun_out/bench_$1.json"; return $rc ;;
  jpegprof)
    mkdir -p gpurun_out/prof_jpeg
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jpeg -o jpeg \
      -- python3 scripts/bench_jpeg.py > gpurun_out/prof_jpeg/jpeg.log 2>&1
    rc=$?; tail -1 gpurun_out/prof_jpeg/jpeg.log | cut -c1-300; return $rc ;;
  layererr)
    timeout -k 10 300 python scripts/layer_error.py > gpurun_out/layer_error.txt 2> gpurun_out/layer_error.err
    rc=$?; tail -3 gpurun_out/layer_error.txt; return $rc ;;
  layers)
    timeout -k 10 300 python scripts/layer_times.py r50 > gpurun_out/layer_times.txt 2>&1
    rc=$?; head -12 gpurun_out/layer_times.txt; return $rc ;;
  incphases)
    { TCAM_LEVEL_VARIANT=2 timeout -k 10 120 python scripts/diag_inc_phases.py &&
      TCAM_LEVEL_VARIANT=0 timeout -k 10 120 python scripts/diag_inc_phases.py &&
      TCAM_BBOX_COMPRESS=0 TCAM_LEVEL_VARIANT=0 timeout -k 10 120 python scripts/diag_inc_phases.py &&
      TCAM_BBOX_INC_CHUNKS=1 TCAM_LEVEL_VARIANT=0 timeout -k 10 120 python scripts/diag_inc_phases.py; } > gpurun_out/inc_phases.txt 2>&1
    rc=$?; cat gpurun_out/inc_phases.txt | grep -v amdgpu.ids; return $rc ;;
  bboxprof)
    mkdir -p gpurun_out/prof_bbox
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bbox -o bbox \
      -- python3 scripts/bench_bbox.py > gpurun_out/prof_bbox/bbox.log 2>&1
    rc=$?; grep "fill" gpurun_out/prof_bbox/bbox.log; return $rc ;;
  bboxdet)
    timeout -k 10 300 python scripts/diag_bbox_determinism.py diag_data/bench_cam_u8.npy > gpurun_out/bbox_det.txt 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/bbox_det.txt; return $rc ;;
  bboxcost)
    timeout -k 10 300 python scripts/diag_bbox_cost.py > gpurun_out/bbox_cost.txt 2>&1
    rc=$?; tail -4 gpurun_out/bbox_cost.txt; return $rc ;;
  tune)
    timeout -k 10 600 python scripts/tune_conv_x6.py > gpurun_out/tune.txt 2>&1
    rc=$?; tail -40 gpurun_out/tune.txt; return $rc ;;
  ab)
    timeout -k 10 600 python scripts/ab_x6.py > gpurun_out/ab.txt 2>&1
    rc=$?; tail -40 gpurun_out/ab.txt; return $rc ;;
  *) echo "unknown step $1"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  run_step "$s" || stop "$s" $?
done
