# A/B: threads per frame of the sorted-list level sweep (TCAM_BBOX_SORTED_THREADS 1024 / 512)
set -o pipefail
d=gpurun_out/bbnt; mkdir -p $d
TCAM_BBOX_SORTED_THREADS=512 timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "bbox or level" > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -2 $d/tests.log
for r in 1 2; do
  for t in 1024 512; do
    TCAM_BBOX_SORTED_THREADS=$t timeout -k 10 200 python scripts/bench_bbox.py > $d/bb.txt 2>&1 || exit $?
    echo "nt=$t $(grep 'bbox_levels' $d/bb.txt | head -1)" | tee -a $d/summary.txt
  done
done
for r in 1 2; do
  for t in 1024 512; do
    TCAM_BBOX_SORTED_THREADS=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt > $d/b.json 2> $d/b.err || exit $?
    echo "nt=$t bench $(python -c 'import json;d=json.loads(open("'$d'/b.json").read().strip().splitlines()[-1]);print(d["value"])')" | tee -a $d/summary.txt
  done
done
