set -o pipefail
for r in 1 2; do for v in base new; do
  if [ $v = base ]; then lp=tcam_wsol_video_amd/libtcam_hip_base.so; else lp=""; fi
  for w in inceptionv3 vgg16; do
    TCAM_LIB_PATH=$lp timeout -k 10 200 python scripts/bench_family.py --workload $w --steps 30 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $v $w', d['frames_per_s'], d['roofline']['frac'])" || exit 1
  done
done; done
