set -o pipefail
mkdir -p gpurun_out
for sk in -1 256; do
  SK=$sk ONLY=${ONLY:-l3.c1,l3.c2,l4.c1,l4.c2,d0.c1,l4.c3ds} TILES=${TILES:-14,15} timeout -k 10 300 python -u scripts/tune_conv_x6.py > gpurun_out/sk_g_$sk.txt 2>&1
  rc=$?; echo "sk=$sk rc=$rc"; cat gpurun_out/sk_g_$sk.txt; [ $rc -eq 0 ] || exit $rc
done
