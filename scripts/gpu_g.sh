set -o pipefail
mkdir -p gpurun_out
export ONLY=l2.c1,l2.c2,l3.c1,l3.c2,l3.c3,l4.c1,l4.c2,l4.c3,l4.c3ds,d0.c1,d1.c1,d2.c1
TILES=0,3,5,10,11,12 timeout -k 10 400 python scripts/tune_conv_x6.py > gpurun_out/tune_g.log 2>&1 &&
SK=0 TILES=0,3,5,10,11,12 timeout -k 10 400 python scripts/tune_conv_x6.py > gpurun_out/tune_g_nosk.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/tune_g.log; cat gpurun_out/tune_g_nosk.log; exit $rc
