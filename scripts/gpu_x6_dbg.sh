set -o pipefail
mkdir -p gpurun_out
export ONLY=l3.c2,l4.c1,l4.c2,l4.c3,l3.c3,d0.c1,l1.c2 TILES=0,3,5
timeout -k 10 300 python scripts/tune_conv_x6.py > gpurun_out/dbg0.log 2>&1 &&
DBG=1 timeout -k 10 300 python scripts/tune_conv_x6.py > gpurun_out/dbg1.log 2>&1 &&
DBG=2 timeout -k 10 300 python scripts/tune_conv_x6.py > gpurun_out/dbg2.log 2>&1
rc=$?; echo "rc=$rc"; for f in 0 1 2; do echo "== DBG $f"; cat gpurun_out/dbg$f.log; done; exit $rc
