# per-launch conv times of the InceptionV3 (8 x 299^2) and VGG16 (32 x 224^2) forwards, and the
# rocprof kernel stats of the family bench
set -o pipefail
mkdir -p gpurun_out/prof_family
export TMPDIR=/tmp
timeout -k 10 300 python scripts/layer_times.py inceptionv3 > gpurun_out/layer_times_inception.txt 2>&1 || exit $?
head -30 gpurun_out/layer_times_inception.txt
timeout -k 10 300 python scripts/layer_times.py vgg16 > gpurun_out/layer_times_vgg16.txt 2>&1 || exit $?
head -12 gpurun_out/layer_times_vgg16.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_family -o family \
  -- python3 scripts/bench_family.py > gpurun_out/prof_family/family.log 2>&1 || exit $?
tail -3 gpurun_out/prof_family/family.log | cut -c1-300
