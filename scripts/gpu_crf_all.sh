set -o pipefail
bash scripts/gpu_crf.sh && bash scripts/gpu_crf_prof.sh
