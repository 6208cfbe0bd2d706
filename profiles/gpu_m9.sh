set -o pipefail
bash profiles/gpu_tests.sh gpurun_out/m9 || exit 1
bash profiles/gpu_scale_rehearsal.sh gpurun_out/m9
