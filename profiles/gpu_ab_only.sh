# Bench lines only: the default build and every variant in noetic-slam_amd/lib/var/.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/abo}
STEPS=${STEPS:-32} bash profiles/variants.sh $OUT
