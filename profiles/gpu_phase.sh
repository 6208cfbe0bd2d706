# Per-phase cycle counts of k_integrate / k_place (diagnostic PHASE build; printf from a few workgroups).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/phase}
mkdir -p $OUT
TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_PHASE.so timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu > $OUT/phase.out 2> $OUT/phase.err
grep -c phase $OUT/phase.out
