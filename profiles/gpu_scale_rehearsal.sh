# Rank-0 rehearsals of the N-GPU scaling runs on one GPU (bench.py --rank-rehearsal N), for the
# real build and every variant in noetic-slam_amd/lib/var/.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/scale}
mkdir -p $OUT
shopt -s nullglob
for lib in "" noetic-slam_amd/lib/var/*.so; do
  n=real; [ -n "$lib" ] && n=$(basename "$lib" .so | sed 's/^libtsdf_hip_//')
  for N in 1 2 4 8; do
    TSDF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu --rank-rehearsal $N > $OUT/${n}_n$N.json 2> $OUT/${n}_n$N.err || { echo "$n N=$N failed"; tail -3 $OUT/${n}_n$N.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${n}_n$N.json')); print('$n', $N, d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
