# k_place A/B, bench only: the default build against the variant builds in noetic-slam_amd/lib/var,
# interleaved, $REPS rounds.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03q}
mkdir -p $O
for i in $(seq 1 ${REPS:-2}); do
  for lib in "" noetic-slam_amd/lib/var/*.so; do
    n=real; [ -n "$lib" ] && n=$(basename "$lib" .so | sed 's/^libtsdf_hip_//')
    TSDF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -5 $O/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('$n', d['value'], d['kernel_ms_per_launch'])"
  done
done
