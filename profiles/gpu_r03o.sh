set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03o}
mkdir -p $O
for i in 1 2; do
  for g in 1.0 0.75 0.5 0.35; do
    TSDF_INT_GRID_SCALE=$g timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/g${g}_$i.json 2> $O/g.err || exit 1
    python3 -c "import json; d=json.load(open('$O/g${g}_$i.json')); print('scale $g', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
