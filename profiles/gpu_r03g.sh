# Wide k_count for tiny batches: parity, then small batches with TSDF_COUNT_WIDE default vs 0.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03g}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_literal.py tests/test_voxblox.py" "" || exit 1
for B in 1 2 4; do
  for W in 256 0; do
    TSDF_COUNT_WIDE=$W timeout -k 10 240 python3 bench.py --no-cpu --steps 256 --warmup 8 --batch $B > $O/b${B}_w$W.json 2> $O/b${B}_w$W.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b${B}_w$W.json')); print('batch $B wide $W', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
