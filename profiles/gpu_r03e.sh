# Pipelined k_integrate_small: parity, then small-batch A/B (SML_K 4 real vs 2 / 8) and thresholds.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03e}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py" "" || exit 1
for B in 1 4; do
  BENCH_ARGS="--batch $B --steps 256 --warmup 8" STEPS=256 bash profiles/variants.sh $O/var_b$B || exit 1
done
BATCHES="6 8" bash profiles/gpu_batch_small.sh $O/bs || exit 1
