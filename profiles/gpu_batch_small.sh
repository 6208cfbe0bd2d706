# Per-scan latency at small batches (a live 10 Hz node): bash profiles/gpu_batch_small.sh <outdir>
# Defaults (k_integrate_small up to 6 scans, 1024-lane k_count up to 256 blocks) against the
# large-batch kernels (TSDF_SMALL_NS=0 TSDF_COUNT_WIDE=0).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/batch_small}
mkdir -p $OUT
for B in ${BATCHES:-1 2 4 6 8 16}; do
  for M in default large; do
    if [ $M = large ]; then E="TSDF_SMALL_NS=0 TSDF_COUNT_WIDE=0"; else E="${SMALL_ENV:-}"; fi
    env $E timeout -k 10 240 python3 bench.py --no-cpu --steps 256 --warmup 8 --batch $B > $OUT/bench_b${B}_$M.json 2> $OUT/bench_b${B}_$M.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_b${B}_$M.json')); print('batch $B $M', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
