# Per-scan latency at small batches (a live 10 Hz node): bash profiles/gpu_batch_small.sh <outdir>
# Batches of <= 8 scans run k_integrate_small unless TSDF_SMALL_NS=0 (then k_order + k_integrate).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/batch_small}
mkdir -p $OUT
for B in ${BATCHES:-1 4 8 16}; do
  for S in 8 0; do
    [ $B -gt 8 ] && [ $S = 0 ] && continue
    TSDF_SMALL_NS=$S timeout -k 10 240 python3 bench.py --no-cpu --steps 256 --warmup 8 --batch $B > $OUT/bench_b${B}_s$S.out 2>&1 || exit $?
    grep '^{' $OUT/bench_b${B}_s$S.out > $OUT/bench_b${B}_s$S.json
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_b${B}_s$S.json')); print('batch $B small_ns $S', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
