# Per-scan latency at small batches (a live 10 Hz node): bash profiles/gpu_batch_small.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/batch_small}
mkdir -p $OUT
for B in 1 4 16; do
  timeout -k 10 240 python3 bench.py --no-cpu --steps 256 --warmup 8 --batch $B > $OUT/bench_b$B.out 2>&1 || exit $?
  grep '^{' $OUT/bench_b$B.out > $OUT/bench_b$B.json
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_b$B.json')); print($B, d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
done
