#!/bin/bash
# Round 5 final: the other workloads on HEAD (Voxblox simple / const / merged, fp32, serial, C4,
# 128-scan batches) with in-bench parity, then rank-0 rehearsals of the N-GPU steps (N = 2, 4, 8).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/final/modes
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --steps 32 --cpu-seconds 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], r['kernel'], r['frac'], d.get('parity',{}).get('bitwise'))"
}
run voxblox_simple --semantics voxblox
run voxblox_const --semantics voxblox --const-weight
run voxblox_merged --semantics voxblox --method merged
run fp32 --semantics vdbfusion
run serial_f64 --pipeline 0
run batch128 --batch 128
run c4 --sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304
for N in 2 4 8; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu --rank-rehearsal $N > $O/rehearsal_n$N.json 2> $O/rehearsal_n$N.err || { tail -3 $O/rehearsal_n$N.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/rehearsal_n$N.json')); print('rehearsal', $N, d['value'], d['ms_per_step'])"
done
