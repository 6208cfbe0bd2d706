#!/bin/bash
# Interleaved A/B of bench.py settings (no CPU leg): bash profiles/gpu_ab_pipe.sh <out> <reps> "<args A>" "<args B>" ...
set -o pipefail
export TMPDIR=/tmp
O=$1; REPS=$2; shift 2
mkdir -p $O
for r in $(seq 1 $REPS); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python3 bench.py --no-cpu $a > $O/v${i}_$r.json 2> $O/v${i}_$r.err || { echo "variant $i failed"; tail -5 $O/v${i}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('$O/v${i}_$r.json').read().strip().splitlines()[-1]);print('v$i', '$a', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
