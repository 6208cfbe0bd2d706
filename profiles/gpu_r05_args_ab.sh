#!/bin/bash
# Round 5: interleaved A/B of bench.py argument sets on one build.
# Usage: gpu_r05_args_ab.sh <tag> <rounds> "name:--arg --arg" ...   ("name:" = defaults)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/$1; R=$2; shift 2
mkdir -p $O
for i in $(seq 1 $R); do
  for na in "$@"; do
    n=${na%%:*}; a=${na#*:}
    timeout -k 10 200 python3 bench.py --no-cpu --steps 32 $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -3 $O/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('${n}_$i', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
