#!/bin/bash
# Round 4: pipeline modes 0 / 1 / 2 on the current build (interleaved), and the paired-k_count
# parity test.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-h}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k paired -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_paired.log 2>&1 || { tail -30 $O/pytest_paired.log; exit 1; }
tail -1 $O/pytest_paired.log
for r in 1 2; do
  for p in 2 1 0; do
    timeout -k 10 200 python3 bench.py --no-cpu --pipeline $p > $O/pipe${p}_$r.json 2> $O/pipe${p}_$r.err || { tail -5 $O/pipe${p}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/pipe${p}_$r.json').read().strip().splitlines()[-1]);print('pipeline $p', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'])"
  done
done
