#!/bin/bash
# Round 4: pipeline 2 with batch b+1's front end released after b's compact (TSDF_PIPE_EARLY=1:
# k_count of b+1 beside k_place and k_integrate of b) against the default; interleaved, in-bench
# bitwise parity; then the pipelined parity test on that mode.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-l}
mkdir -p $O
L=noetic-slam_amd/lib/var/libtsdf_hip_early.so
for r in 1 2; do
  for e in 1 0; do
    TSDF_HIP_LIB=$L TSDF_PIPE_EARLY=$e timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/early${e}_$r.json 2> $O/early${e}_$r.err || { tail -5 $O/early${e}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/early${e}_$r.json').read().strip().splitlines()[-1]);p=d['parity'];print('early=$e', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
  done
done
TSDF_HIP_LIB=$L TSDF_PIPE_EARLY=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "pipelined or batch_composition" -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_early.log 2>&1 || { tail -30 $O/pytest_early.log; exit 1; }
tail -1 $O/pytest_early.log
