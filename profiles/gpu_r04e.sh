#!/bin/bash
# Round 4: per-phase wall clocks of k_count (TSDF_CNT_PHASE), k_place and k_integrate (ABLATE=PHASE)
# in diagnostic builds, batches one after another (--pipeline 0), a few steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-e}
mkdir -p $O
TSDF_HIP_LIB=noetic-slam_amd/lib/var/libtsdf_hip_cph.so timeout -k 10 200 python3 bench.py --no-cpu --no-profile --pipeline 0 --steps 4 --warmup 2 > $O/cph.out 2> $O/cph.err || { tail -5 $O/cph.err; exit 1; }
grep -c cntphase $O/cph.out
TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_PHASE.so timeout -k 10 200 python3 bench.py --no-cpu --no-profile --pipeline 0 --steps 4 --warmup 2 > $O/phase.out 2> $O/phase.err || { tail -5 $O/phase.err; exit 1; }
grep -c phase $O/phase.out
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu > $O/base_$r.json 2> $O/base_$r.err || { tail -5 $O/base_$r.err; exit 1; }
  for v in key32 emit4; do
    TSDF_HIP_LIB=noetic-slam_amd/lib/var/libtsdf_hip_$v.so timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
  done
  for f in base key32 emit4; do
    python3 -c "import json;d=json.loads(open('$O/${f}_$r.json').read().strip().splitlines()[-1]);p=d['parity'];print('$f', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
  done
done
