#!/bin/bash
# Round 4: k_integrate at six waves per SIMD (fewer register-cached samples per window / 32-scan
# windows, so LDS and VGPRs both allow 6 workgroups per CU) against the current build;
# interleaved, in-bench bitwise parity.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-i}
mkdir -p $O
for r in 1 2; do
  for v in base int4w6 int5w6w32 int4w6w32; do
    L=noetic-slam_amd/lib/libtsdf_hip.so; [ $v != base ] && L=noetic-slam_amd/lib/var/libtsdf_hip_$v.so
    TSDF_HIP_LIB=$L timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]);p=d['parity'];print('$v', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
  done
done
