#!/bin/bash
# Round 4: k_count tail reordered (first probes in flight across the block scan, run-start bits set
# while the cell atomics are in flight) against the previous build (lib/var/libtsdf_hip_prev.so),
# interleaved, both semantics; bitwise parity in-bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-g}
mkdir -p $O
for r in 1 2 3; do
  for v in new prev; do
    L=noetic-slam_amd/lib/libtsdf_hip.so; [ $v = prev ] && L=noetic-slam_amd/lib/var/libtsdf_hip_prev.so
    TSDF_HIP_LIB=$L timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]);p=d['parity'];print('$v', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
  done
done
for v in new prev; do
  L=noetic-slam_amd/lib/libtsdf_hip.so; [ $v = prev ] && L=noetic-slam_amd/lib/var/libtsdf_hip_prev.so
  TSDF_HIP_LIB=$L timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 --semantics vdbfusion > $O/fp32_${v}.json 2> $O/fp32_${v}.err || { tail -5 $O/fp32_${v}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/fp32_${v}.json').read().strip().splitlines()[-1]);p=d['parity'];print('fp32 $v', d['value'], d['ms_per_step'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
done
