#!/bin/bash
# profiles/gpu_r04_final.sh (final evidence on HEAD), then one interleaved pair of the k_resolve
# variant against the build (in-bench bitwise parity) and the CNT_NORET ablation.
set -o pipefail
bash profiles/gpu_r04_final.sh final || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/j
mkdir -p $O
for v in split base; do
  L=noetic-slam_amd/lib/libtsdf_hip.so; [ $v != base ] && L=noetic-slam_amd/lib/var/libtsdf_hip_$v.so
  TSDF_HIP_LIB=$L timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/${v}_1.json 2> $O/${v}_1.err || { tail -5 $O/${v}_1.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${v}_1.json').read().strip().splitlines()[-1]);p=d['parity'];print('$v', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
done
v=CNT_NORET
TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_$v.so timeout -k 10 200 python3 bench.py --no-cpu > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], 'serial', d['serial_kernel_ms_per_launch'])"
