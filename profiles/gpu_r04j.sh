#!/bin/bash
# Round 4: k_count's global phase split into k_resolve (TSDF_CNT_SPLIT variant) against the
# current build, interleaved, in-bench bitwise parity; the GPU parity suite on the variant; then
# the k_count ablations CNT_NORET / CNT_NOWALK (results wrong by design, in-bounds).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-j}
mkdir -p $O
for r in 1 2; do
  for v in base split; do
    L=noetic-slam_amd/lib/libtsdf_hip.so; [ $v != base ] && L=noetic-slam_amd/lib/var/libtsdf_hip_$v.so
    TSDF_HIP_LIB=$L timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]);p=d['parity'];print('$v', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
  done
done
TSDF_HIP_LIB=noetic-slam_amd/lib/var/libtsdf_hip_split.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
for v in CNT_NORET CNT_NOWALK; do
  TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_$v.so timeout -k 10 200 python3 bench.py --no-cpu > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], 'serial', d['serial_kernel_ms_per_launch'])"
done
