#!/bin/bash
# profiles/gpu_r04_final.sh, then two k_count ablation builds (results wrong by design, in-bounds):
# CNT_NORET (cell atomics not waited for) and CNT_NOWALK, batches one after another.
set -o pipefail
bash profiles/gpu_r04_final.sh final || exit 1
O=gpurun_out/r04/abl
mkdir -p $O
for v in CNT_NORET CNT_NOWALK; do
  TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_$v.so timeout -k 10 200 python3 bench.py --no-cpu > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], 'serial', d['serial_kernel_ms_per_launch'])"
done
