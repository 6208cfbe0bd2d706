#!/bin/bash
# Round 6: k_count's run lists in j-major slot order (TSDF_CNT_JMAJOR, r05's rejected patch, which
# now compiles without spills) against the build: interleaved bench lines, then the variant's
# in-bench parity line and its C4 line.
set -o pipefail
export TMPDIR=/tmp
V=noetic-slam_amd/lib/var/libtsdf_hip_jm.so
bash profiles/gpu_r06_ab.sh jm 3 base= jm=$V || exit 1
O=gpurun_out/r06/jm
TSDF_HIP_LIB=$V timeout -k 10 300 python3 bench.py --steps 16 --cpu-seconds 2 --parity-steps 1 > $O/jm_parity.json 2> $O/jm_parity.err || { tail -5 $O/jm_parity.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/jm_parity.json')); print('jm parity', d['value'], (d.get('parity') or {}).get('bitwise'))"
BENCH_ARGS="--sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304" bash profiles/gpu_r06_ab.sh jm_c4 1 base= jm=$V || exit 1
