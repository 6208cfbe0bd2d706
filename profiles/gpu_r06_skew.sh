#!/bin/bash
# Round 6: k_integrate z-layer LDS skew A/B (headline + C4) after the parity tests, then the
# Merged bench with parity (key table emptied by k_mg_clear).
set -o pipefail
export TMPDIR=/tmp
V=noetic-slam_amd/lib/var/libtsdf_hip_noskew.so
TESTS="tests/test_gpu_parity.py tests/test_voxblox_merged.py tests/test_walk.py" \
  bash profiles/gpu_r06_ab.sh skew 3 skew= noskew=$V || exit 1
BENCH_ARGS="--sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304" \
  bash profiles/gpu_r06_ab.sh skew_c4 2 skew= noskew=$V || exit 1
O=gpurun_out/r06/skew
timeout -k 10 300 python3 bench.py --method merged --semantics voxblox --cpu-seconds 2 --parity-steps 1 > $O/merged.json 2> $O/merged.err || { tail -5 $O/merged.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/merged.json')); print('merged', d['value'], d['ms_per_step'], (d.get('parity') or {}).get('bitwise'))"
