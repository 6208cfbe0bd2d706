#!/bin/bash
# Round 6: k_integrate cells zeroed by the fuse chains (the build) against a zeroing pass per
# window (zpass): parity tests, then interleaved headline / C4 / Voxblox-const A/Bs.
set -o pipefail
export TMPDIR=/tmp
V=noetic-slam_amd/lib/var/libtsdf_hip_zpass.so
TESTS="tests/test_gpu_parity.py tests/test_walk.py tests/test_voxblox.py tests/test_voxblox_merged.py" \
  bash profiles/gpu_r06_ab.sh zero 3 zfuse= zpass=$V || exit 1
BENCH_ARGS="--sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304" \
  bash profiles/gpu_r06_ab.sh zero_c4 2 zfuse= zpass=$V || exit 1
BENCH_ARGS="--semantics voxblox --const-weight" bash profiles/gpu_r06_ab.sh zero_vb 2 zfuse= zpass=$V || exit 1
