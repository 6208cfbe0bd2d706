#!/bin/bash
# Round 6: 128-scan windows (two-word masks) in the 512-scan k_integrate (the build) against 64
# (w64): the 512-scan and sector parity tests, then interleaved rank rehearsals at N = 8 and 4 and
# the headline (unchanged instantiation).
set -o pipefail
export TMPDIR=/tmp
V=noetic-slam_amd/lib/var/libtsdf_hip_w64.so
TESTS="tests/test_walk.py tests/test_multigpu.py tests/test_voxblox_merged.py tests/test_sectors.py" \
  BENCH_ARGS="--rank-rehearsal 8 --steps 16" bash profiles/gpu_r06_ab.sh win128_n8 3 w128= w64=$V || exit 1
BENCH_ARGS="--rank-rehearsal 4 --steps 16" bash profiles/gpu_r06_ab.sh win128_n4 2 w128= w64=$V || exit 1
bash profiles/gpu_r06_ab.sh win128_n1 2 w128= w64=$V || exit 1
