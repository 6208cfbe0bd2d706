#!/bin/bash
# Round 5: 12-B Voxblox 1/z^2 sample records and the prefetching k_mg_merge -- GPU tests of both,
# then A/B against the round-4 build (old3) for Simple and Merged.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/call9; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_voxblox.py tests/test_voxblox_merged.py tests/test_growth.py tests/test_bench_workload.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--semantics voxblox" bash profiles/gpu_r05_ab.sh vb12 2 real= old3=noetic-slam_amd/lib/var/libtsdf_hip_old3.so || exit 1
BENCH_ARGS="--semantics voxblox --method merged" bash profiles/gpu_r05_ab.sh mg 2 real= old3=noetic-slam_amd/lib/var/libtsdf_hip_old3.so || exit 1
