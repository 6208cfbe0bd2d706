#!/bin/bash
# Round 5: one-point bundles skip k_mg_merge's look-ahead (batch-wide key table) -- tests, A/B
# against HEAD, kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/call14; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_voxblox_merged.py tests/test_configs.py tests/test_multigpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "merged or Merged or c5_voxblox" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--semantics voxblox --method merged" bash profiles/gpu_r05_ab.sh mgfast 2 real= head=noetic-slam_amd/lib/var/libtsdf_hip_head.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --steps 16 --warmup 2 --semantics voxblox --method merged > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_merged.csv && rm -rf $O/prof
