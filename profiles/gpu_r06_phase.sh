#!/bin/bash
# Round 6: per-phase clocks of k_count (TSDF_CNT_PHASE) and of k_place / k_integrate (ABLATE=PHASE)
# on this round's code, diagnostic builds, batches one after another, a few steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/phase
mkdir -p $O
TSDF_HIP_LIB=noetic-slam_amd/lib/var/libtsdf_hip_cph.so timeout -k 10 200 python3 bench.py --no-cpu --no-profile --pipeline 0 --steps 4 --warmup 2 > $O/cph.out 2> $O/cph.err || { tail -5 $O/cph.err; exit 1; }
grep -c cntphase $O/cph.out
TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_PHASE.so timeout -k 10 200 python3 bench.py --no-cpu --no-profile --pipeline 0 --steps 4 --warmup 2 > $O/phase.out 2> $O/phase.err || { tail -5 $O/phase.err; exit 1; }
grep -c phase $O/phase.out
