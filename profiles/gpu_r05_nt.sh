#!/bin/bash
# Round 5: non-temporal sample stores (k_place) / loads (k_integrate) as variant builds: parity of
# the combined variant, then an interleaved A/B against the shipped build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/nt
mkdir -p $O
L=noetic-slam_amd/lib/var
TSDF_HIP_LIB=$L/libtsdf_hip_ntboth.so timeout -k 10 300 python3 -u -m pytest tests/test_bench_workload.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_nt.log 2>&1 || { tail -30 $O/t_nt.log; exit 1; }
tail -1 $O/t_nt.log
bash profiles/gpu_r05_ab.sh nt 2 real= ntst=$L/libtsdf_hip_ntst.so ntld=$L/libtsdf_hip_ntld.so ntboth=$L/libtsdf_hip_ntboth.so
