#!/bin/bash
# Round 5: k_count's run lists in j-major slot order (TSDF_CNT_JMAJOR variant build): parity of
# the variant first, then an interleaved A/B against the shipped build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/jm
mkdir -p $O
V=noetic-slam_amd/lib/var/libtsdf_hip_jm.so
TSDF_HIP_LIB=$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_bench_workload.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_jm.log 2>&1 || { tail -30 $O/t_jm.log; exit 1; }
tail -1 $O/t_jm.log
bash profiles/gpu_r05_ab.sh jm 3 real= jm=$V
