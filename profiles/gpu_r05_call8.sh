#!/bin/bash
# Round 5: k_place<3>'s weight-store ablation, the modes with rocprof stats, and the GPU idle
# time of the pipelined headline (kernel trace -> profiles/busy_trace.py).
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--semantics voxblox" bash profiles/gpu_r05_ab.sh nosmw 2 real= nosmw=noetic-slam_amd/lib/var/libtsdf_hip_nosmw.so || exit 1
# k_place<1> (constant weight) at two workgroups per CU instead of three (7744 staged samples)
BENCH_ARGS="--semantics voxblox --const-weight" bash profiles/gpu_r05_ab.sh occ2 2 real= occ2=noetic-slam_amd/lib/var/libtsdf_hip_occ2.so || exit 1
bash profiles/gpu_r05_modes.sh modes3 || exit 1
O=gpurun_out/r05/busy; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu --steps 32 --warmup 4 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 profiles/busy_trace.py $O/tr | tee $O/busy.txt
rm -rf $O/tr
