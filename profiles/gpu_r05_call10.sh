#!/bin/bash
# Round 5: k_finish folded into k_integrate's last workgroup and the compact scan into
# k_compact_sum's -- parity tests, A/B against the build before (prefold), idle trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/call10; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_growth.py tests/test_bench_workload.py tests/test_voxblox.py tests/test_multigpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash profiles/gpu_r05_ab.sh fold 3 real= prefold=noetic-slam_amd/lib/var/libtsdf_hip_prefold.so || exit 1
B=gpurun_out/r05/busy2; mkdir -p $B
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $B/tr -o run -- python3 bench.py --no-cpu --steps 32 --warmup 4 > $B/bench.json 2> $B/bench.err || { tail -5 $B/bench.err; exit 1; }
python3 profiles/busy_trace.py $B/tr | tee $B/busy.txt
rm -rf $B/tr
