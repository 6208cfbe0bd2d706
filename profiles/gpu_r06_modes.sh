#!/bin/bash
# Round 6: the other workloads on the current build, one bench line each, into gpurun_out/r06/<tag>/:
# Voxblox merged / simple (1/z^2) / const, the rank rehearsals at N = 2, 4, 8 with both sector rules,
# the border-brick bytes of both rules, the live host path with 4 sector contexts (both rules).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/$1
mkdir -p $O
run() {  # name, timeout, args...
  local nm=$1 tl=$2; shift 2
  timeout -k 10 $tl python3 "$@" > $O/$nm.json 2> $O/$nm.err || { echo "FAILED $nm"; tail -5 $O/$nm.err; exit 1; }
  python3 - "$O/$nm.json" "$nm" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    ln = ln.strip()
    if not ln.startswith("{"): continue
    d = json.loads(ln)
    keys = ("value", "ms_per_step", "serial_kernel_ms_per_launch", "kernel_ms_per_launch")
    print(sys.argv[2], {k: d.get(k) for k in keys if k in d} or d, (d.get("parity") or {}).get("bitwise"))
PY
}
B="bench.py --no-cpu --steps 16"
P="bench.py --steps 16 --cpu-seconds 2 --parity-steps 1"  # with the in-bench parity check
run merged 300 $P --semantics voxblox --method merged
run vb_simple 300 $P --semantics voxblox
run vb_const 300 $P --semantics voxblox --const-weight
for nr in 2 4 8; do
  run reh_index_n$nr 300 $B --rank-rehearsal $nr --sector-rule index
  run reh_world_n$nr 300 $B --rank-rehearsal $nr --sector-rule world
done
run border_bytes 600 profiles/border_bytes.py --scans 128 640 --n 2 4 8
run live_index_s4 300 profiles/host_path.py --sectors 4 --sector-rule index
run live_world_s4 300 profiles/host_path.py --sectors 4 --sector-rule world
run live_s1 300 profiles/host_path.py
# k_integrate / k_place per-phase cycles on this round's code (diagnostic PHASE build)
TSDF_HIP_LIB=noetic-slam_amd/lib/ablate/libtsdf_hip_PHASE.so timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu > $O/phase.out 2> $O/phase.err || { echo "FAILED phase"; tail -3 $O/phase.err; exit 1; }
grep -c phase $O/phase.out
