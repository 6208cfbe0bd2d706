#!/bin/bash
# Round 6, final build: the other workloads, one bench line each (in-bench parity where the oracle
# is quick enough), into gpurun_out/r06/final_modes/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/final_modes
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
    keys = ("value", "ms_per_step", "serial_kernel_ms_per_launch")
    print(sys.argv[2], {k: d.get(k) for k in keys if k in d} or d, (d.get("parity") or {}).get("bitwise"))
PY
}
B="bench.py --no-cpu --steps 16"
P="bench.py --steps 16 --cpu-seconds 2 --parity-steps 1"
run merged 300 $P --semantics voxblox --method merged
run vb_simple 300 $P --semantics voxblox
run vb_const 300 $P --semantics voxblox --const-weight
run c4 300 $P --sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304
for nr in 2 4 8; do
  run reh_index_n$nr 300 $B --rank-rehearsal $nr --sector-rule index
done
run reh_world_n8 300 $B --rank-rehearsal 8 --sector-rule world
run live_index_s4 300 profiles/host_path.py --sectors 4 --sector-rule index
run live_world_s4 300 profiles/host_path.py --sectors 4 --sector-rule world
run live_s1 300 profiles/host_path.py
