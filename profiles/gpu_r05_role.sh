#!/bin/bash
# Round 5: role streams (front end / back end on their own streams) with HIP stream priorities,
# A/B against the default pipeline 2, two interleaved rounds.  Logs under gpurun_out/r05/<tag>/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-role}
mkdir -p $O
run() {  # name, role, args...
  local n=$1 r=$2; shift 2
  TSDF_ROLE_STREAMS=$r timeout -k 10 200 python3 bench.py --no-cpu --steps 32 "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
}
for i in 1 2; do
  run base_$i 0
  run role1_p2_$i 1
  run role2_p2_$i 2
  run role2_p1_$i 2 --pipeline 1
  run role3_p1_$i 3 --pipeline 1
done
