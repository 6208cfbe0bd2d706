#!/bin/bash
# Round 6: host-side time split of the live input path (TSDF_HOST_TIMING): one context, four
# index-rule and four world-rule sector contexts on one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/live_timing
mkdir -p $O
for cfg in "s1:" "index_s4:--sectors 4 --sector-rule index" "world_s4:--sectors 4 --sector-rule world"; do
  n=${cfg%%:*}; a=${cfg#*:}
  TSDF_HOST_TIMING=1 timeout -k 10 300 python3 profiles/host_path.py $a > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(cat $O/$n.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["call_us_per_scan"])')"
  grep "host launch timing" $O/$n.err
done
