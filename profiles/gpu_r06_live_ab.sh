#!/bin/bash
# Round 6: same-box A/B of the live input path -- per-scan H2D copies (prehb) against one deferred
# H2D per batch (the real build), interleaved, for one context and four index-rule contexts.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/live_ab
mkdir -p $O
V=noetic-slam_amd/lib/var/libtsdf_hip_prehb.so
for i in 1 2 3; do
  for cfg in "s1:" "index_s4:--sectors 4 --sector-rule index" "world_s4:--sectors 4 --sector-rule world"; do
    n=${cfg%%:*}; a=${cfg#*:}
    for lib in "new:" "prehb:$V"; do
      ln=${lib%%:*}; lp=${lib#*:}
      TSDF_HIP_LIB=$lp timeout -k 10 300 python3 profiles/host_path.py $a > $O/${n}_${ln}_$i.json 2> $O/${n}_${ln}_$i.err || { tail -5 $O/${n}_${ln}_$i.err; exit 1; }
      echo "$i $n $ln $(python3 -c "import json; d=json.load(open('$O/${n}_${ln}_$i.json')); print(d['value'], d['call_us_per_scan'])")"
    done
  done
done
