#!/bin/bash
# Round 6: the live index-rule path on one GPU against the contexts' batch size (four quarter-scan
# contexts share the card, so their batches are a quarter of the single context's), then its
# rocprofv3 kernel stats at the default batch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/live_batch
mkdir -p $O
for mb in 32 64 128; do
  for r in index world; do
    timeout -k 10 300 python3 profiles/host_path.py --sectors 4 --sector-rule $r --max-batch $mb > $O/${r}_mb$mb.json 2> $O/${r}_mb$mb.err || { tail -5 $O/${r}_mb$mb.err; exit 1; }
    echo "$r mb$mb $(python3 -c "import json; d=json.load(open('$O/${r}_mb$mb.json')); print(d['value'], d['call_us_per_scan'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 profiles/host_path.py --sectors 4 --sector-rule index > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
find $O/prof -type f ! -name "*stats.csv" -delete
