#!/bin/bash
# Round 5, last check on the final tree: smoke() and the driver's default bench command (the
# bench's parity leg and CPU baseline go through the oracle, whose read-outs changed late).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/final_check
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/smoke.log; cat $O/bench.json
exit $rc
