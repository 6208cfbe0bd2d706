#!/bin/bash
# Round 5: kernel stats of the N = 8 rank-0 rehearsal (serial batches: every kernel alone).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/reh; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --steps 8 --warmup 2 --rank-rehearsal 8 --pipeline 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_n8_serial.csv && rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --steps 8 --warmup 2 --pipeline 0 > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_n1_serial.csv && rm -rf $O/prof
