#!/bin/bash
# rocprofv3 kernel stats of one bench configuration (default: the merged pre-pass), into
# gpurun_out/r06/<tag>/; only the *_stats.csv files are kept (the traces exceed gpurun's pull cap).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/$1; shift
ARGS=${@:---semantics voxblox --method merged}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $ARGS --no-cpu --steps 8 --warmup 2 --no-profile > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
find $O/prof -type f ! -name "*stats.csv" -delete
for f in $(find $O/prof -name "*kernel_stats.csv"); do head -14 $f | cut -d, -f1-8; done
