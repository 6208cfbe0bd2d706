#!/bin/bash
# rocprofv3 kernel stats of the merged bench (the pre-pass kernels' times), into gpurun_out/r06/<tag>/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o merged -- python3 bench.py --semantics voxblox --method merged --no-cpu --steps 8 --warmup 2 --no-profile > $O/merged_prof.json 2> $O/merged_prof.err || { tail -5 $O/merged_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
for f in $(find $O/prof -name "*kernel_stats.csv"); do head -12 $f | cut -d, -f1-8; done
