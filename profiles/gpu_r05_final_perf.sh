#!/bin/bash
# Round 5 final evidence on HEAD (one call): PMC traffic per kernel, the bench line with it,
# rocprofv3 stats of the pipelined and serial bench, and the per-unit PMC pass that names the bound.
# Outputs under gpurun_out/r05/final/ (copied to profiles/r05/final/ afterwards).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/final
mkdir -p $O
bash profiles/run_round.sh $O perf || { echo "run_round perf failed"; exit 1; }
bash profiles/collect_pmc_units.sh $O/units > $O/units.log 2>&1 || { tail -5 $O/units.log; exit 1; }
tail -40 $O/units/units.txt
