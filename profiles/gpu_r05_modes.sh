#!/bin/bash
# Round 5: Voxblox workloads (1/z^2 simple = voxblox's default weight, const weight, merged) with
# parity, rocprof kernel stats of simple and merged, and the A/B of the sem-3 capacity knobs
# .  Logs under gpurun_out/r05/<tag>/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-modes}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --steps 32 --cpu-seconds 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], r['kernel'], r['frac'], d.get('parity',{}).get('bitwise'))"
}
run voxblox_simple --semantics voxblox
run voxblox_const --semantics voxblox --const-weight
run voxblox_merged --semantics voxblox --method merged
run headline
for m in simple merged; do
  a="--semantics voxblox"; [ $m = merged ] && a="$a --method merged"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --no-cpu --steps 16 --warmup 2 $a > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_$m.csv && rm -rf $O/prof_$m
done
