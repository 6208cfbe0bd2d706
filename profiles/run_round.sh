#!/bin/bash
# Round evidence on one MI355X (run from the repo root on the GPU box):
#   tests: 1. GPU parity tests                                         -> $OUT/pytest_gpu.log
#   perf:  2. PMC counters per kernel (separate --pmc passes, no tracing) -> $OUT/pmc/{summary.txt,traffic.json}
#          3. the bench line, roofline.traffic read from step 2           -> $OUT/bench.json
#          4. rocprofv3 --kernel-trace --stats of the same bench command  -> $OUT/kernel_stats.csv
#          5. the same with --pipeline 0 (every kernel alone: the roofline kernel's duration is the
#             serial leg's)                                              -> $OUT/kernel_stats_serial.csv
#   copy $OUT/traffic.json to profiles/traffic_r0N.json afterwards (bench.py's default; it carries
#   the library's sha, so a later kernel change shows as stale: roofline.traffic_source)
#   bash profiles/run_round.sh <out> [tests|perf|all]
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
OUT=${1:-gpurun_out/round}
WHAT=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$WHAT" != perf ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      --durations=15 > "$OUT/pytest_gpu.log" 2>&1
  tail -1 "$OUT/pytest_gpu.log"
fi
if [ "$WHAT" != tests ]; then
  bash profiles/collect_pmc.sh "$OUT/pmc" > "$OUT/pmc.log" 2>&1
  cp "$OUT/pmc/traffic.json" "$OUT/traffic.json"
  timeout -k 10 300 python3 bench.py --traffic-json "$OUT/traffic.json" > "$OUT/bench.out" 2> "$OUT/bench.err"
  grep '^{' "$OUT/bench.out" > "$OUT/bench.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof" -o bench -- \
      python3 bench.py --no-cpu --traffic-json "$OUT/traffic.json" > "$OUT/rocprof_bench.out" 2>&1
  find "$OUT/rocprof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  rm -rf "$OUT/rocprof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof" -o bench -- \
      python3 bench.py --no-cpu --pipeline 0 --traffic-json "$OUT/traffic.json" > "$OUT/rocprof_serial.out" 2>&1
  find "$OUT/rocprof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_serial.csv" \;
  rm -rf "$OUT/rocprof"
  cat "$OUT/bench.json"
  head -8 "$OUT/kernel_stats.csv"
fi
