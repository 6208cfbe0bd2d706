#!/bin/bash
# Bench every A/B build in noetic-slam_amd/lib/var/ (make -C noetic-slam_amd/csrc variants) next to
# the real build; one JSON line per variant into $OUT/<name>.json.
OUT=${1:-gpurun_out/var}
mkdir -p "$OUT"
shopt -s nullglob
for lib in "" noetic-slam_amd/lib/var/*.so; do
  n=real; [ -n "$lib" ] && n=$(basename "$lib" .so | sed 's/^libtsdf_hip_//')
  TSDF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps ${STEPS:-16} --warmup 2 --no-cpu $BENCH_ARGS > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['value'], d['kernel_ms_per_launch'])"
done
