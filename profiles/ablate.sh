#!/bin/bash
# Timing shares of the batch kernels' phases: the bench (kernel times from HIP events) on the real build
# and on the diagnostic builds of `make -C noetic-slam_amd/csrc ablate`.
set -e
OUT=${1:-gpurun_out/ablate}
mkdir -p "$OUT"
for v in ${VARIANTS:-real PL_NOWALK PL_NOCOPY CNT_NOWALK INT_NOP1 INT_NOP3 INT_NOP4}; do
  lib=""
  [ "$v" != real ] && lib="noetic-slam_amd/lib/ablate/libtsdf_hip_$v.so"
  TSDF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps ${STEPS:-16} --warmup 2 --no-cpu > "$OUT/$v.json"
  python3 -c "import json,sys; d=json.load(open('$OUT/$v.json')); print('$v', d['value'], d['kernel_ms_per_launch'])"
done
