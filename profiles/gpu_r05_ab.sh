#!/bin/bash
# Round 5: interleaved A/B of library builds.  Usage: gpu_r05_ab.sh <tag> <rounds> name=lib ...
# (lib "" = the real build).  One bench line per (round, name) into gpurun_out/r05/<tag>/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/$1; R=$2; shift 2
mkdir -p $O
for i in $(seq 1 $R); do
  for nl in "$@"; do
    n=${nl%%=*}; lib=${nl#*=}
    TSDF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 32 $BENCH_ARGS > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -3 $O/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('${n}_$i', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
