# The other bench workloads (not the headline line): pipelined batches, Voxblox semantics, C4.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/modes}
mkdir -p $OUT
timeout -k 10 200 python3 bench.py --no-cpu --pipeline > $OUT/bench_pipeline.json 2> $OUT/p.err || { tail -5 $OUT/p.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu --semantics voxblox > $OUT/bench_voxblox.json 2> $OUT/v.err || { tail -5 $OUT/v.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu --sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304 > $OUT/bench_c4.json 2> $OUT/c.err || { tail -5 $OUT/c.err; exit 1; }
for f in pipeline voxblox c4; do python3 -c "import json; d=json.load(open('$OUT/bench_$f.json')); print('$f', d['value'], d['kernel_ms_per_launch'])"; done
