# Other workloads with the round-4 code (bench defaults otherwise: pipeline 2, 64-scan batches).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r04/modes}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu --steps 32 "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], r['kernel'], r['frac'])"
}
run fp32 --semantics vdbfusion
run voxblox --semantics voxblox
run serial_f64 --pipeline 0
run batch128 --batch 128
run c4 --sensor os1_128_2048 --voxel 0.02 --trunc 0.06 --hz 20 --max-bricks 4194304
