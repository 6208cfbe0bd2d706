set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m8
for N in 1 2 4 8; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu --rank-rehearsal $N --pipeline > gpurun_out/m8/pipe_n$N.json 2> gpurun_out/m8/pipe_n$N.err || { tail -3 gpurun_out/m8/pipe_n$N.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/m8/pipe_n$N.json')); print('pipeline', $N, d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
done
