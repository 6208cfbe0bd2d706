# Every rank of an N-GPU step rehearsed on one GPU (bench.py --rank-rehearsal N
# --rehearsal-sector K): the real step is the slowest rank's.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/sector_balance}
N=${N:-8}
mkdir -p $O
for K in $(seq 0 $((N - 1))); do
  timeout -k 10 300 python3 bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu --rank-rehearsal $N --rehearsal-sector $K > $O/n${N}_k$K.json 2> $O/k$K.err || { tail -3 $O/k$K.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/n${N}_k$K.json')); print('N $N rank $K', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
done
