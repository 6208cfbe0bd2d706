set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03m}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_growth.py tests/test_walk.py" "" || exit 1
for i in 1 2; do
  for P in 0 1 2; do
    timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --pipeline $P > $O/p${P}_$i.json 2> $O/p$P.err || exit 1
    python3 -c "import json; d=json.load(open('$O/p${P}_$i.json')); print('pipeline $P', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
done
