# Event-cost A/B: bench with per-kernel events (boundary-shared) vs --no-profile, twice each.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03b}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_metrics.py tests/test_gpu_parity.py" "" || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/prof$i.json 2> $O/prof$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/prof$i.json')); print('profiled', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
  timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --no-profile > $O/noprof$i.json 2> $O/noprof$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/noprof$i.json')); print('no-profile', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --pipeline > $O/pipe.json 2> $O/pipe.err || exit 1
python3 -c "import json; d=json.load(open('$O/pipe.json')); print('pipeline', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
