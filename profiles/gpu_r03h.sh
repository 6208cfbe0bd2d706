set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03h}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_growth.py tests/test_walk.py" "" || exit 1
BATCHES="1 4" bash profiles/gpu_batch_small.sh $O/bs || exit 1
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/b64.json 2> $O/b64.err || exit 1
python3 -c "import json; d=json.load(open('$O/b64.json')); print('b64', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
