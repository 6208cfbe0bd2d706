set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03i}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_growth.py tests/test_metrics.py tests/test_host_replay.py" "" || exit 1
bash profiles/gpu_gap.sh $O/gap || exit 1
BATCHES="1 4" bash profiles/gpu_batch_small.sh $O/bs || exit 1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/b64_$i.json 2> $O/b64.err || exit 1
python3 -c "import json; d=json.load(open('$O/b64_$i.json')); print('b64', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
done
