set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03j}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_growth.py tests/test_metrics.py tests/test_host_replay.py tests/test_multigpu.py" "" || exit 1
bash profiles/gpu_gap.sh $O/gap || exit 1
TSDF_HOST_TIMING=1 timeout -k 10 200 python3 profiles/host_enqueue.py --batch 1 || exit 1
BATCHES="1 4" bash profiles/gpu_batch_small.sh $O/bs || exit 1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/b64_$i.json 2> $O/b64.err || exit 1
python3 -c "import json; d=json.load(open('$O/b64_$i.json')); print('b64', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
done
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --pipeline > $O/pipe.json 2> $O/pipe.err || exit 1
python3 -c "import json; d=json.load(open('$O/pipe.json')); print('pipe', d['value'], d['ms_per_step'])"
