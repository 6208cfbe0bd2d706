# Round-3 iteration: small-batch + merged-order parity, A/B of the order merge, event cost,
# small batches and the live paths.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03a}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py -k small --durations=5" "" || exit 1
bash profiles/gpu_iter.sh $O/t2 "tests/test_gpu_parity.py tests/test_multigpu.py tests/test_walk.py tests/test_growth.py" "" || exit 1
bash profiles/variants.sh $O/var || exit 1
STEPS=32 bash profiles/variants.sh $O/var2 || exit 1
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --no-profile > $O/noprof.json 2> $O/noprof.err || exit 1
python3 -c "import json; d=json.load(open('$O/noprof.json')); print('no-profile', d['value'], d['ms_per_step'])"
bash profiles/gpu_batch_small.sh $O/bs || exit 1
bash profiles/gpu_live.sh $O/live || exit 1
