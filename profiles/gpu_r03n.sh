set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03n}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_growth.py tests/test_walk.py tests/test_voxblox.py" "" || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/b_$i.json 2> $O/b.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$i.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], r['kernel'], r['frac'], r['launches_timed'], r['path_frac'], d['path_ms_per_scan'])"
done
timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --pipeline 0 > $O/serial.json 2> $O/s.err || exit 1
python3 -c "import json; d=json.load(open('$O/serial.json')); r=d['roofline']; print('serial', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['path_frac'])"
