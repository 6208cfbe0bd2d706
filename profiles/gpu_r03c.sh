# Packet-timed kernels: parity, bench profiled vs --no-profile, and rocprofv3 stats of the same bench.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03c}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_metrics.py tests/test_gpu_parity.py tests/test_walk.py" "" || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/prof$i.json 2> $O/prof$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/prof$i.json')); print('profiled', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
  timeout -k 10 200 python3 bench.py --steps 32 --no-cpu --no-profile > $O/noprof$i.json 2> $O/noprof$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/noprof$i.json')); print('no-profile', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 32 --no-cpu > $O/rocprof_bench.json 2> $O/rocprof.err || { tail -5 $O/rocprof.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/rocprof_bench.json')); print('under rocprof', d['value'], d['kernel_ms_per_launch'])"
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'tsdf' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
