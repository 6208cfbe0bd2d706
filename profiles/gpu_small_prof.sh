# rocprofv3 kernel stats of small-batch benches (one scan / four scans per batch).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/small_prof}
mkdir -p $O
for B in ${BATCHES:-1 4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$B -o run --output-format csv -- python3 bench.py --no-cpu --steps 256 --warmup 8 --batch $B > $O/bench_b$B.json 2> $O/b$B.err || { tail -5 $O/b$B.err; exit 1; }
  f=$(find $O/p$B -name '*kernel_stats.csv')
  cp $f $O/kernel_stats_b$B.csv
  rm -rf $O/p$B
  python3 - $O/kernel_stats_b$B.csv $B <<'PY'
import csv, sys
print('batch', sys.argv[2])
for r in csv.DictReader(open(sys.argv[1])):
    if 'tsdf' in r['Name']:
        print('  ', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done
