# HIP API time per 1-scan batch on the host (rocprofv3 --hip-trace --stats; no counters).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/hostapi}
mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 profiles/host_enqueue.py --batch 1 --steps 512 > $O/enq.json 2> $O/enq.err || { tail -5 $O/enq.err; exit 1; }
cat $O/enq.json
f=$(find $O/tr -name '*hip_api_stats.csv')
cp $f $O/hip_api_stats.csv
rm -rf $O/tr
python3 - $O/hip_api_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:15]:
    print("%-36s calls %7s  avg %8.2f us  total %9.1f ms" % (r["Name"][:36], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
