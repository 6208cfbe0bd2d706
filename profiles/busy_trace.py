#!/usr/bin/env python3
"""GPU idle time of a pipelined bench from a rocprofv3 --kernel-trace CSV: over the timed part of
the run (the last 3/4 of the tsdf kernels), the union of all kernel intervals against the wall span,
and the idle gaps before each kernel kind (time in which NO kernel ran).
python3 profiles/busy_trace.py <rocprof out dir> [launches]"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "tsdf" in n:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("::")[-1]))
rows.sort()
rows = rows[len(rows) // 4:]
span = rows[-1][1] - rows[0][0]
busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
idle_before = {}
for s, e, n in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        idle_before.setdefault(n.split("<")[0], []).append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
n_int = sum(1 for r in rows if r[2].startswith("k_integrate"))
print("span %.3f ms, busy %.3f ms, idle %.3f ms (%.1f%%) over %d k_integrate launches" % (
    span / 1e6, busy / 1e6, (span - busy) / 1e6, 100.0 * (span - busy) / span, n_int))
if n_int:
    print("per launch: span %.4f ms, idle %.4f ms" % (span / 1e6 / n_int, (span - busy) / 1e6 / n_int))
for k, v in sorted(idle_before.items(), key=lambda kv: -sum(kv[1])):
    print("  idle before %-22s n %5d  median %7.1f us  total %8.3f ms" % (
        k, len(v), statistics.median(v) / 1e3, sum(v) / 1e6))
