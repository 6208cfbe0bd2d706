#!/usr/bin/env python3
"""Per-batch GPU timeline of a small-batch bench from rocprofv3 --kernel-trace --memory-copy-trace
CSVs: median duration of every tsdf kernel and of the idle gap before it (the previous command's
end to its start), over the timed batches.  python3 profiles/gap_trace.py <rocprof out dir>"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]
                     .replace("void ", "")))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
rows.sort()
# keep the last 3/4 (timed steps; warmup and setup first)
rows = [r for r in rows if "tsdf" in r[2] or r[2].startswith("copy")]
rows = rows[len(rows) // 4:]
dur, gap = {}, {}
prev_end = None
for s, e, n in rows:
    dur.setdefault(n, []).append(e - s)
    if prev_end is not None:
        gap.setdefault(n, []).append(s - prev_end)
    prev_end = max(prev_end or 0, e)
for n in dur:
    print("%-40s n=%5d  dur %8.1f us  gap-before %8.1f us" % (
        n[:40], len(dur[n]), statistics.median(dur[n]) / 1e3,
        statistics.median(gap.get(n, [0])) / 1e3))
