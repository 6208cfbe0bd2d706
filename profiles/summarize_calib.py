#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration summary (profiles/tools/fetch_calib.hip, profiles/gpu_calib.sh):
per calibration kernel, the counter (KiB) x 1024 / the bytes the kernel moves.  Prints JSON.
    python3 profiles/summarize_calib.py gpurun_out/calib > profiles/r03/calib/calib.json"""
import collections
import csv
import json
import os
import sys


def main(d):
    known = json.load(open(os.path.join(d, "bytes.json")))["bytes"]
    out = {"bytes": known, "ratio": {}}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(os.path.join(d, c, "pmc_counter_collection.csv"))):
            agg[r["Kernel_Name"].split("(")[0].replace("void ", "")] += float(r["Counter_Value"])
        for k, v in agg.items():
            key = "gather4_lines" if k == "gather4" else k
            if key in known:
                out["ratio"].setdefault(k, {})[c] = round(v * 1024 / known[key], 4)
    out["reading"] = (
        "contiguous reads of 4/8/12/16 B per lane: FETCH_SIZE x 1024 = 0.5 x bytes (the x2 correction "
        "holds for every width); random 4-B gathers, one per 64-B line: FETCH_SIZE x 1024 = 64 B per "
        "gather, i.e. 128 B (one L2 line) after the x2 correction; writes of 4/8/16 B per lane and "
        "8-B records in scattered runs of 12: WRITE_SIZE x 1024 = 1.0 x bytes")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib")
