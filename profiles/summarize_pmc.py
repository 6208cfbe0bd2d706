"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch for the tsdf kernels.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE under-reports wide coalesced reads by 2x
(MI355X_MICROARCH.md, HBM) — both the raw value and the x2-corrected read bytes are printed; the
correction is exact only for 16-B/lane streaming reads, so it is an upper bound for this mix.
"""
import collections
import csv
import glob
import json
import os
import sys


def main(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if "tsdf::" not in k:
                    continue
                name = k.split("tsdf::")[1].split("(")[0].split("<")[0]
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for kname in sorted(vals):
        out[kname] = {c: sum(v) / len(v) for c, v in sorted(vals[kname].items())}
        print(kname)
        for c, v in sorted(out[kname].items()):
            print("  %-24s %16.1f  (n=%d)" % (c, v, len(vals[kname][c])))
        d = out[kname]
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            print("  HBM bytes/launch: read %.1f MB (x2 corr %.1f MB), write %.1f MB" %
                  (d["FETCH_SIZE"] * 1024 / 1e6, 2 * d["FETCH_SIZE"] * 1024 / 1e6,
                   d["WRITE_SIZE"] * 1024 / 1e6))
    with open(os.path.join(root, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    # roofline.traffic for bench.py: HBM-side bytes per launch = 2 x FETCH_SIZE (the gfx950
    # correction of MI355X_MICROARCH.md, exact for 16-B/lane streaming reads) + WRITE_SIZE, KiB -> B
    traffic = {"bytes_per_launch": {}, "fetch_bytes_raw": {}, "write_bytes": {},
               "note": "per dispatch means of rocprofv3 --pmc passes (profiles/collect_pmc.sh); "
                       "bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE "
                       "correction per MI355X_MICROARCH.md, calibrated on this box's counters "
                       "for 4/8/12/16-B contiguous reads (exact) and random 4-B gathers (128 B, "
                       "one L2 line, per gather): profiles/r03/calib/calib.json)"}
    # the build the counters were measured on: bench.py reports roofline.traffic only when this
    # matches the library it loaded (a kernel change makes the file stale visibly, not silently)
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "noetic-slam_amd", "lib", "libtsdf_hip.so")
    lib = os.environ.get("TSDF_HIP_LIB") or lib
    with open(lib, "rb") as fh:
        traffic["lib_sha16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
    for kname, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d and not kname.startswith("k_fill"):
            f, w = d["FETCH_SIZE"] * 1024.0, d["WRITE_SIZE"] * 1024.0
            traffic["bytes_per_launch"][kname] = round(2 * f + w)
            traffic["fetch_bytes_raw"][kname] = round(f)
            traffic["write_bytes"][kname] = round(w)
    with open(os.path.join(root, "traffic.json"), "w") as fh:
        json.dump(traffic, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
