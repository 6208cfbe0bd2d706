#!/usr/bin/env python3
"""The ROS node's own per-scan path, measured headless: a DLIO-like topic
stream (100 Hz poses + 10 Hz world-frame dlio::Point clouds of the C1/M1 synthetic sensor) is
written once, then host/tsdf_replay -- MapCore, the object tsdf_map_node runs -- pairs every cloud
with the pose track and integrates it through tsdf_integrate_pose, holding the message instead of
copying it.  The replay reads the stream into memory first and times dispatch + integrate + sync.
Prints one JSON line per max_batch."""
import argparse
import json
import os
import struct
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "noetic-slam_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=256)
    ap.add_argument("--batches", default="8,32")
    ap.add_argument("--semantics", default="vdbfusion_f64")
    ap.add_argument("--path", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "node.topics"))
    args = ap.parse_args()
    from tsdf_map.scan_gen import OusterSim, pose_on_circle
    sim = OusterSim()
    t0 = 1_000_000_000
    with open(args.path, "wb") as f:
        f.write(b"TSDFSTR2")
        for k in range(args.scans + 1):
            for j in range(10):
                t = t0 + (k * 10 + j) * 10_000_000
                p0 = np.asarray(pose_on_circle(k)[0])
                p1 = np.asarray(pose_on_circle(k + 1)[0])
                pos = p0 + (j / 10.0) * (p1 - p0)
                f.write(b"P" + struct.pack("<q3d4d", t, *pos, 0.0, 0.0, 0.0, 1.0))
                if j == 0 and k < args.scans:
                    xyz, _ = sim.scan(k)
                    rec = np.zeros((xyz.shape[0], 8), np.float32)
                    rec[:, :3] = xyz
                    rec[:, 3] = 1.0
                    f.write(b"C" + struct.pack("<qQIIi", t, rec.shape[0], 32, 0, 0) + rec.tobytes())
    exe = os.path.join(REPO, "noetic-slam_amd", "lib", "tsdf_replay")
    for mb in [int(x) for x in args.batches.split(",")]:
        out = subprocess.run([exe, args.path, os.path.join(os.path.dirname(args.path), "n.bricks"),
                              "0.05", "0.15", args.semantics, str(mb)],
                             capture_output=True, text=True, check=True)
        rate = [l for l in out.stdout.splitlines() if "rate" in l][0]
        print(json.dumps({"metric": "scans/s through the node's MapCore (tsdf_replay topic stream)",
                          "value": float(rate.split("rate ")[1].split()[0]), "max_batch": mb,
                          "scans": args.scans, "semantics": args.semantics, "line": rate}),
              flush=True)


if __name__ == "__main__":
    main()
