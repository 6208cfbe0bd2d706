#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer boundary: scans/s when every scan arrives
as a host dlio::Point PointCloud2 buffer (32 B/point, x at offset 0; dlio.h:85-106) through
tsdf_integrate — the call tsdf_map_node makes per scan — including the pinned staging copy and the
H2D transfer.  Same synthetic C1/M1 workload as bench.py.  Prints one JSON line.  Not the bench
`value` (that is HBM-resident throughput)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "noetic-slam_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=320)
    ap.add_argument("--warmup", type=int, default=32)
    args = ap.parse_args()
    import torch
    from tsdf_map import HipTSDFVolume
    from tsdf_map.scan_gen import TorchOusterSim

    dev = torch.device("cuda", 0)
    sim = TorchOusterSim(dev)
    clouds, origins = [], []
    for k in range(args.warmup + args.scans):
        pts, org = sim.scan(k)
        xyz = pts.cpu().numpy()
        rec = np.zeros((xyz.shape[0], 8), np.float32)  # dlio::Point: x y z 1 | intensity pad t pad
        rec[:, :3] = xyz
        rec[:, 3] = 1.0
        clouds.append(rec)
        origins.append(np.asarray(org, np.float64))
    vol = HipTSDFVolume(0.05, 0.15, max_points=1 << 17, max_bricks=1 << 20, max_batch=32)

    def run(lo, hi):
        for k in range(lo, hi):
            c = clouds[k]
            vol.integrate_cloud(c, c.shape[0], 32, 0, origins[k])
        vol.sync()

    run(0, args.warmup)
    t0 = time.perf_counter()
    run(args.warmup, args.warmup + args.scans)
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "scans/s, host dlio::Point buffers via tsdf_integrate (PCIe incl.)",
                      "value": round(args.scans / dt, 2), "scans": args.scans,
                      "bytes_per_scan_host": int(clouds[0].nbytes),
                      "h2d_GBps_equiv": round(args.scans * clouds[0].nbytes / dt / 1e9, 2)}))


if __name__ == "__main__":
    main()
