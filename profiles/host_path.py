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
    ap.add_argument("--sectors", type=int, default=0,
                    help="N > 1: the live N-GPU input path rehearsed on one GPU -- N sector contexts "
                         "fed by tsdf_integrate_sectors (--sector-input: fanout = one H2D and "
                         "device copies, h2d = one H2D per context, split = host classification)")
    ap.add_argument("--sector-input", default="fanout", choices=("fanout", "h2d", "split"),
                    help="tsdf_params.sector_input of the N contexts (ABI v8; world rule only)")
    ap.add_argument("--sector-rule", default="index", choices=("index", "world"),
                    help="tsdf_params.sector_rule (ABI v10): index = each context packs and copies "
                         "only its contiguous 1/N of the cloud")
    ap.add_argument("--semantics", default="vdbfusion_f64")
    ap.add_argument("--max-batch", type=int, default=32)
    args = ap.parse_args()
    import ctypes as C

    import torch
    from tsdf_map import HipTSDFVolume, _abi
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
    n = max(1, args.sectors)
    vols = [HipTSDFVolume(0.05, 0.15, max_points=1 << 17, max_bricks=1 << 20,
                          max_batch=args.max_batch, semantics=args.semantics,
                          n_sectors=n if n > 1 else 0, sector=k,
                          sector_input=args.sector_input, sector_rule=args.sector_rule)
            for k in range(n)]
    vol = vols[0]
    lib = vol._lib
    ctxs = (C.c_void_p * n)(*[v._ctx.value for v in vols])
    poses = [np.concatenate([o, [0.0, 0.0, 0.0, 1.0]]) for o in origins]

    in_call = [0.0]

    def run(lo, hi):
        for k in range(lo, hi):
            c = clouds[k]
            t = time.perf_counter()
            if n > 1:  # one host cloud for the sector contexts
                rc = lib.tsdf_integrate_sectors(ctxs, n, c.ctypes.data_as(C.c_void_p), c.shape[0], 32,
                                                0, 0, poses[k].ctypes.data_as(_abi.D3))
                vol._check(rc, "integrate_sectors")
            else:
                vol.integrate_cloud(c, c.shape[0], 32, 0, origins[k])
            in_call[0] += time.perf_counter() - t
        for v in vols:
            v.sync()

    run(0, args.warmup)
    in_call[0] = 0.0
    t0 = time.perf_counter()
    run(args.warmup, args.warmup + args.scans)
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "scans/s, host dlio::Point buffers via %s (PCIe incl.)" %
                                ("tsdf_integrate_sectors over %d contexts on ONE GPU" % n if n > 1
                                 else "tsdf_integrate"),
                      "value": round(args.scans / dt, 2), "scans": args.scans, "sectors": n,
                      "sector_input": args.sector_input if n > 1 else None,
                      "sector_rule": args.sector_rule if n > 1 else None,
                      "semantics": args.semantics, "max_batch": args.max_batch,
                      "bytes_per_scan_host": int(clouds[0].nbytes),
                      "h2d_bytes_per_scan": int(clouds[0].shape[0] * 12),
                      "h2d_GBps_equiv": round(args.scans * clouds[0].nbytes / dt / 1e9, 2),
                      # time inside the integrate calls (packing, copies, API calls, and any wait
                      # for a staging buffer still in use on the GPU)
                      "call_us_per_scan": round(in_call[0] / args.scans * 1e6, 1)}))


if __name__ == "__main__":
    main()
