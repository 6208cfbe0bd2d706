#!/usr/bin/env python3
"""Border-brick bytes at read-out for the two sector rules.

N sector contexts on one GPU (tsdf_create_sharded with every device id 0: the N ranks' fields are
the same whichever GPU holds them) integrate the bench trajectory (TorchOusterSim, 10 Hz circle,
5 cm / 15 cm, vdbfusion_f64) as resident device batches, then one tsdf_border_reduce_local.  The
reduce moves one 4112-B tile (TSDF_TILE_WORDS u32) per brick held by a non-owner: those are the
read-out bytes a real N-GPU run sends over xGMI.  Printed as one JSON line per (rule, N, scans).

    python3 profiles/border_bytes.py --scans 128 640 --n 2 4 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "noetic-slam_amd"))

TILE_BYTES = 1028 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, nargs="+", default=[128, 640])
    ap.add_argument("--n", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rules", nargs="+", default=["index", "world"])
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    import torch
    from tsdf_map import HipTSDFVolume, border_reduce_local
    from tsdf_map.scan_gen import TorchOusterSim

    dev = torch.device("cuda", 0)
    sim = TorchOusterSim(dev)
    total = max(args.scans)
    steps = []
    for s0 in range(0, total, args.batch):
        parts, offs, org = [], [0], []
        for k in range(s0, min(total, s0 + args.batch)):
            p, o = sim.scan(k)
            parts.append(p)
            offs.append(offs[-1] + p.shape[0])
            org.append(o)
        steps.append((torch.cat(parts).contiguous(), np.array(offs, np.uint64), np.stack(org)))
    torch.cuda.synchronize()
    for n_scans in args.scans:
        for n in args.n:
            for rule in args.rules:
                vols = HipTSDFVolume.sharded(n, 0.05, 0.15, device_ids=[0] * n,
                                             max_points=1 << 17, max_batch=args.batch,
                                             max_bricks=1 << 18, sector_rule=rule)
                done = 0
                for x, offs, org in steps:
                    if done >= n_scans:
                        break
                    for v in vols:
                        v.integrate_batch_device(x.data_ptr(), offs, org)
                    done += len(org)
                for v in vols:
                    v.sync()
                held = [v.num_bricks() for v in vols]
                t0 = time.perf_counter()
                moved = border_reduce_local(vols)
                ms = (time.perf_counter() - t0) * 1e3
                after = [v.num_bricks() for v in vols]
                print(json.dumps({"rule": rule, "n": n, "scans": done, "bricks_held": held,
                                  "bricks_total": int(sum(held)), "border_tiles": int(moved),
                                  "border_bytes": int(moved) * TILE_BYTES,
                                  "border_frac": round(moved / max(1, sum(held)), 4),
                                  "reduce_ms_one_gpu": round(ms, 2), "bricks_after": after}),
                      flush=True)
                for v in vols:
                    v.close()
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
