#!/usr/bin/env python3
"""Host-side cost of a batch launch: wall time of K integrate_batch_device calls with no sync
(the enqueue rate) against the time until the GPU has drained them.  One JSON line."""
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
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    import torch
    from tsdf_map import HipTSDFVolume
    from tsdf_map.scan_gen import TorchOusterSim
    dev = torch.device("cuda", 0)
    sim = TorchOusterSim(dev)
    steps = []
    for s in range(a.steps + 8):
        parts, offs, orgs = [], [0], []
        for j in range(a.batch):
            p, o = sim.scan(s * a.batch + j)
            parts.append(p)
            offs.append(offs[-1] + p.shape[0])
            orgs.append(o)
        steps.append((torch.cat(parts).contiguous(), np.array(offs, np.uint64), np.stack(orgs)))
    torch.cuda.synchronize()
    vol = HipTSDFVolume(0.05, 0.15, max_points=1 << 17, max_bricks=1 << 20, max_batch=a.batch,
                        semantics="vdbfusion_f64")
    if a.profile:
        vol.set_profiling(True)
    for i in range(8):
        x, o, g = steps[i]
        vol.integrate_batch_device(x.data_ptr(), o, g)
    vol.sync()
    t0 = time.perf_counter()
    for i in range(8, 8 + a.steps):
        x, o, g = steps[i]
        vol.integrate_batch_device(x.data_ptr(), o, g)
    t1 = time.perf_counter()
    vol.sync()
    t2 = time.perf_counter()
    print(json.dumps({"batch": a.batch, "profile": a.profile,
                      "host_enqueue_us_per_batch": round((t1 - t0) / a.steps * 1e6, 1),
                      "total_us_per_batch": round((t2 - t0) / a.steps * 1e6, 1)}))


if __name__ == "__main__":
    main()
