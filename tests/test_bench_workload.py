"""The driver-timed workload under parity: bench.py's exact settings —
`vdbfusion_f64`, 64 full 128x1024 TorchOusterSim scans per device batch through
tsdf_integrate_batch_device, pipelined batches — must give the CPU oracle's field bit for bit.
bench.py runs the same comparison on its first two timed steps after the timed region and prints
it in its line (`parity`); this test pins it in the GPU suite, for every pipeline mode.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

VS, TAU = 0.05, 0.15


@pytest.fixture(scope="module")
def bench_scans():
    import torch
    from tsdf_map.scan_gen import TorchOusterSim
    sim = TorchOusterSim(torch.device("cuda", 0))
    steps = []
    for s in range(2):  # two 64-scan steps (bench.py's step layout: one tensor + offsets per step)
        parts, offs, orgs = [], [0], []
        for j in range(64):
            p, o = sim.scan(1000 + 64 * s + j)
            parts.append(p)
            offs.append(offs[-1] + p.shape[0])
            orgs.append(o)
        steps.append((torch.cat(parts).contiguous(), np.array(offs, np.uint64), np.stack(orgs)))
    torch.cuda.synchronize()
    ref = {}
    for sem in ("vdbfusion_f64", "vdbfusion"):
        ov = oracle.OracleTSDFVolume(VS, TAU, semantics=sem, threads=8)
        for x, offs, orgs in steps:
            xs = x.cpu().numpy()
            for j in range(len(orgs)):
                ov.integrate(xs[offs[j]:offs[j + 1]], orgs[j])
        ref[sem] = ov.export_voxels()
    return steps, ref


@pytest.mark.parametrize("pipeline", [2, 0])
@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion"])
def test_bench_settings_bitwise(bench_scans, pipeline, semantics):
    from tsdf_map import HipTSDFVolume
    steps, ref = bench_scans
    if semantics == "vdbfusion" and pipeline == 0:
        pytest.skip("covered by the serial cases of test_gpu_parity.py")
    g = HipTSDFVolume(VS, TAU, max_points=1 << 17, max_bricks=1 << 20, max_batch=64,
                      pipeline=pipeline, semantics=semantics)
    for x, offs, orgs in steps:
        g.integrate_batch_device(x.data_ptr(), offs, orgs)
    gi, gs, gw = g.export_voxels()
    oi, os_, ow = ref[semantics]
    assert gi.shape[0] > 5_000_000
    assert gi.shape == oi.shape and np.array_equal(gi, oi)
    assert np.array_equal(gw.view(np.uint32), ow.view(np.uint32))
    bad = np.count_nonzero(gs.view(np.uint32) != os_.view(np.uint32))
    assert bad == 0, "%d sdf mismatches" % bad


@pytest.mark.parametrize("method", ["simple", "merged"])
def test_bench_voxblox_settings_bitwise(method):
    """`bench.py --semantics voxblox [--method merged]` (round 5): 64 full scans with their
    7-element poses (the 1/z^2 weight's sensor axis) as one device batch, pipelined -- the 12-B
    sample records carrying the weights and the Merged pre-pass (hashed bundle ids) at the bench's
    scale, bit for bit against the oracle."""
    import math
    import torch
    from tsdf_map import HipTSDFVolume
    from tsdf_map.scan_gen import TorchOusterSim, pose_on_circle
    sim = TorchOusterSim(torch.device("cuda", 0))
    parts, offs, poses = [], [0], []
    for j in range(64):
        k = 2000 + j
        p, o = sim.scan(k)
        yaw = pose_on_circle(k)[1]
        parts.append(p)
        offs.append(offs[-1] + p.shape[0])
        poses.append(np.concatenate([o, [0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2)]]))
    x = torch.cat(parts).contiguous()
    offs, poses = np.array(offs, np.uint64), np.stack(poses)
    torch.cuda.synchronize()
    g = HipTSDFVolume(VS, TAU, max_points=1 << 17, max_bricks=1 << 20, max_batch=64, pipeline=2,
                      semantics="voxblox", method=method, use_const_weight=False)
    g.integrate_batch_device(x.data_ptr(), offs, poses)
    ov = oracle.OracleTSDFVolume(VS, TAU, semantics="voxblox", method=method,
                                 use_const_weight=False, threads=8)
    xs = x.cpu().numpy()
    for j in range(64):
        ov.integrate(xs[offs[j]:offs[j + 1]], poses[j])
    gi, gs, gw = g.export_voxels()
    oi, os_, ow = ov.export_voxels()
    assert gi.shape[0] > 2_000_000
    assert gi.shape == oi.shape and np.array_equal(gi, oi)
    assert np.array_equal(gw.view(np.uint32), ow.view(np.uint32))
    bad = np.count_nonzero(gs.view(np.uint32) != os_.view(np.uint32))
    assert bad == 0, "%d sdf mismatches" % bad
    assert g.stats()["n_rays_total"] == ov.stats()["n_rays_total"]
