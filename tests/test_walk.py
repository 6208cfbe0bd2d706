"""The single-walk front end (tsdf_params.walk = TSDF_WALK_SINGLE): k_walk walks every ray ONCE, keeps its
samples in registers, stages them per workgroup and writes them linearly; k_spans lists every
brick's samples as span records for k_integrate.  It must give the two-walk path's field (k_count +
k_place, the default) and the oracle's, bit for bit, and run exactly when asked for and the band's
walk has a proven bound (no carving, no Voxblox clearing rays, <= 4 bricks and <= 32 voxels per
ray)."""
import numpy as np
import pytest

import oracle
from conftest import decimate

pytestmark = pytest.mark.gpu

VS, TAU = 0.05, 0.15


def hip(**kw):
    from tsdf_map import HipTSDFVolume
    return HipTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def ora(**kw):
    for k in ("max_batch", "pipeline", "walk", "max_points"):
        kw.pop(k, None)
    return oracle.OracleTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def fields_equal(a, b):
    ai, as_, aw = a.export_voxels()
    bi, bs, bw = b.export_voxels()
    return (ai.shape == bi.shape and np.array_equal(ai, bi) and np.array_equal(aw, bw)
            and np.array_equal(as_.view(np.uint32), bs.view(np.uint32)))


def front_end(vol, pts, org):
    """Integrate with profiling on; return which front end ran ("walk" or "count")."""
    vol.set_profiling(True)
    vol.integrate(pts, org)
    vol.sync()
    launches = vol.stats()["kernel_launches"]
    assert (launches["walk"] > 0) != (launches["count"] > 0)
    return "walk" if launches["walk"] else "count"


def test_full_c1_scan_single_walk_bitwise(scan0):
    g, t, o = hip(walk="single"), hip(), ora()
    assert front_end(g, *scan0) == "walk"
    assert front_end(t, *scan0) == "count"
    o.integrate(*scan0)
    assert fields_equal(g, o) and fields_equal(g, t)
    sg, st = g.stats(), t.stats()
    for k in ("n_voxels_last", "n_rays_total", "n_pairs_last", "n_active_last", "n_bricks"):
        assert sg[k] == st[k], k


@pytest.mark.parametrize("mb,pipe", [(1, False), (7, True), (64, False), (64, True), (9, 2)])
def test_sequences_both_front_ends(sim, mb, pipe):
    scans = [(decimate(p, 8), o) for p, o in (sim.scan(k) for k in range(70))]
    o = ora()
    g = hip(max_batch=mb, pipeline=pipe, walk="single")
    t = hip(max_batch=mb, pipeline=pipe)
    for p, org in scans:
        o.integrate(p, org)
        g.integrate(p, org)
        t.integrate(p, org)
    assert fields_equal(g, o) and fields_equal(t, o)


@pytest.mark.parametrize("semantics,extra,want", [
    ("vdbfusion", {}, "walk"),
    ("vdbfusion_f64", {}, "walk"),
    ("voxblox", {"use_const_weight": True}, "walk"),  # max_range = inf: no clearing ray can exist
    ("voxblox", {}, "count"),                     # 1/z^2 weights (the default) are per sample
    ("voxblox", {"use_const_weight": True, "max_range": 30.0}, "count"),  # clearing rays to 30 m
    ("voxblox", {"use_const_weight": True, "max_range": 30.0, "allow_clear": False}, "walk"),
    ("vdbfusion", {"space_carving": True, "max_range": 40.0}, "count"),
    ("vdbfusion", {"sdf_trunc": 0.1745}, "walk"),  # band 6.98 voxels: the 32-slot walk
    ("vdbfusion", {"sdf_trunc": 0.2}, "count"),    # band 8 voxels: up to 7 bricks per ray
])
def test_eligibility_and_parity(scan0, semantics, extra, want):
    pts, org = decimate(scan0[0], 2), scan0[1]
    kw = dict(semantics=semantics, **extra)
    g = hip(walk="single", **kw)
    assert front_end(g, pts, org) == want
    o = ora(**kw)
    o.integrate(pts, org)
    assert fields_equal(g, o)
    if want == "walk":
        t = hip(**kw)
        t.integrate(pts, org)
        assert fields_equal(g, t)


def test_c4_geometry_single_walk(sim):
    """C4: OS-1-128 2048-column scans at 2 cm / 6 cm (band 6 voxels, 16 register slots)."""
    from tsdf_map.scan_gen import OusterSim
    s4 = OusterSim(beams="os1_128_2048")
    scans = [s4.scan(k) for k in (0, 3)]
    kw = dict(voxel_size=0.02, sdf_trunc=0.06, max_bricks=1 << 21, max_points=1 << 19)
    g, o = hip(walk="single", **kw), ora(**kw)
    assert front_end(g, *scans[0]) == "walk"
    g.integrate(*scans[1])
    for p, org in scans:
        o.integrate(p, org)
    assert fields_equal(g, o)


@pytest.mark.parametrize("walk", ["single", "two"])
def test_batch_of_512_scans_single_walk(sim, walk):
    """The sector-sharded multi-GPU step is one batch of up to 512 scans (k_integrate<MAXS=512>
    and 513 cells per brick row, the totals cell after the last scan; windows of up to 128 scans
    with two-word masks: decimated scans leave a brick few samples per scan, so its windows reach
    past 64 scans)."""
    import torch
    scans = [(decimate(p, 32), o) for p, o in (sim.scan(k) for k in range(300))]
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    org = np.stack([o for _, o in scans])
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    g = hip(max_batch=512, walk=walk)
    g.set_profiling(True)
    g.integrate_batch_device(d.data_ptr(), offs, org)
    g.sync()
    st = g.stats()
    assert st["n_batches"] == 1 and st["kernel_launches"]["walk" if walk == "single" else "count"] == 1
    o = ora()
    for p, q in scans:
        o.integrate(p, q)
    assert fields_equal(g, o)
