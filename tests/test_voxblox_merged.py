"""Voxblox MergedTsdfIntegrator (tsdf_params.voxblox_method = TSDF_VB_MERGED; SURVEY §8a9,
DESIGN.md §2d): a scan's points are bundled by the voxel they fall in; each bundle casts ONE ray to
its weighted mean point, carrying the summed point weights; clearing points (beyond max_range) are
bundled apart and a clearing bundle keeps its first point only.

Known answers pin the oracle's restatement (oracle/tsdf_oracle.c mg_bundle) against closed forms:
single-point bundles are SimpleTsdfIntegrator's rays; a bundle of k equal-weight points is the
Simple ray to their running mean with k times the weight; a clearing bundle is its first point's
clearing ray; zero-weight points (|z| <= 1e-6 under the 1/z^2 weight) do not enter the mean.  The
GPU tests (marked gpu) hold the HIP pre-pass + walk bit-exact against the oracle."""
import math

import numpy as np
import pytest

import oracle
from conftest import decimate

VS, TAU = 0.05, 0.15
F = np.float32


def ora(**kw):
    kw.setdefault("semantics", "voxblox")
    return oracle.OracleTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def hip(**kw):
    from tsdf_map import HipTSDFVolume
    kw.setdefault("semantics", "voxblox")
    return HipTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def running_mean(d, w):
    """integrateVoxel's merge in float32: m = (m W + d w) / (W + w) per component, W += w."""
    m = np.zeros(3, F)
    mw = F(0)
    for di, wi in zip(d, w):
        wi = F(wi)
        if wi < F(1e-6):
            continue
        nw = F(mw + wi)
        m = ((m * mw + di.astype(F) * wi) / nw).astype(F)
        mw = F(mw + wi)
    return m, mw


def fields(v):
    i, s, w = v.export_voxels()
    return {tuple(k): (a, b) for k, a, b in zip(i.tolist(), s.tolist(), w.tolist())}


O = np.array([0.012, 0.013, 0.011])


def test_single_point_bundles_are_simple_rays():
    """Points in distinct voxels, constant weight: every bundle is one point, (0 + d 1) / 1 = d, so
    the merged field is SimpleTsdfIntegrator's bit for bit."""
    p = (O + np.array([[3.0, 0.4, -0.2], [-2.0, 1.5, 0.3], [0.5, -4.0, 0.8]])).astype(F)
    a = ora(use_const_weight=True, method="merged")
    b = ora(use_const_weight=True)
    a.integrate(p, O)
    b.integrate(p, O)
    for x, y in zip(a.export_voxels(), b.export_voxels()):
        assert np.array_equal(x, y)


def test_bundle_is_the_weighted_mean_ray():
    """Three points in one voxel (constant weight 1, no dropoff): one ray to their running mean,
    weight 3 at every voxel it updates; sdf within fixed-point rounding of the Simple ray's."""
    base = np.array([3.2, 0.41, -0.22])
    p = (O + base + np.array([[0.0, 0.0, 0.0], [0.011, 0.004, 0.0], [0.003, 0.017, -0.02]])).astype(F)
    assert len({tuple(np.floor(q / VS + 1e-6).astype(int)) for q in p}) == 1
    d = p - O.astype(F)
    m, mw = running_mean(d, [1, 1, 1])
    assert mw == 3
    merged_pt = (O.astype(F) + m).astype(F)
    a = ora(use_const_weight=True, use_weight_dropoff=False, method="merged")
    a.integrate(p, O)
    s = ora(use_const_weight=True, use_weight_dropoff=False)
    s.integrate(merged_pt[None], O)
    fa, fs = fields(a), fields(s)
    assert fa.keys() == fs.keys() and len(fa) > 5
    for k in fa:
        assert fa[k][1] == 3.0 and fs[k][1] == 1.0
        assert abs(fa[k][0] - fs[k][0]) <= 1e-6


def test_clearing_bundle_keeps_its_first_point():
    """Two points past max_range in one voxel: the clearing bundle is the FIRST point's clearing
    ray, weight 1 (integrateVoxel breaks after the first kept point of a clearing bundle)."""
    far = (O + np.array([[30.0, 1.0, 0.5], [30.013, 1.004, 0.502]])).astype(F)
    assert len({tuple(np.floor(q / VS + 1e-6).astype(int)) for q in far}) == 1
    a = ora(use_const_weight=True, method="merged", max_range=20.0)
    a.integrate(far, O)
    s = ora(use_const_weight=True, max_range=20.0)
    s.integrate(far[:1], O)
    for x, y in zip(a.export_voxels(), s.export_voxels()):
        assert np.array_equal(x, y)
    assert a.export_voxels()[0].shape[0] > 0


def test_zero_weight_points_leave_the_mean():
    """1/z^2 weight, identity pose: a point at the sensor's height (z = 0) weighs 0 and is skipped
    (kEpsilon); the bundle is the other point's ray with its 1/z^2 weight."""
    q = np.array([0.0, 0.0, 0.0, 1.0])
    p = (O + np.array([[3.2, 0.41, 0.0], [3.21, 0.42, 0.03]])).astype(F)
    assert len({tuple(np.floor(x / VS + 1e-6).astype(int)) for x in p}) == 1
    d = p - O.astype(F)
    w = [0.0, F(1.0) / (abs(d[1, 2]) * abs(d[1, 2]))]
    m, mw = running_mean(d, w)
    a = ora(use_const_weight=False, use_weight_dropoff=False, method="merged")
    a.integrate(p, np.concatenate([O, q]))
    _, _, wa = a.export_voxels()
    assert wa.size > 3 and np.all(wa == mw), (np.unique(wa), mw)


def test_merged_bundles_reduce_rays(sim):
    """On a full C1 scan at 5 cm the bundles are fewer than the points (near-range points share
    voxels: ~2.6% fewer rays); every point is still counted as input."""
    p, org = sim.scan(0)
    a = ora(method="merged", use_const_weight=True)
    a.integrate(p, org)
    n_b = a.stats()["n_rays_total"]
    assert 0.9 * p.shape[0] < n_b < p.shape[0]
    assert a.stats()["n_points_in"] == p.shape[0]


def test_method_validation():
    with pytest.raises(ValueError):
        ora(method="fast")


# -- GPU: the pre-pass (k_mg_count, k_mg_scan, k_mg_scatter, k_mg_group) + the walk, bit for bit --

def assert_bitwise(g, o):
    gi, gs, gw = g.export_voxels()
    oi, os_, ow = o.export_voxels()
    assert gi.shape == oi.shape and np.array_equal(gi, oi)
    assert np.array_equal(gw.view(np.uint32), ow.view(np.uint32))
    bad = np.flatnonzero(gs.view(np.uint32) != os_.view(np.uint32))
    assert bad.size == 0, "sdf differs at %d voxels" % bad.size
    return gi.shape[0]


def _posed(sim, ks, decim):
    out = []
    for j, k in enumerate(ks):
        p, org = sim.scan(k)
        a = 0.3 * j - 0.2
        q = np.array([math.sin(a / 2), 0.0, 0.1 * j, math.cos(a / 2)])
        out.append((decimate(p, decim), np.concatenate([org, q])))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [
    dict(use_const_weight=True),
    dict(use_const_weight=False),
    dict(use_const_weight=False, max_range=20.0),                              # clearing bundles
    dict(use_const_weight=False, space_carving=True, max_range=5.0, min_range=0.1),  # defaults
    dict(use_const_weight=True, max_batch=3, pipeline=2),
], ids=["const", "z2", "clearing", "upstream-defaults", "batched"])
def test_gpu_merged_bitwise(sim, kw):
    k = 16 if kw.get("space_carving") else 2
    scans = _posed(sim, (0, 1, 2, 30, 31), k)
    g, o = hip(method="merged", **kw), ora(method="merged", **{
        a: b for a, b in kw.items() if a not in ("max_batch", "pipeline")})
    for p, q in scans:
        g.integrate(p, q)
        o.integrate(p, q)
    g.sync()
    assert assert_bitwise(g, o) > 1000
    assert g.stats()["n_rays_total"] == o.stats()["n_rays_total"]  # the same bundles


@pytest.mark.gpu
def test_gpu_merged_full_scans_device_batches(sim):
    """Full 128x1024 scans as one 8-scan device batch (the bench's layout)."""
    import torch
    scans = [sim.scan(k) for k in range(8)]
    x = torch.from_numpy(np.concatenate([p for p, _ in scans])).cuda()
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans])
    g = hip(method="merged", max_batch=8)
    g.integrate_batch_device(x.data_ptr(), offs, np.stack([o for _, o in scans]))
    o = ora(method="merged")
    for p, q in scans:
        o.integrate(p, q)
    g.sync()
    assert assert_bitwise(g, o) > 100000


@pytest.mark.gpu
def test_gpu_merged_many_small_scans_one_batch(sim):
    """300 small scans as ONE device batch (the pre-pass's bucket bases off(t) / 1024 + t over
    hundreds of scans, scans of one bucket): decimated scans with a few jittered copies of their
    points (multi-point bundles in every scan), empty scans and one-point scans between them."""
    import torch
    rng = np.random.default_rng(11)
    scans = []
    for k in range(300):
        if k % 37 == 5:
            scans.append((np.zeros((0, 3), F), sim.scan(k % 40)[1]))
            continue
        p, org = sim.scan(k % 40)
        if k % 53 == 7:
            scans.append((p[rng.integers(0, p.shape[0], 1)], org))
            continue
        q = p[rng.integers(0, p.shape[0], 600)]
        dup = q[:40] + rng.uniform(-0.004, 0.004, (40, 3)).astype(F)
        scans.append((np.concatenate([q, dup]).astype(F), org))
    x = torch.from_numpy(np.concatenate([p for p, _ in scans])).cuda()
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans])
    g = hip(method="merged", max_batch=300, use_const_weight=False)
    g.integrate_batch_device(x.data_ptr(), offs, np.stack([o for _, o in scans]))
    o = ora(method="merged", use_const_weight=False)
    for p, q in scans:
        o.integrate(p, q)
    g.sync()
    assert assert_bitwise(g, o) > 10000
    assert g.stats()["n_rays_total"] == o.stats()["n_rays_total"]
    assert o.stats()["n_rays_total"] < offs[-1]  # bundles formed


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [0.5, 0.012], ids=["half-scan", "1500-points"])
def test_gpu_merged_single_voxel_blob_bounded(sim, frac):
    """A degenerate cloud: part of a full scan's points collapsed into ONE voxel 0.4 m from the
    sensor (self-returns / a near-range blob).  The bundle's running weighted mean is sequential
    (bit for bit upstream's integrateVoxel), so it runs on one lane: half a scan is more members
    than k_mg_group's LDS list holds (its bucket takes the forward walk), 1500 points fit it (the
    sorted-list path with one long bundle).  The field stays bit-exact and the scan's integration
    stays bounded (measured against the same scan without the blob)."""
    import time
    p, org = sim.scan(3)
    rng = np.random.default_rng(7)
    n = int(p.shape[0] * frac)
    centre = np.floor((org + np.array([0.4, 0.1, -0.05])) / VS) * VS + VS / 2
    blob = p.copy()
    blob[:n] = (centre + rng.uniform(-0.45 * VS, 0.45 * VS, (n, 3))).astype(F)
    assert len({tuple(np.floor(q / VS).astype(int)) for q in blob[:n:97]}) == 1
    pose = np.concatenate([org, [0.0, 0.0, 0.0, 1.0]])

    def run(cloud, reps=3):
        best = 1e9
        for _ in range(reps):
            g = hip(method="merged", use_const_weight=False)
            g.integrate(cloud, pose)  # warm the context
            g.sync()
            t0 = time.perf_counter()
            g.integrate(cloud, pose)
            g.sync()
            best = min(best, time.perf_counter() - t0)
        return best, g

    t_blob, g = run(blob)
    t_ref, _ = run(p)
    o = ora(method="merged", use_const_weight=False)
    o.integrate(blob, pose)
    o.integrate(blob, pose)
    assert assert_bitwise(g, o) > 1000
    assert g.stats()["n_rays_total"] == o.stats()["n_rays_total"]
    print("blob scan %.2f ms, plain scan %.2f ms (%d points in one voxel)" % (
        1e3 * t_blob, 1e3 * t_ref, n))
    assert t_blob < 0.05 + 4 * t_ref, (t_blob, t_ref)
