"""Voxblox-semantics mode (TSDF_SEM_VOXBLOX).

The reference names Voxblox as backend idx 2 (README.md:44-50) but ships none of its code, so the
oracle's restatement (oracle/tsdf_oracle.c walk_ray_vb: SimpleTsdfIntegrator + RayCaster +
updateTsdfVoxel with a constant weight) is pinned here by closed-form known answers: an axis ray's
voxel list, projective distances and dropoff weights, the clamp and max_weight rules of the fuse,
clearing rays, the carving walk's step count.  Against the literal per-sample Voxblox update (the
oracle's SEQUENTIAL mode) the scan-fused field is REPORTED with a tolerance (0.1 tau),
not gated bitwise: the clamps make Voxblox order dependent.

The GPU tests (marked gpu) hold the HIP path bit-exact against the oracle's scan-fused mode, like
the VDBFusion mode in test_gpu_parity.py.
"""
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


def dropoff(sdf, vs=VS, tau=TAU):
    return max(0.0, (tau + sdf) / (tau - vs)) if sdf < -vs else 1.0


# -- oracle known answers -------------------------------------------------------------------------

@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_axis_ray_projective_sdf_and_dropoff(sign):
    """A ray along +-x: voxels floor((p -+ tau)/vs + 1e-6) along x, projective sdf = d - (c - o).u,
    weight 1 down to -vs, then (tau + sdf)/(tau - vs), weightless voxels dropped."""
    o = np.array([0.012, 0.013, 0.011])
    p = (o + [sign * 5.0, 0.0, 0.0]).astype(F)
    ijk, s = ora().ray_voxels(p, o)
    j, k = math.floor(o[1] / VS), math.floor(o[2] / VS)
    a, b = math.floor((p[0] - TAU) / VS + 1e-6), math.floor((p[0] + TAU) / VS + 1e-6)
    xs = range(a, b + 1) if sign > 0 else range(b, a - 1, -1)
    exp = []
    for i in xs:
        sdf = 5.0 - sign * ((i + 0.5) * VS - o[0])
        if dropoff(sdf) >= 2.0 ** -16:
            exp.append(((i, j, k), sdf))
    assert [tuple(x) for x in ijk.tolist()] == [e[0] for e in exp]
    np.testing.assert_allclose(s, [e[1] for e in exp], atol=2e-6)
    assert min(s) < -VS  # the band reaches the dropoff zone


def test_fuse_clamps_distance_and_caps_weight():
    """updateTsdfVoxel: S' = (s w + S W)/(W + w) clamped to +-tau, W = min(max_weight, W + w);
    one scan per integrate, so the scan-fused and sequential modes agree exactly here."""
    o = np.array([0.012, 0.013, 0.011])
    p = (o + [5.0, 0.0, 0.0]).astype(F)
    for mode in (oracle.MODE_SCAN_FUSED, oracle.MODE_SEQUENTIAL):
        v = ora(max_weight=2.5, mode=mode)
        ijk, s = v.ray_voxels(p, o)
        S = {tuple(x): F(0.0) for x in ijk.tolist()}
        W = {tuple(x): F(0.0) for x in ijk.tolist()}
        for _ in range(4):
            v.integrate(p[None], o)
            for x, sd in zip(ijk.tolist(), s):
                x = tuple(x)
                w = F(dropoff(float(sd)))
                nw = F(W[x] + w)
                ns = F(F(F(sd) * w + S[x] * W[x]) / nw)
                S[x] = F(min(TAU, ns)) if ns > 0 else F(max(-TAU, ns))
                W[x] = F(min(F(2.5), nw))
        gi, gs, gw = v.export_voxels()
        for x, sd, w in zip(gi.tolist(), gs, gw):
            assert gw.max() == F(2.5)
            np.testing.assert_allclose(sd, S[tuple(x)], atol=1e-6)
            # scan-fused: w passes through trunc(w 2^32) fixed point first
            np.testing.assert_allclose(w, W[tuple(x)], rtol=1e-6)


def test_clearing_rays():
    """A return beyond max_range is a clearing ray when allow_clear (length min(d - tau,
    max_range); without carving one voxel at its end, whose far-positive sdf clamps to tau), and is
    dropped otherwise."""
    o = np.array([0.012, 0.013, 0.011])
    p = (o + [0.0, 5.0, 0.0]).astype(F)
    v = ora(max_range=3.0)
    ijk, s = v.ray_voxels(p, o)
    assert ijk.tolist() == [[0, math.floor((o[1] + 3.0) / VS + 1e-6), 0]]
    np.testing.assert_allclose(s, [5.0 - ((ijk[0, 1] + 0.5) * VS - o[1])], atol=2e-6)
    v.integrate(p[None], o)
    _, gs, gw = v.export_voxels()
    assert gs.tolist() == [F(TAU)] and gw.tolist() == [1.0]
    assert ora(max_range=3.0, allow_clear=False).ray_voxels(p, o) is None


def test_carving_walk_is_a_6_connected_path_of_l1_length():
    """voxel_carving_enabled: the walk starts at the origin's voxel and takes exactly
    |floor(end) - floor(start)|_1 unit steps, each along one axis in the ray's direction."""
    rng = np.random.default_rng(3)
    o = np.array([0.31, -0.27, 1.13])
    v = ora(space_carving=True, max_range=60.0)
    for _ in range(50):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        p = (o + d * rng.uniform(1.0, 40.0)).astype(F)
        u = (p - o) / np.linalg.norm(p - o)
        ijk, s = v.ray_voxels(p, o)
        start = np.floor(o / VS + 1e-6).astype(int)
        end = np.floor((p + u * TAU) / VS + 1e-6).astype(int)
        steps = np.abs(np.diff(ijk, axis=0))
        assert (steps.sum(1) == 1).all()
        assert (np.sign(np.diff(ijk, axis=0)) * np.sign(u) >= 0).all()
        # weightless tail voxels (sdf < -tau) are dropped, so the walk may end early
        assert tuple(ijk[0]) == tuple(start)
        assert len(ijk) <= np.abs(end - start).sum() + 1
        assert np.abs(np.abs(end - start).sum() + 1 - len(ijk)) <= 2
        np.testing.assert_allclose(s[0], np.linalg.norm(p - o) - np.dot((start + 0.5) * VS - o, u),
                                   atol=1e-4)


def test_background_and_weight_gate():
    v = ora()
    s, w = v.query_dense([0, 0, 0], [2, 2, 2])
    assert (s == 0).all() and (w == 0).all()  # voxblox TsdfVoxel: distance 0, weight 0
    with pytest.raises(Exception):
        ora(max_weight=0.0)


def test_sequential_vs_scan_fused_reported(sim):
    """The literal per-sample Voxblox update against the scan-fused restatement on C1 scans
    (no carving): W agrees to float rounding, |dS| <= 0.1 tau for >= 99.9% of voxels (SURVEY §8c;
    reported, not a bitwise bar: the per-sample clamps make Voxblox order dependent)."""
    scans = [(decimate(p, 8), org) for p, org in (sim.scan(k) for k in (0, 1, 2))]
    a, b = ora(), ora(mode=oracle.MODE_SEQUENTIAL)
    for p, org in scans:
        a.integrate(p, org)
        b.integrate(p, org)
    ai, as_, aw = a.export_voxels()
    bi, bs, bw = b.export_voxels()
    assert np.array_equal(ai, bi)
    np.testing.assert_allclose(aw, bw, rtol=1e-5, atol=1e-6)
    d = np.abs(as_ - bs)
    print("voxblox scan-fused vs sequential: %d voxels, max %.3g mean %.3g p99.9 %.3g m"
          % (d.size, d.max(), d.mean(), np.quantile(d, 0.999)))
    assert np.quantile(d, 0.999) <= 0.1 * TAU


def test_default_params():
    """ABI v8 defaults: VDBFusion at upstream's precisions (the conforming mode), Voxblox's
    config defaults (1/z^2 weight, dropoff, clearing, max_weight 1e4); the Python facade agrees."""
    from tsdf_map import _abi
    from tsdf_map.volume import TSDFVolume
    lib = oracle.load()
    p = _abi.default_params(lib)
    assert p.semantics == _abi.SEM_VDBFUSION_F64 and p.allow_clear == 1 and p.use_weight_dropoff == 1
    assert p.max_weight == 10000.0 and p.depth_weight == 1
    q = TSDFVolume.make_params(lib, 0.05, 0.15)
    for f in ("semantics", "allow_clear", "use_weight_dropoff", "max_weight", "depth_weight",
              "pipeline", "space_carving"):
        assert getattr(p, f) == getattr(q, f), f


# -- GPU: bit-exact against the oracle's scan-fused Voxblox mode ---------------------------------

def assert_bitwise(g, o):
    gi, gs, gw = g.export_voxels()
    oi, os_, ow = o.export_voxels()
    assert gi.shape == oi.shape, (gi.shape, oi.shape)
    assert np.array_equal(gi, oi)
    assert np.array_equal(gw.view(np.uint32), ow.view(np.uint32))
    bad = np.flatnonzero(gs.view(np.uint32) != os_.view(np.uint32))
    assert bad.size == 0, "sdf differs at %d voxels, e.g. %s: gpu %r oracle %r" % (
        bad.size, gi[bad[:3]].tolist(), gs[bad[:3]].tolist(), os_[bad[:3]].tolist())
    return gi.shape[0]


def run_both(scans, **kw):
    g, o = hip(**kw), ora(**kw)
    for pts, org in scans:
        g.integrate(pts, org)
        o.integrate(pts, org)
    g.sync()
    return g, o


@pytest.mark.gpu
def test_gpu_voxblox_scan_sequence_bitwise(sim):
    scans = [(decimate(p, 2), org) for p, org in (sim.scan(k) for k in (0, 1, 2, 30))]
    g, o = run_both(scans)
    n = assert_bitwise(g, o)
    assert n > 100000
    assert g.num_bricks() == o.num_bricks()


@pytest.mark.gpu
def test_gpu_voxblox_full_scan_batched_bitwise(sim):
    """Full 128x1024 scans, 8 per GPU batch, pipelined batches."""
    scans = [sim.scan(k) for k in range(10)]
    g, o = run_both(scans, max_batch=8, pipeline=True)
    assert_bitwise(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [
    dict(use_weight_dropoff=False),
    dict(max_weight=2.5),
    dict(max_range=20.0),                                     # clearing rays past 20 m
    dict(max_range=20.0, allow_clear=False),
    dict(space_carving=True, max_range=40.0, min_range=0.5),  # carving from the origin
], ids=["no-dropoff", "max-weight", "clearing", "no-clear", "carving"])
def test_gpu_voxblox_options_bitwise(sim, kw):
    k = 64 if kw.get("space_carving") else 8
    scans = [(decimate(p, k), org) for p, org in (sim.scan(j) for j in (0, 1, 2, 3))]
    g, o = run_both(scans, **kw)
    assert assert_bitwise(g, o) > 1000


@pytest.mark.gpu
def test_gpu_voxblox_query_background(sim):
    g = hip()
    p, org = sim.scan(0)
    g.integrate(decimate(p, 16), org)
    s, w = g.query_dense([-600, -600, -100], [-598, -598, -98])
    assert (s == 0).all() and (w == 0).all()


# -- Voxblox's default weight: 1 / z^2 of the sensor-frame depth (use_const_weight = False) -----

def _zaxis(q):
    """The sensor z axis of pose quaternion q (x, y, z, w) as the libraries compute it."""
    x, y, z, w = np.asarray(q, np.float64) / np.linalg.norm(q)
    return np.array([2 * (x * z + w * y), 2 * (y * z - w * x), 1 - 2 * (x * x + y * y)]).astype(F)


@pytest.mark.parametrize("pitch", [0.0, 0.4, -1.1])
def test_depth_weight_is_inverse_z_squared(pitch):
    """One ray, no dropoff: every voxel's weight is getVoxelWeight(point_C) = 1 / z^2 with z the
    point's depth along the sensor's z axis (here pitched about y by `pitch`)."""
    o = np.array([0.012, 0.013, 0.011])
    q = (0.0, math.sin(pitch / 2), 0.0, math.cos(pitch / 2))
    p = (o + [3.0, 0.4, -1.2]).astype(F)
    vol = ora(use_const_weight=False, use_weight_dropoff=False)
    vol.integrate(p[None], np.concatenate([o, q]))
    _, _, w = vol.export_voxels()
    zx, zy, zz = _zaxis(q)
    d = p - o.astype(F)
    z = abs(zx * d[0] + (zy * d[1] + zz * d[2]))
    w0 = F(1.0) / (z * z)
    assert w.size > 3 and np.all(w == w0), (w[:3], w0)
    # the const-weight mode (and the default integrate's world z axis) are unchanged
    c = ora(use_weight_dropoff=False)
    c.integrate(p[None], o)
    assert np.all(c.export_voxels()[2] == 1.0)


IDENT = [0.0, 0.0, 0.0, 1.0]  # identity orientation (qx, qy, qz, qw): the sensor z axis = world z


def test_depth_weight_tiny_z_gives_zero_weight():
    """|z| <= kEpsilon: weight 0, the samples are dropped (deviation 2)."""
    o = np.array([0.012, 0.013, 0.011])
    p = (o + [3.0, 0.4, 0.0]).astype(F)  # z = 0 along the world z axis
    vol = ora(use_const_weight=False)
    vol.integrate(p[None], np.concatenate([o, IDENT]))
    assert vol.export_voxels()[0].shape[0] == 0


def test_origin_only_scans_take_constant_weight():
    """A bare origin carries no orientation: with the 1/z^2 weight on, such a scan fuses with
    weight 1 (use_const_weight's field), not 1/(p.z - o.z)^2 of the world z axis (ABI v8)."""
    o = np.array([0.012, 0.013, 0.011])
    p = (o + [[3.0, 0.4, 0.0], [2.0, -1.0, 0.7]]).astype(F)
    a = ora(use_const_weight=False)
    a.integrate(p, o)
    b = ora(use_const_weight=True)
    b.integrate(p, o)
    for x, y in zip(a.export_voxels(), b.export_voxels()):
        assert np.array_equal(x, y)
    assert a.export_voxels()[0].shape[0] > 0


def test_depth_weight_is_capped():
    """Points a hair off the sensor plane (|z| ~ 1e-5 m: 1/z^2 ~ 1e10) take the capped weight
    min(max_weight, 2^16) per sample, so the exact int64 sums cannot overflow; the fused weight of
    one such sample is the cap."""
    o = np.array([0.0, 0.0, 0.0])
    for mw, cap in ((10000.0, 10000.0), (1e9, 65536.0)):
        pts = np.array([[3.0, 0.4, 1e-5], [3.0, 0.4, 2e-5]], F)
        vol = ora(use_const_weight=False, use_weight_dropoff=False, max_weight=mw)
        vol.integrate(pts[:1], np.concatenate([o, IDENT]))
        ijk, s, w = vol.export_voxels()
        assert ijk.shape[0] > 0 and np.all(w == np.float32(cap)), (mw, np.unique(w))
        assert np.all(np.abs(s) <= 0.15 + 1e-6)


def _posed_scans(sim, ks, decim):
    out = []
    for j, k in enumerate(ks):
        p, org = sim.scan(k)
        a, b = 0.3 * j - 0.2, 0.15 * j
        q = np.array([math.sin(a / 2) * math.cos(b), math.sin(a / 2) * math.sin(b), 0.1 * j,
                      math.cos(a / 2)])
        out.append((decimate(p, decim), np.concatenate([org, q])))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [
    dict(),
    dict(use_weight_dropoff=False),
    dict(space_carving=True, max_range=5.0, min_range=0.1),   # voxblox's defaults
], ids=["dropoff", "no-dropoff", "upstream-defaults"])
def test_gpu_voxblox_depth_weight_bitwise(sim, kw):
    k = 32 if kw.get("space_carving") else 4
    scans = _posed_scans(sim, (0, 1, 2, 30), k)
    g, o = run_both(scans, use_const_weight=False, **kw)
    assert assert_bitwise(g, o) > 1000
    gw = g.export_voxels()[2]
    assert np.unique(gw).size > 100  # weights are not counts any more


@pytest.mark.gpu
def test_gpu_voxblox_depth_weight_batch_device_poses(sim):
    """tsdf_integrate_batch_device_pose: device-resident scans with one pose each, 3 per batch."""
    import torch
    scans = _posed_scans(sim, range(7), 4)
    g = hip(use_const_weight=False, max_batch=3)
    o = ora(use_const_weight=False)
    x = torch.from_numpy(np.concatenate([p for p, _ in scans])).cuda()
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans])
    g.integrate_batch_device(x.data_ptr(), offs, np.stack([q for _, q in scans]))
    for p, q in scans:
        o.integrate(p, q)
    g.sync()
    assert assert_bitwise(g, o) > 1000
