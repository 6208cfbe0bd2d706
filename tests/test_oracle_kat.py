"""Pin the CPU oracle (oracle/tsdf_oracle.c) with closed-form known-answer tests.

No test in the reference pins TSDF values (the TSDF node and its backends are absent, SURVEY.md
§0/§8c), so the oracle's restatement of VDBFusion's Integrate is pinned here analytically:
single rays (exact voxel list + sdf in closed form), a plane wall and a sphere (sdf bounded by the
point-to-surface geometry), plus the invariances the semantics imply.
"""
import math

import numpy as np
import pytest

import oracle

VS, TAU = 0.05, 0.15


def vol(**kw):
    return oracle.OracleTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def closed_form_axis_ray(p, o, vs=VS, tau=TAU):
    """Ray parallel to +x: voxels floor(x/vs) over the band, sdf = sign * |p - c|."""
    d = p[0] - o[0]
    j, k = math.floor(o[1] / vs), math.floor(o[2] / vs)
    lo = math.floor((o[0] + d - tau) / vs)
    hi = math.floor((o[0] + d + tau) / vs)
    out = []
    for i in range(lo, hi + 1):
        c = np.array([(i + 0.5) * vs, (j + 0.5) * vs, (k + 0.5) * vs])
        dist = float(np.linalg.norm(np.asarray(p) - c))
        sdf = dist if np.dot(c - o, np.asarray(p) - c) > 0 else -dist
        if sdf > -tau:
            out.append(((i, j, k), min(tau, sdf)))
    return out


@pytest.mark.parametrize("p,o", [
    ((5.01, 0.01, 0.02), (0.001, 0.01, 0.02)),
    ((12.337, -3.21, 1.013), (-0.2, -3.21, 1.013)),
    ((-40.0, 7.77, -1.81), (0.5, 7.77, -1.81)),   # a -x ray
])
def test_single_axis_ray_closed_form(p, o):
    p, o = np.array(p), np.array(o)
    v = vol()
    got = v.ray_voxels(p, o)
    assert got is not None
    ijk, s = got
    if p[0] < o[0]:
        # mirror: a -x ray visits the same voxel set in descending order
        exp = closed_form_axis_ray_neg(p, o)
    else:
        exp = closed_form_axis_ray(p, o)
    assert [tuple(x) for x in ijk.tolist()] == [e[0] for e in exp]
    np.testing.assert_allclose(s, [e[1] for e in exp], rtol=0, atol=2e-6)


def closed_form_axis_ray_neg(p, o, vs=VS, tau=TAU):
    d = o[0] - p[0]
    j, k = math.floor(o[1] / vs), math.floor(o[2] / vs)
    hi = math.floor((o[0] - (d - tau)) / vs)
    lo = math.floor((o[0] - (d + tau)) / vs)
    out = []
    for i in range(hi, lo - 1, -1):
        c = np.array([(i + 0.5) * vs, (j + 0.5) * vs, (k + 0.5) * vs])
        dist = float(np.linalg.norm(np.asarray(p) - c))
        sdf = dist if np.dot(c - o, np.asarray(p) - c) > 0 else -dist
        if sdf > -tau:
            out.append(((i, j, k), min(tau, sdf)))
    return out


def _dda_float64(p, o, vs=VS, tau=TAU):
    """Independent float64 segment/voxel traversal (reference for the fp32 DDA)."""
    d = np.asarray(p, float) - o
    depth = np.linalg.norm(d)
    u = d / depth
    a = (o + u * (depth - tau)) / vs
    b = (o + u * (depth + tau)) / vs
    return a, b


def test_diagonal_rays_traverse_the_band():
    rng = np.random.default_rng(7)
    v = vol(space_carving=False)
    for _ in range(200):
        o = rng.uniform(-3, 3, 3).astype(np.float32).astype(np.float64)
        p = (o + rng.normal(size=3) * rng.uniform(2, 40)).astype(np.float32).astype(np.float64)
        got = v.ray_voxels(p, o)
        ijk, s = got
        assert len(ijk) >= 3
        steps = np.abs(np.diff(ijk.astype(np.int64), axis=0)).sum(1)
        # gating only removes voxels at the far (behind-surface) end, so the list stays 6-connected
        assert np.all(steps == 1)
        a, _ = _dda_float64(p, o)
        assert np.array_equal(ijk[0], np.floor(a).astype(np.int32)) or \
            np.min(np.abs(a - np.round(a))) < 1e-4
        # every sample is a truncated point-to-voxel distance
        c = (ijk + 0.5) * VS
        dist = np.linalg.norm(p - c, axis=1)
        # fp32 cancellation in p - c: a few ulp of the coordinates (|p| <= ~45 m -> ulp 3.8e-6)
        np.testing.assert_allclose(np.abs(s), np.minimum(dist, TAU), rtol=0, atol=2e-5)
        assert np.all(s > -TAU) and np.all(s <= TAU)


def _fan(center_dir, half_angle_deg, n, rng):
    """n unit directions within half_angle of center_dir."""
    c = np.asarray(center_dir, float)
    c /= np.linalg.norm(c)
    t1 = np.cross(c, [0.0, 0.0, 1.0] if abs(c[2]) < 0.9 else [1.0, 0.0, 0.0])
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(c, t1)
    ang = np.deg2rad(half_angle_deg) * np.sqrt(rng.uniform(0, 1, n))
    phi = rng.uniform(0, 2 * np.pi, n)
    return (np.cos(ang)[:, None] * c + np.sin(ang)[:, None] *
            (np.cos(phi)[:, None] * t1 + np.sin(phi)[:, None] * t2))


def test_plane_wall_kat():
    """KAT-2: wall x = 10 seen from the origin within a 20 degree cone."""
    rng = np.random.default_rng(1)
    u = _fan([1, 0, 0], 20.0, 20000, rng)
    p = (u * (10.0 / u[:, :1])).astype(np.float32)
    v = vol()
    v.integrate(p, np.zeros(3))
    ijk, s, w = v.export_voxels()
    c = (ijk + 0.5) * VS
    d = 10.0 - c[:, 0]
    L = VS * math.sqrt(3) / 2 + np.abs(d) * math.tan(math.radians(20.0))
    lo = np.minimum(np.abs(d), TAU)
    hi = np.minimum(np.sqrt(d * d + L * L), TAU)
    a = np.abs(s.astype(np.float64))
    assert np.all(a >= lo - 1e-5)
    assert np.all(a <= hi + 1e-5)
    far = np.abs(d) > VS
    assert np.all(np.sign(s[far]) == np.sign(d[far]))
    assert np.all(w >= 1)


def test_sphere_kat():
    """KAT-3: sphere of radius 5 around the origin, normal incidence everywhere."""
    rng = np.random.default_rng(2)
    u = rng.normal(size=(30000, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    p = (5.0 * u).astype(np.float32)
    v = vol()
    v.integrate(p, np.zeros(3))
    ijk, s, w = v.export_voxels()
    c = (ijk + 0.5) * VS
    r = np.linalg.norm(c, axis=1)
    d = 5.0 - r
    L = VS * math.sqrt(3) / 2 + 1e-3
    lo = np.minimum(np.abs(d), TAU)
    hi = np.minimum(np.sqrt(d * d + L * L), TAU)
    a = np.abs(s.astype(np.float64))
    assert np.all(a >= lo - 1e-4)
    assert np.all(a <= hi + 1e-4)
    far = np.abs(d) > VS
    assert np.all(np.sign(s[far]) == np.sign(d[far]))


def test_permutation_invariance_bitwise(scan0):
    """Scan-fused accumulation is exact: point order cannot change a single bit."""
    pts, o = scan0
    sub = np.ascontiguousarray(pts[::8])
    perm = np.random.default_rng(3).permutation(sub.shape[0])
    a, b = vol(), vol()
    a.integrate(sub, o)
    b.integrate(sub[perm], o)
    for x, y in zip(a.export_voxels(), b.export_voxels()):
        assert np.array_equal(x, y)


def test_sequential_vdbfusion_order_within_tolerance(scan0, sim):
    """The literal per-sample fp32 running average (VDBFusion order) vs the scan-fused field:
    identical voxel set and weights, |dSDF| <= 1e-5 m (the stated parity tolerance)."""
    seq = vol(mode=oracle.MODE_SEQUENTIAL)
    fus = vol()
    for k in range(2):
        pts, o = sim.scan(k)
        pts = np.ascontiguousarray(pts[::4])
        seq.integrate(pts, o)
        fus.integrate(pts, o)
    i1, s1, w1 = seq.export_voxels()
    i2, s2, w2 = fus.export_voxels()
    assert np.array_equal(i1, i2)
    assert np.array_equal(w1, w2)
    assert np.max(np.abs(s1 - s2)) <= 1e-5


def test_scan_order_changes_only_rounding(sim):
    a, b = vol(), vol()
    A = sim.scan(0)
    B = sim.scan(5)
    A = (np.ascontiguousarray(A[0][::8]), A[1])
    B = (np.ascontiguousarray(B[0][::8]), B[1])
    a.integrate(*A)
    a.integrate(*B)
    b.integrate(*B)
    b.integrate(*A)
    i1, s1, w1 = a.export_voxels()
    i2, s2, w2 = b.export_voxels()
    assert np.array_equal(i1, i2) and np.array_equal(w1, w2)
    assert np.max(np.abs(s1 - s2)) <= 1e-6


def test_range_filter_and_degenerate_points():
    v = vol(min_range=1.0, max_range=30.0)
    pts = np.array([[0, 0, 0],            # Ouster r = 0 -> (0,0,0)
                    [0.5, 0, 0],          # < min_range
                    [40, 0, 0],           # > max_range
                    [np.nan, 1, 1],
                    [np.inf, 0, 0],
                    [5.01, 0.01, 0.02]], np.float32)
    v.integrate(pts, np.zeros(3))
    st = v.stats()
    assert st["n_rays_total"] == 1
    ijk, s, w = v.export_voxels()
    assert len(ijk) == len(v.ray_voxels(pts[-1], np.zeros(3))[0])


def test_empty_scan():
    v = vol()
    v.integrate(np.zeros((0, 3), np.float32), np.zeros(3))
    assert v.export_voxels()[0].shape == (0, 3)
    assert v.num_bricks() == 0


def test_space_carving_marks_free_space():
    v = vol(space_carving=True, max_range=100.0)
    o = np.array([0.001, 0.01, 0.02])
    p = np.array([5.01, 0.01, 0.02], np.float32)
    ijk, s = v.ray_voxels(p, o)
    # voxel 103 (centre 5.175) is 0.166 m behind the hit: gated out by sdf > -tau
    assert ijk[0, 0] == 0 and ijk[-1, 0] == 102
    assert np.all(np.abs(np.diff(ijk[:, 0])) == 1)
    free = (ijk[:, 0] + 0.5) * VS < 5.01 - TAU
    assert np.all(s[free] == np.float32(TAU))


def test_brick_export_matches_voxel_export(scan0):
    pts, o = scan0
    v = vol()
    v.integrate(np.ascontiguousarray(pts[::16]), o)
    from tsdf_map import bricks_to_voxels
    a = bricks_to_voxels(*v.export_bricks())
    b = v.export_voxels()
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    # dense query over the bounding box agrees with the sparse export
    ijk, s, w = b
    lo = ijk[len(ijk) // 2] - np.array([20, 20, 10])  # a box around an observed voxel
    hi = lo + np.array([40, 40, 20])
    qs, qw = v.query_dense(lo, hi)
    m = np.all((ijk >= lo) & (ijk < hi), 1)
    rel = ijk[m] - lo
    assert np.array_equal(qs[rel[:, 2], rel[:, 1], rel[:, 0]], s[m])
    assert np.array_equal(qw[rel[:, 2], rel[:, 1], rel[:, 0]], w[m])
    assert np.count_nonzero(qw) == np.count_nonzero(m) > 0
    assert np.all(qs[qw == 0] == np.float32(TAU))


def test_import_merges_as_weighted_mean(scan0):
    pts, o = scan0
    a, b, ab = vol(), vol(), vol()
    half = np.ascontiguousarray(pts[::8])
    a.integrate(half[0::2], o)
    b.integrate(half[1::2], o)
    ab.import_bricks(*a.export_bricks())
    ab.import_bricks(*b.export_bricks())
    ref = vol()
    ref.integrate(half, o)
    i1, s1, w1 = ab.export_voxels()
    i2, s2, w2 = ref.export_voxels()
    assert np.array_equal(i1, i2) and np.array_equal(w1, w2)
    assert np.max(np.abs(s1 - s2)) <= 1e-6


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion"])
@pytest.mark.parametrize("origin", [(3.1, -7.3, 0.7), (2.0, -1.5, 0.25)])
def test_zero_range_point_is_origin_ray(semantics, origin):
    """an Ouster r = 0 pixel becomes the sensor origin rounded to float
    (cartesian.h:64-65 after the pose).  fp32 restatement: that point minus (float)origin is zero,
    the ray has no length and is dropped.  VDBFusion at its precisions: the point minus the DOUBLE
    origin is a rounding error, unless the origin is a float, so a non-float origin keeps a
    micrometre ray whose band surrounds the origin (as upstream's Integrate would); DLIO's crop box
    (min_range 1 m) drops it in both modes."""
    o = np.array(origin, np.float64)
    p = o.astype(np.float32).reshape(1, 3)
    exact = bool(np.all(p[0].astype(np.float64) == o))
    for min_range, keep in ((0.0, semantics == "vdbfusion_f64" and not exact), (1.0, False)):
        v = vol(semantics=semantics, min_range=min_range)
        v.integrate(p, o)
        assert v.stats()["n_rays_total"] == (1 if keep else 0), (min_range, exact)
        ijk, s, w = v.export_voxels()
        if keep:  # the band of a ray of ~0 length: voxels around the origin, all within tau
            c = (ijk.astype(np.float64) + 0.5) * VS
            assert len(ijk) > 0 and np.all(np.linalg.norm(c - o, axis=1) <= TAU + VS)
        else:
            assert len(ijk) == 0
