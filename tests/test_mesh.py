"""Marching-cubes mesh extraction (VDBFusion VDBVolume::extract_triangle_mesh).

The case table is generated, not transcribed, so it is pinned here by what a
correct marching-cubes table must satisfy: the product library's table equals the oracle's
independent construction; single-corner cases give one triangle on that corner's three edges;
and the mesh of a closed analytic surface is watertight, consistently oriented, of Euler
characteristic 2 and encloses the analytic volume.  The GPU mesh is then compared with the
oracle's bit for bit (same triangles, same order).
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle

VS, TAU = 0.05, 0.15


def table(lib):
    buf = (C.c_uint8 * (256 * 32))()
    assert lib.tsdf_mc_table(buf) == 0
    return np.frombuffer(buf, np.uint8).reshape(256, 32).copy()


def sphere_bricks(radius, center=(0.013, -0.021, 0.007), vs=VS, tau=TAU):
    """Bricks covering a ball of `radius` (+ margin), S = clamp(|c - center| - r, -tau, tau),
    W = 1 on every voxel: a fully observed field whose zero level set is a closed sphere."""
    lo = math.floor((-radius - 4 * vs) / (8 * vs)) - 1
    hi = math.floor((radius + 4 * vs) / (8 * vs)) + 1
    ax = np.arange(lo, hi + 1)
    bz, by, bx = np.meshgrid(ax, ax, ax, indexing="ij")
    coords = np.stack([bx.ravel(), by.ravel(), bz.ravel()], 1).astype(np.int32)
    l = np.arange(512)
    lx, ly, lz = l & 7, (l >> 3) & 7, l >> 6
    vx = coords[:, 0:1] * 8 + lx
    vy = coords[:, 1:2] * 8 + ly
    vz = coords[:, 2:3] * 8 + lz
    c = np.asarray(center)
    d = np.sqrt(((vx + 0.5) * vs - c[0]) ** 2 + ((vy + 0.5) * vs - c[1]) ** 2 +
                ((vz + 0.5) * vs - c[2]) ** 2) - radius
    sdf = np.clip(d, -tau, tau).astype(np.float32)
    return coords, sdf, np.ones_like(sdf)


def mesh_topology(verts):
    """(V, E, F, directed-edge balance ok, signed volume) of a triangle soup, vertices merged by
    exact position."""
    v = verts.reshape(-1, 3, 3)
    key = {}
    idx = np.empty(v.shape[:2], np.int64)
    for t in range(v.shape[0]):
        for j in range(3):
            k = tuple(v[t, j].tolist())
            idx[t, j] = key.setdefault(k, len(key))
    directed = {}
    for a, b, c in idx:
        for e in ((a, b), (b, c), (c, a)):
            directed[e] = directed.get(e, 0) + 1
    balanced = all(n == 1 and directed.get((e[1], e[0]), 0) == 1 for e, n in directed.items())
    undirected = {tuple(sorted(e)) for e in directed}
    vol = float(np.sum(np.einsum("ij,ij->i", v[:, 0].astype(np.float64),
                                 np.cross(v[:, 1].astype(np.float64), v[:, 2].astype(np.float64))))
                / 6.0)
    return len(key), len(undirected), v.shape[0], balanced, vol


def test_table_kats():
    t = table(oracle.load())
    assert t[0, 0] == 0 and t[255, 0] == 0
    edges = [(b, b | (1 << d)) for d in range(3) for b in range(8) if not b & (1 << d)]
    for c in range(8):  # one inside corner: one triangle on that corner's three edges
        for k in (1 << c, 255 ^ (1 << c)):
            assert t[k, 0] == 1, k
            tri = set(t[k, 1:4].tolist())
            assert tri == {e for e, (a, b) in enumerate(edges) if c in (a, b)}, k
    for k in range(256):  # every triangle vertex lies on a sign-change edge
        for e in t[k, 1:1 + 3 * t[k, 0]]:
            a, b = edges[e]
            assert ((k >> a) & 1) != ((k >> b) & 1), (k, e)
    assert t[:, 0].max() <= 10


def test_product_table_equals_oracle_table():
    from tsdf_map._lib import load_hip_library
    assert np.array_equal(table(load_hip_library()), table(oracle.load()))


@pytest.mark.parametrize("radius", [0.37, 1.1])
def test_sphere_mesh_is_closed_and_encloses_the_ball(radius):
    o = oracle.OracleTSDFVolume(VS, TAU)
    o.import_bricks(*sphere_bricks(radius))
    verts, tris = o.extract_triangle_mesh()
    assert tris.shape[0] > 50
    V, E, F, balanced, vol = mesh_topology(verts)
    assert balanced  # every directed edge once, its reverse once: closed and consistently oriented
    assert V - E + F == 2
    r = np.linalg.norm(verts - np.array([0.013, -0.021, 0.007]), axis=1)
    assert np.all(np.abs(r - radius) < VS)  # vertices on the sphere, within a voxel
    assert abs(abs(vol) - 4.0 / 3.0 * math.pi * radius ** 3) < 0.03 * 4.0 / 3.0 * math.pi * radius ** 3


def test_unobserved_voxels_are_not_meshed():
    o = oracle.OracleTSDFVolume(VS, TAU)
    coords, sdf, w = sphere_bricks(0.37)
    w[:, ::2] = 0.0  # every other voxel unobserved: no cube has 8 observed corners
    o.import_bricks(coords, sdf, w)
    assert o.extract_triangle_mesh()[1].shape[0] == 0
    o2 = oracle.OracleTSDFVolume(VS, TAU)
    o2.import_bricks(coords, sdf, np.ones_like(sdf))
    assert o2.extract_triangle_mesh(min_weight=2.0)[1].shape[0] == 0
    assert o2.extract_triangle_mesh(min_weight=1.0)[1].shape[0] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("radius", [0.37, 1.1])
def test_gpu_sphere_mesh_bitwise(radius):
    from tsdf_map import HipTSDFVolume
    bricks = sphere_bricks(radius)
    o = oracle.OracleTSDFVolume(VS, TAU)
    o.import_bricks(*bricks)
    g = HipTSDFVolume(VS, TAU, max_bricks=1 << 16, max_points=1 << 12)
    g.import_bricks(*bricks)
    vo, _ = o.extract_triangle_mesh()
    vg, _ = g.extract_triangle_mesh()
    assert vg.shape == vo.shape and np.array_equal(vg, vo)


@pytest.mark.gpu
def test_gpu_scan_mesh_bitwise(sim):
    from conftest import decimate
    from tsdf_map import HipTSDFVolume
    o = oracle.OracleTSDFVolume(VS, TAU)
    g = HipTSDFVolume(VS, TAU, max_bricks=1 << 18)
    for k in range(6):
        p, org = sim.scan(k)
        p = decimate(p, 4)
        o.integrate(p, org)
        g.integrate(p, org)
    for mw in (0.0, 2.0):
        vo, _ = o.extract_triangle_mesh(min_weight=mw)
        vg, _ = g.extract_triangle_mesh(min_weight=mw)
        assert vo.shape[0] > 1000
        assert vg.shape == vo.shape and np.array_equal(vg, vo), mw


def table_of(lib, which):
    buf = (C.c_uint8 * (256 * 32))()
    assert lib.tsdf_mc_table_of(which, buf) == 0
    return np.frombuffer(buf, np.uint8).reshape(256, 32).copy()


def _ambiguous_face(k):
    """Some cube face has its two inside corners on a diagonal."""
    for d in range(3):
        u, w = (d + 1) % 3, (d + 2) % 3
        for s in range(2):
            q = [(s << d) | (a << u) | (b << w) for a, b in ((0, 0), (1, 0), (1, 1), (0, 1))]
            i = [(k >> c) & 1 for c in q]
            if i[0] == i[2] and i[1] == i[3] and i[0] != i[1]:
                return True
    return False


def test_lorensen_table_rule():
    """TSDF_MC_LORENSEN (VDBFusion's classic table rule): it differs from the
    generated table exactly on the cases with an ambiguous face and more than 4 inside corners,
    and the product library builds the same table as the oracle."""
    from tsdf_map._lib import load_hip_library
    g = table_of(oracle.load(), 0)
    lo = table_of(oracle.load(), 1)
    assert np.array_equal(lo, table_of(load_hip_library(), 1))
    assert np.array_equal(g, table(oracle.load()))
    differ = {k for k in range(256) if not np.array_equal(g[k], lo[k])}
    expect = {k for k in range(256) if _ambiguous_face(k) and bin(k).count("1") > 4}
    assert differ == expect and len(differ) > 0
    edges = [(b, b | (1 << d)) for d in range(3) for b in range(8) if not b & (1 << d)]
    for k in range(256):  # still on sign-change edges
        for e in lo[k, 1:1 + 3 * lo[k, 0]]:
            a, b = edges[e]
            assert ((k >> a) & 1) != ((k >> b) & 1), (k, e)


@pytest.mark.gpu
@pytest.mark.parametrize("radius", [0.37, 1.1])
def test_gpu_sphere_mesh_lorensen_bitwise(radius):
    from tsdf_map import HipTSDFVolume
    bricks = sphere_bricks(radius)
    o = oracle.OracleTSDFVolume(VS, TAU)
    o.import_bricks(*bricks)
    g = HipTSDFVolume(VS, TAU, max_bricks=1 << 16, max_points=1 << 12)
    g.import_bricks(*bricks)
    vo, _ = o.extract_triangle_mesh(table="lorensen")
    vg, _ = g.extract_triangle_mesh(table="lorensen")
    assert vg.shape == vo.shape and np.array_equal(vg, vo)


@pytest.mark.gpu
def test_gpu_scan_mesh_lorensen_bitwise(sim):
    """Integrated scans (noisy surfaces: ambiguous cubes occur) meshed with the classic table, GPU
    == oracle bit for bit; the two tables' meshes differ only where ambiguous cubes are."""
    from conftest import decimate
    from tsdf_map import HipTSDFVolume
    o = oracle.OracleTSDFVolume(VS, TAU)
    g = HipTSDFVolume(VS, TAU, max_bricks=1 << 18)
    for k in range(6):
        p, org = sim.scan(k)
        p = decimate(p, 4)
        o.integrate(p, org)
        g.integrate(p, org)
    vo, _ = o.extract_triangle_mesh(table="lorensen")
    vg, _ = g.extract_triangle_mesh(table="lorensen")
    assert vo.shape[0] > 1000
    assert vg.shape == vo.shape and np.array_equal(vg, vo)
