"""Marching-cubes mesh extraction (VDBFusion VDBVolume::extract_triangle_mesh).

The default case table is generated; TSDF_MC_LORENSEN is the published table
VDBFusion compiles in (include/tsdf_mc_tables.h), checked structurally and compared case by case
with the generated one below.  The generated table is pinned by what a correct marching-cubes
table must satisfy: the product library's table equals the oracle's
independent construction; single-corner cases give one triangle on that corner's three edges;
and the mesh of a closed analytic surface is watertight, consistently oriented, of Euler
characteristic 2 and encloses the analytic volume.  The oracle's mesh itself (corner gather, halo
tiles, min_weight) equals a plain numpy restatement bit for bit.  The GPU mesh is then compared with
the oracle's bit for bit (same triangles, same order).
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


def published_table():
    """include/tsdf_mc_tables.h's triangle table (Bourke numbering), parsed from the header."""
    import os
    import re
    from conftest import REPO
    hdr = open(os.path.join(REPO, "include", "tsdf_mc_tables.h")).read()
    body = hdr[hdr.index("tsdf_mc_tri_table[256][16] = {"):]
    rows = re.findall(r"\{([-0-9, ]+)\}", body)
    assert len(rows) == 256
    return [[int(x) for x in r.split(",") if int(x) >= 0] for r in rows]


BOURKE_V = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
BOURKE_E = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6),
            (3, 7)]


def test_published_table_structure():
    """The committed triangle table is a marching-cubes table: every case uses exactly its
    sign-change edges, its triangles form a consistently oriented manifold patch whose boundary runs
    over the cube's faces through every crossing once, and every triangle faces the inside corners
    (the trilinear field decreases along its normal)."""
    rows = published_table()
    mid = {e: (np.array(BOURKE_V[a]) + np.array(BOURKE_V[b])) / 2.0 for e, (a, b) in enumerate(BOURKE_E)}

    def faces(e):
        pa, pb = BOURKE_V[BOURKE_E[e][0]], BOURKE_V[BOURKE_E[e][1]]
        return {(ax, pa[ax]) for ax in range(3) if pa[ax] == pb[ax]}

    for k, r in enumerate(rows):
        assert len(r) % 3 == 0 and len(r) <= 15, k
        cross = {e for e, (a, b) in enumerate(BOURKE_E) if (k >> a & 1) != (k >> b & 1)}
        assert set(r) == cross, k
        de = {}
        for t in range(0, len(r), 3):
            tri = r[t:t + 3]
            assert len(set(tri)) == 3, k
            for i in range(3):
                key = (tri[i], tri[(i + 1) % 3])
                assert key not in de, k  # each directed edge once: consistent orientation
                de[key] = 1
        bnd = [(a, b) for (a, b) in de if (b, a) not in de]
        assert sorted(a for a, _ in bnd) == sorted(cross) == sorted(b for _, b in bnd), k
        for a, b in bnd:
            assert faces(a) & faces(b), (k, a, b)

        def f(x):
            v = 0.0
            for c, (vx, vy, vz) in enumerate(BOURKE_V):
                w = (x[0] if vx else 1 - x[0]) * (x[1] if vy else 1 - x[1]) * (x[2] if vz else 1 - x[2])
                v += w * (-1.0 if k >> c & 1 else 1.0)
            return v
        for t in range(0, len(r), 3):
            p0, p1, p2 = (mid[e] for e in r[t:t + 3])
            n = np.cross(p1 - p0, p2 - p0)
            n /= np.linalg.norm(n)
            c = (p0 + p1 + p2) / 3
            assert f(c + 0.05 * n) < f(c - 0.05 * n), (k, t)


def renumbered_published():
    """The published table in this library's layout (corner c = (c&1, c>>1&1, c>>2&1), edges
    axis-major): what TSDF_MC_LORENSEN must hold, triangle order and winding kept."""
    kv = [0, 1, 3, 2, 4, 5, 7, 6]
    ke = [0, 5, 1, 4, 2, 7, 3, 6, 8, 9, 11, 10]
    out = np.zeros((256, 32), np.uint8)
    for b, r in enumerate(published_table()):
        k = sum(1 << kv[v] for v in range(8) if b >> v & 1)
        out[k, 0] = len(r) // 3
        out[k, 1:1 + len(r)] = [ke[e] for e in r]
    return out


def test_lorensen_is_the_published_table():
    from tsdf_map._lib import load_hip_library
    exp = renumbered_published()
    assert np.array_equal(table_of(oracle.load(), 1), exp)
    assert np.array_equal(table_of(load_hip_library(), 1), exp)


def _cycles(t, k, reverse=False):
    tris = [tuple(int(x) for x in t[k, 1 + 3 * i:4 + 3 * i]) for i in range(t[k, 0])]
    if reverse:
        tris = [(a, c, b) for a, b, c in tris]
    de = {(x, y) for a, b, c in tris for x, y in ((a, b), (b, c), (c, a))}
    nxt = {a: b for (a, b) in de if (b, a) not in de}
    cyc, seen = set(), set()
    for a in nxt:
        if a in seen:
            continue
        c, x = [], a
        while x not in seen:
            seen.add(x)
            c.append(x)
            x = nxt[x]
        i = c.index(min(c))
        cyc.add(tuple(c[i:] + c[:i]))
    return frozenset(cyc)


def test_published_table_vs_the_builders_tables():
    """Where the builder's tables differ from the published one: the GENERATED
    table has the published table's polygons in every case (the same crossings joined into the same
    cycles) with the opposite winding and its own fan triangulation; the round-3 'Lorensen rule'
    (complement symmetry, now TSDF_MC_LORENSEN_RULE) joins them differently in exactly the 44 cases
    that have an ambiguous face and more than 4 inside corners -- the published table does not
    follow complement symmetry there."""
    pub, gen, rule = renumbered_published(), table_of(oracle.load(), 0), table_of(oracle.load(), 2)
    assert all(_cycles(pub, k) == _cycles(gen, k, reverse=True) for k in range(256))
    differ = {k for k in range(256) if _cycles(pub, k) != _cycles(rule, k, reverse=True)}
    expect = {k for k in range(256) if _ambiguous_face(k) and bin(k).count("1") > 4}
    assert differ == expect and len(differ) == 44
    same_rows = sum(np.array_equal(pub[k], gen[k]) for k in range(256))
    assert same_rows == 2  # the empty and full cases: the triangulations themselves differ


def test_lorensen_rule_table():
    """TSDF_MC_LORENSEN_RULE (the classic complement-symmetry rule): it differs from the generated
    table exactly on the cases with an ambiguous face and more than 4 inside corners, and the
    product library builds the same table as the oracle."""
    from tsdf_map._lib import load_hip_library
    g = table_of(oracle.load(), 0)
    lo = table_of(oracle.load(), 2)
    assert np.array_equal(lo, table_of(load_hip_library(), 2))
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
    """Integrated scans (noisy surfaces: ambiguous cubes occur) meshed with the published table,
    GPU == oracle bit for bit."""
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


def numpy_marching_cubes(coords, sdf, weight, local, tab, vs, min_weight):
    """An independent restatement of the oracle's mesh (oracle/tsdf_oracle.c mesh_impl) over a
    dense grid: the cubes whose min voxel lies in a `local` brick, bricks in (z, y, x) order, cubes
    by in-brick index, triangles in table order; vertex = corner a's centre + t vs along the edge,
    t = S_a / (S_a - S_b), all in fp32."""
    edges = [(b, b | (1 << d)) for d in range(3) for b in range(8) if not b & (1 << d)]
    lo = coords.min(0) * 8
    dim = (coords.max(0) - coords.min(0) + 2) * 8  # +1 brick of unobserved margin
    S = np.zeros(dim[::-1], np.float32)
    U = np.zeros(dim[::-1], bool)
    for c, s, w in zip(coords, sdf.reshape(-1, 8, 8, 8), weight.reshape(-1, 8, 8, 8)):
        o = c * 8 - lo
        S[o[2]:o[2] + 8, o[1]:o[1] + 8, o[0]:o[0] + 8] = s
        U[o[2]:o[2] + 8, o[1]:o[1] + 8, o[0]:o[0] + 8] = (w > 0) & (w >= min_weight)
    vs32 = np.float32(vs)
    out = []
    order = np.lexsort((coords[local, 0], coords[local, 1], coords[local, 2]))
    for c in coords[local][order]:
        o = c * 8 - lo
        for l in range(512):
            x, y, z = o[0] + (l & 7), o[1] + ((l >> 3) & 7), o[2] + (l >> 6)
            cs = [(x + (q & 1), y + ((q >> 1) & 1), z + (q >> 2)) for q in range(8)]
            if not all(U[k[2], k[1], k[0]] for k in cs):
                continue
            sv = [S[k[2], k[1], k[0]] for k in cs]
            case = sum(1 << q for q in range(8) if sv[q] < 0)
            gx, gy, gz = (c[0] * 8 + (l & 7), c[1] * 8 + ((l >> 3) & 7), c[2] * 8 + (l >> 6))
            for t in range(tab[case, 0]):
                for j in range(3):
                    a, b = edges[tab[case, 1 + 3 * t + j]]
                    ax = {1: 0, 2: 1, 4: 2}[a ^ b]
                    tt = np.float32(sv[a] / np.float32(sv[a] - sv[b]))
                    p = [(np.float32(g + ((a >> i) & 1)) + np.float32(0.5)) * vs32
                         for i, g in enumerate((gx, gy, gz))]
                    p[ax] = np.float32(p[ax] + np.float32(tt * vs32))
                    out.append(p)
    return np.asarray(out, np.float32).reshape(-1, 3)


@pytest.mark.parametrize("tname", ["generated", "lorensen"])
@pytest.mark.parametrize("min_weight", [0.0, 0.75])
@pytest.mark.parametrize("with_halo", [False, True])
def test_oracle_mesh_equals_numpy_restatement(tname, min_weight, with_halo):
    """Pins the oracle's marching cubes (its dense-tile corner gather, its halo precedence and the
    min_weight rule) against the plain restatement above, bit for bit, on a sphere with holes,
    low-weight voxels and, with_halo, the +x half of the bricks handed over as halo tiles."""
    from tsdf_map import _abi
    rng = np.random.default_rng(7)
    coords, sdf, w = sphere_bricks(0.37)
    sdf = (sdf + rng.normal(0, 0.004, sdf.shape)).astype(np.float32)
    w = np.where(rng.random(w.shape) < 0.03, 0.0, np.where(rng.random(w.shape) < 0.05, 0.5, 1.0))
    w = w.astype(np.float32)
    local = coords[:, 0] < 1 if with_halo else np.ones(len(coords), bool)
    o = oracle.OracleTSDFVolume(VS, TAU)
    o.import_bricks(coords[local], sdf[local], w[local])
    halo = None
    tiles = np.zeros((int((~local).sum()), _abi.TILE_WORDS), np.uint32)
    if with_halo:
        for k, i in enumerate(np.nonzero(~local)[0]):
            tiles[k, :512] = sdf[i].reshape(-1).view(np.uint32)
            tiles[k, 512:1024] = w[i].reshape(-1).view(np.uint32)
            key = sum(int(coords[i, a] + (1 << 20)) << (21 * a) for a in range(3))
            tiles[k, 1024], tiles[k, 1025] = key & 0xFFFFFFFF, key >> 32
        halo = (tiles.ctypes.data, tiles.shape[0])
    verts, _ = o.extract_triangle_mesh(min_weight=min_weight, table=tname, halo=halo)
    buf = (C.c_uint8 * (256 * 32))()
    assert oracle.load().tsdf_mc_table_of(_abi.MC_TABLES[tname], buf) == 0
    tab = np.frombuffer(buf, np.uint8).reshape(256, 32)
    ref = numpy_marching_cubes(coords, sdf, w, local, tab, VS, min_weight)
    assert ref.shape[0] > 300
    assert verts.shape == ref.shape and np.array_equal(verts.view(np.uint32), ref.view(np.uint32))
    if with_halo:  # the halo is what meshes the cubes on the local / halo border
        assert o.extract_triangle_mesh(min_weight=min_weight, table=tname)[0].shape[0] < ref.shape[0]
