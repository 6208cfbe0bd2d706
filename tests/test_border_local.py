"""ABI v9 on the CPU oracle (the GPU library's twin): the border reduce as a transaction
(tsdf_border_commit_device), the one-process sharded calls (tsdf_create_sharded,
tsdf_integrate_sectors[_origin], tsdf_border_reduce_local), and the sharded mesh
(tsdf_halo_* / tsdf_extract_mesh_local).  tests/test_multigpu.py runs the same on the GPU."""
import ctypes as C

import numpy as np
import pytest

import oracle
from test_distributed import tri_set
from test_multigpu import emulated_reduce_host, voxels_equal_bitwise
from tsdf_map import _abi, border_reduce_local, extract_mesh_local, integrate_sectors

VS, TAU = 0.05, 0.15


def sharded(n, yaw0=0.3, **kw):
    lib = oracle.load()
    p = oracle.OracleTSDFVolume.make_params(lib, VS, TAU, sector_yaw0=yaw0, **kw)
    out = (C.c_void_p * n)()
    assert lib.tsdf_create_sharded(C.byref(p), n, None, out) == 0
    vols = []
    for k in range(n):
        v = oracle.OracleTSDFVolume.__new__(oracle.OracleTSDFVolume)
        v._lib = lib
        v._ctx = C.c_void_p(out[k])
        q = _abi.TsdfParams.from_buffer_copy(p)
        q.n_sectors, q.sector = n, k
        v._adopt(q)
        vols.append(v)
    return vols


def union_voxels(vols):
    from tsdf_map import bricks_to_voxels
    parts = [v.export_bricks() for v in vols]
    keep = [(w.reshape(len(c), -1) > 0).any(1) for c, _, w in parts]
    coords = np.concatenate([c[k] for (c, _, _), k in zip(parts, keep)])
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]  # each brick once
    return bricks_to_voxels(coords, np.concatenate([s[k] for (_, s, _), k in zip(parts, keep)]),
                            np.concatenate([w[k] for (_, _, w), k in zip(parts, keep)]))


def test_abort_restores_every_field(sim):
    """pack + merge + commit(0): every context's field is the one before, bit for bit; while the
    reduce is open the contexts refuse scans and imports."""
    n = 3
    vols = [oracle.OracleTSDFVolume(VS, TAU, n_sectors=n, sector=r, sector_yaw0=0.3) for r in range(n)]
    for k in (0, 2):
        pts, org = sim.scan(k)
        for v in vols:
            v.integrate(np.ascontiguousarray(pts[::4]), org)
    before = [v.export_voxels() for v in vols]
    keys = [np.empty(max(v.num_bricks(), 1), np.int64) for v in vols]
    counts = [v.brick_keys_into(k.ctypes.data, k.size) for v, k in zip(vols, keys)]
    stride = max(counts)
    allk = np.full((n, stride), -1, np.int64)
    for r in range(n):
        allk[r, :counts[r]] = keys[r][:counts[r]]
    sends, splits = [], []
    for r, v in enumerate(vols):
        s = np.empty((max(counts[r], 1), 1028), np.int32)
        splits.append(v.border_pack(allk.ctypes.data, counts, stride, n, r, s.ctypes.data, s.shape[0]))
        sends.append(s)
    assert sum(map(sum, splits)) > 50
    for d, v in enumerate(vols):
        parts = [sends[r][sum(splits[r][:d]):sum(splits[r][:d]) + splits[r][d]] for r in range(n)]
        rc = [splits[r][d] for r in range(n)]
        recv = np.ascontiguousarray(np.concatenate(parts)) if sum(rc) else np.empty((1, 1028), np.int32)
        v.border_merge(recv.ctypes.data, rc)
    pts, org = sim.scan(4)
    with pytest.raises(Exception, match="border reduce is open"):
        vols[1].integrate(np.ascontiguousarray(pts[::4]), org)
    assert any(not voxels_equal_bitwise(v.export_voxels(), b) for v, b in zip(vols, before))
    for v in vols:
        v.border_commit(False)
    for v, b in zip(vols, before):
        assert voxels_equal_bitwise(v.export_voxels(), b)
    vols[1].integrate(np.ascontiguousarray(pts[::4]), org)  # open no more


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "voxblox"])
def test_reduce_local_matches_emulated(sim, semantics):
    """tsdf_border_reduce_local (C) equals the collective's steps driven from Python, and the union
    equals the single-volume field (VDBFusion: weights exact, |dS| <= 1e-5 m)."""
    n = 4
    a = sharded(n, semantics=semantics)
    b = [oracle.OracleTSDFVolume(VS, TAU, n_sectors=n, sector=r, sector_yaw0=0.3,
                                 semantics=semantics) for r in range(n)]
    ref = oracle.OracleTSDFVolume(VS, TAU, semantics=semantics)
    for k in (0, 1, 5):
        pts, org = sim.scan(k)
        pose = np.concatenate([org, [0.0, 0.0, np.sin(0.05 * k), np.cos(0.05 * k)]])
        pts = np.ascontiguousarray(pts[::4])
        integrate_sectors(a, pts, pose)
        for v in b + [ref]:
            v.integrate(pts, pose)
    assert border_reduce_local(a) > 50
    emulated_reduce_host(b)
    for r in range(n):
        assert voxels_equal_bitwise(a[r].export_voxels(), b[r].export_voxels()), r
    if semantics != "voxblox":  # Voxblox partial fields merge approximately (clamps)
        mi, ms, mw = union_voxels(a)
        ri, rs, rw = ref.export_voxels()
        assert np.array_equal(mi, ri) and np.array_equal(mw, rw)
        assert np.max(np.abs(ms - rs)) <= 1e-5


def test_sectors_bare_origin_keeps_constant_weight(sim):
    """a bare origin on the sectors path carries no orientation, like `integrate`:
    under Voxblox's 1/z^2 default the sector fields equal the sectors of the unsharded
    integrate(points, origin) field (constant weight), not world-z 1/z^2 weights."""
    n = 3
    kw = dict(semantics="voxblox", use_const_weight=False, max_range=100.0)
    a = sharded(n, **kw)
    b = [oracle.OracleTSDFVolume(VS, TAU, n_sectors=n, sector=r, sector_yaw0=0.3, **kw)
         for r in range(n)]
    tilted = [oracle.OracleTSDFVolume(VS, TAU, n_sectors=n, sector=r, sector_yaw0=0.3, **kw)
              for r in range(n)]
    for k in (0, 3):
        pts, org = sim.scan(k)
        pts = np.ascontiguousarray(pts[::4])
        integrate_sectors(a, pts, org)
        for v in b:
            v.integrate(pts, org)
        for v in tilted:
            v.integrate(pts, np.concatenate([org, [0.0, 0.0, 0.0, 1.0]]))
    for r in range(n):
        assert voxels_equal_bitwise(a[r].export_voxels(), b[r].export_voxels()), r
    assert not voxels_equal_bitwise(a[0].export_voxels(), tilted[0].export_voxels())


@pytest.mark.parametrize("table", ["generated", "lorensen"])
def test_mesh_local_is_mesh_of_union(sim, table):
    """tsdf_extract_mesh_local: border reduce, halo exchange, one mesh per context; the soups
    together are the mesh of the union field triangle for triangle, and the unsharded mesh's
    triangle count within the border voxels' rounding."""
    n = 4
    a = sharded(n)
    ref = oracle.OracleTSDFVolume(VS, TAU)
    for k in (0, 2):
        pts, org = sim.scan(k)
        pts = np.ascontiguousarray(pts[::4])
        integrate_sectors(a, pts, org)
        ref.integrate(pts, org)
    v, _ = extract_mesh_local(a, table=table)
    union = oracle.OracleTSDFVolume(VS, TAU)
    for vol in a:
        c, s, w = vol.export_bricks()
        keep = (w.reshape(len(c), -1) > 0).any(1)
        union.import_bricks(c[keep], s[keep], w[keep])
    want = union.extract_triangle_mesh(table=table)[0]
    assert v.shape[0] > 3000
    assert np.array_equal(tri_set(v), tri_set(want))
    full = ref.extract_triangle_mesh(table=table)[0]
    assert abs(full.shape[0] - v.shape[0]) <= 0.001 * full.shape[0]
