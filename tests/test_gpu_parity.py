"""GPU parity: libtsdf_hip.so (through the C-ABI) against the CPU oracle on the same inputs.

Bar: the touched-voxel set, the weights AND the sdf values are BIT-EXACT against
the oracle's scan-fused mode — both run the same fp32 op sequence and sum each scan's samples as
exact fixed point, so no tolerance is needed.  The multi-sector merge is the one place a tolerance
applies (fp32 weighted means of partial fields): |dSDF| <= 1e-5 m, weights exact.
"""
import math

import numpy as np
import pytest

import oracle
from conftest import decimate

pytestmark = pytest.mark.gpu

VS, TAU = 0.05, 0.15


# Every case runs in both VDBFusion modes: the ABI default vdbfusion_f64 (upstream's precisions,
# the bench's mode) and the fp32 restatement; a case that names its semantics keeps them.
_SEM = {"default": "vdbfusion_f64"}


def pytest_generate_tests(metafunc):
    if "semantics" not in metafunc.fixturenames:
        metafunc.parametrize("vdb_mode", ["vdbfusion_f64", "vdbfusion"], indirect=True)


@pytest.fixture(autouse=True)
def vdb_mode(request):
    _SEM["default"] = getattr(request, "param", "vdbfusion_f64")
    yield _SEM["default"]
    _SEM["default"] = "vdbfusion_f64"


def hip(**kw):
    from tsdf_map import HipTSDFVolume
    kw.setdefault("semantics", _SEM["default"])
    return HipTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def ora(**kw):
    kw.setdefault("semantics", _SEM["default"])
    return oracle.OracleTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def assert_bitwise(g, o):
    gi, gs, gw = g.export_voxels()
    oi, os_, ow = o.export_voxels()
    assert gi.shape == oi.shape, (gi.shape, oi.shape)
    assert np.array_equal(gi, oi)
    assert np.array_equal(gw, ow)
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


def test_single_rays():
    scans = [(np.array([[5.01, 0.01, 0.02]], np.float32), np.array([0.001, 0.01, 0.02])),
             (np.array([[-40.0, 7.77, -1.81], [3.3, -2.2, 1.1]], np.float32), np.array([0.5, 7.77, -1.81]))]
    g, o = run_both(scans)
    assert assert_bitwise(g, o) > 0


def test_decimated_scan_bitwise(scan0):
    pts, org = scan0
    g, o = run_both([(decimate(pts, 16), org)])
    assert assert_bitwise(g, o) > 10000


def test_full_c1_scan_bitwise(scan0):
    """C1: one full 128x1024 synthetic Ouster scan (the trajectory's first pose: origin (8, 0, 0),
    yaw pi/2), 5 cm / 15 cm."""
    g, o = run_both([scan0])
    n = assert_bitwise(g, o)
    st = g.stats()
    assert st["n_voxels_last"] == n  # U_vox counted by the kernel == oracle's voxel count
    assert st["n_rays_total"] == scan0[0].shape[0]
    assert st["n_bricks"] == o.num_bricks()


def test_scan_sequence_bitwise(sim):
    scans = [sim.scan(k) for k in (0, 1, 2, 30)]
    g, o = run_both(scans)
    assert_bitwise(g, o)


def test_batch_composition_is_invisible(sim):
    """Scans integrated 1, 3 or 32 per GPU batch (host queue) and through the device batch API
    give the same bits, equal to the oracle's scan-by-scan integration."""
    import torch
    scans = [(decimate(p, 4), o) for p, o in (sim.scan(k) for k in range(10))]
    o = ora()
    for p, org in scans:
        o.integrate(p, org)
    ref = o.export_voxels()
    for mb in (1, 3, 32):
        g = hip(max_batch=mb)
        for p, org in scans:
            g.integrate(p, org)
        got = g.export_voxels()
        st = g.stats()
        assert st["n_batches"] == -(-10 // mb) and st["n_scans"] == 10
        for x, y in zip(got, ref):
            assert np.array_equal(x, y), mb
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    g = hip(max_batch=4)
    g.integrate_batch_device(d.data_ptr(), offs, np.stack([org for _, org in scans]))
    for x, y in zip(g.export_voxels(), ref):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("semantics", ["vdbfusion", "vdbfusion_f64", "voxblox", "voxblox_z2"])
def test_small_batch_kernel_bitwise(sim, monkeypatch, semantics):
    """Batches of <= 8 scans fuse in k_integrate_small (one wave per brick, dense LDS cells, no
    size order) and, below 256 blocks, count in 1024-lane k_count workgroups; TSDF_SMALL_NS=0 and
    TSDF_COUNT_WIDE=0 force k_integrate and the 256-lane k_count.  Both equal the oracle bit for bit
    at 1, 3 and 8 scans per batch, on a full scan (long per-voxel runs of one scan) and with
    carving."""
    from tsdf_map import bricks_to_voxels
    kw = dict(semantics="voxblox", use_const_weight=False) if semantics == "voxblox_z2" else \
        dict(semantics=semantics)
    full = [sim.scan(0)] + [(decimate(p, 4), org) for p, org in (sim.scan(k) for k in range(1, 6))]
    carve = [(decimate(p, 16), org) for p, org in (sim.scan(k) for k in range(4))]
    for scans, extra in ((full, {}), (carve, dict(space_carving=True, max_range=20.0))):
        o = ora(**kw, **extra)
        for p, org in scans:
            o.integrate(p, org)
        ref = o.export_voxels()
        for mb in (1, 3, 8):
            got = {}
            for small in ("8", "0") if mb != 3 else ("8",):
                monkeypatch.setenv("TSDF_SMALL_NS", small)
                monkeypatch.setenv("TSDF_COUNT_WIDE", "256" if small != "0" else "0")
                g = hip(max_batch=mb, **kw, **extra)
                for p, org in scans:
                    g.integrate(p, org)
                got[small] = g.export_bricks()  # the same batches: the same pool slots
            for x, y in zip(bricks_to_voxels(*got["8"]), ref):
                assert np.array_equal(x, y), (mb, extra)
            if "0" in got:
                for x, y in zip(got["8"], got["0"]):
                    assert np.array_equal(x, y), (mb, extra)


def test_paired_count_workgroups_bitwise(sim, monkeypatch):
    """TSDF_COUNT_PAIRED=1: k_count takes two 1024-ray blocks per 512-lane workgroup (one LDS brick
    hash, per-(block, half) sub-runs).  Scans decimated by 3 have an odd block count (43), so
    workgroups also straddle two scans (the block bit in the LDS key); with and without carving
    (long rays: the per-pair emission path).  Equal to the oracle bit for bit."""
    monkeypatch.setenv("TSDF_COUNT_PAIRED", "1")
    monkeypatch.setenv("TSDF_COUNT_WIDE", "0")
    scans = [(decimate(p, 3), org) for p, org in (sim.scan(k) for k in range(5))]
    for extra in ({}, dict(space_carving=True, max_range=20.0)):
        g, o = run_both(scans, max_batch=5, **extra)
        assert assert_bitwise(g, o) > 10000, extra


def test_pipelined_and_64_scan_batches_bitwise(sim):
    """Overlapped batches (tsdf_params.pipeline: batch b+1's count/compact/place beside batch b's
    integrate, two streams) and 64-scan batches give the oracle's bits, through the host queue and
    the device batch API, with read-outs interleaved between integrations."""
    import torch
    scans = [(decimate(p, 8), o) for p, o in (sim.scan(k) for k in range(70))]
    o = ora()
    for p, org in scans:
        o.integrate(p, org)
    ref = o.export_voxels()
    for mb, pipe in ((2, True), (5, True), (64, False), (64, True), (7, 2), (64, 2)):
        g = hip(max_batch=mb, pipeline=pipe)
        for k, (p, org) in enumerate(scans):
            g.integrate(p, org)
            if k == 33:
                assert g.num_bricks() > 0  # read-out in the middle joins both streams
        for x, y in zip(g.export_voxels(), ref):
            assert np.array_equal(x, y), (mb, pipe)
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    orgs = np.stack([org for _, org in scans])
    g = hip(max_batch=7, pipeline=True)
    for lo, hi in ((0, 20), (20, 21), (21, 70)):  # several calls, each several batches
        g.integrate_batch_device(d.data_ptr() + 12 * int(offs[lo]),
                                 (offs[lo:hi + 1] - offs[lo]).astype(np.uint64), orgs[lo:hi])
    for x, y in zip(g.export_voxels(), ref):
        assert np.array_equal(x, y)


def test_queued_scans_flush_before_readout(sim):
    """A query right after queued host scans sees them (the queue is flushed first)."""
    p, org = sim.scan(0)
    g = hip(max_batch=32)
    g.integrate(decimate(p, 4), org)
    assert g.num_bricks() > 0
    assert g.stats()["n_scans"] == 1


def test_golden_fixture(tmp_path):
    from conftest import GOLDEN
    import os
    z = np.load(os.path.join(GOLDEN, "golden_c1_decimated.npz"), allow_pickle=False)
    g = hip(voxel_size=float(z["voxel_size"]), sdf_trunc=float(z["sdf_trunc"]), semantics="vdbfusion")
    offs = z["scan_offsets"]
    for s in range(len(offs) - 1):
        g.integrate(z["points"][offs[s]:offs[s + 1]], z["origins"][s])
    i, s_, w = g.export_voxels()
    assert np.array_equal(i, z["ijk"])
    assert np.array_equal(w, z["weight"])
    assert np.array_equal(s_.view(np.uint32), z["sdf"].view(np.uint32))


def test_permutation_invariance_bitwise(scan0):
    pts, org = scan0
    perm = np.random.default_rng(11).permutation(pts.shape[0])
    a, b = hip(), hip()
    a.integrate(pts, org)
    b.integrate(pts[perm], org)
    for x, y in zip(a.export_voxels(), b.export_voxels()):
        assert np.array_equal(x, y)


def test_repeatability_bitwise(scan0):
    a, b = hip(), hip()
    for v in (a, b):
        v.integrate(*scan0)
    for x, y in zip(a.export_bricks(), b.export_bricks()):
        assert np.array_equal(x, y)


def test_c4_dense_2048_2cm():
    """C4 as configured: full OS-1-128 2048-column scans (262,144 points each), 2 cm voxels, 6 cm
    truncation, 20 Hz trajectory, two consecutive scans."""
    from tsdf_map.scan_gen import OusterSim
    sim4 = OusterSim("os1_128_2048", hz=20.0)
    scans = [sim4.scan(0), sim4.scan(1)]
    assert scans[0][0].shape[0] == 128 * 2048
    g, o = run_both(scans, voxel_size=0.02, sdf_trunc=0.06, max_points=1 << 19,
                    max_bricks=1 << 21)
    assert assert_bitwise(g, o) > 2_000_000


def test_long_runs_unpacked_cells(scan0):
    """(brick, scan) runs longer than the packed-cell limit (count carried in the int64 sum:
    n tau 2^32 < 2^43) take the two-atomic path: 20000 returns on one point per scan, mixed with
    ordinary scans in the same windows, and a 2 m truncation where the limit is ~1000."""
    pts, org = scan0
    hot = np.tile(np.array([[4.0, 1.0, 0.3]], np.float32), (20000, 1))
    for tau in (TAU, 2.0):
        scans = [(decimate(pts, 8), org), (np.concatenate([decimate(pts, 16), hot]), org),
                 (hot[:3000] + np.float32(0.01), org)]
        g, o = run_both(scans, sdf_trunc=tau)
        assert assert_bitwise(g, o) > 0


def test_c3_10cm(scan0):
    """C3 voxel size: 10 cm, 30 cm truncation."""
    g, o = run_both([(decimate(scan0[0], 4), scan0[1])], voxel_size=0.10, sdf_trunc=0.30)
    assert_bitwise(g, o)


def test_space_carving_bitwise(scan0):
    pts, org = scan0
    g, o = run_both([(decimate(pts, 64), org)], space_carving=True, max_range=60.0)
    assert_bitwise(g, o)


def test_range_filter_and_degenerate_points():
    pts = np.array([[0, 0, 0], [0.5, 0, 0], [40, 0, 0], [np.nan, 1, 1], [np.inf, 0, 0],
                    [5.01, 0.01, 0.02], [-3.0, 4.0, -1.0]], np.float32)
    g, o = run_both([(pts, np.zeros(3))], min_range=1.0, max_range=30.0)
    assert assert_bitwise(g, o) > 0
    assert g.stats()["n_rays_total"] == 2


def test_empty_and_zero_scans():
    g = hip()
    g.integrate(np.zeros((0, 3), np.float32), np.zeros(3))
    g.integrate(np.zeros((1000, 3), np.float32), np.zeros(3))  # all r = 0 returns
    g.sync()
    assert g.num_bricks() == 0
    assert g.export_voxels()[0].shape == (0, 3)


def test_negative_and_far_coordinates(scan0):
    """Origins far from zero and in the negative octant (brick key packing, floor of negatives)."""
    pts, org = scan0
    sub = decimate(pts, 8)
    shift = np.array([-12345.6, 5432.1, -77.7])
    g, o = run_both([((sub + shift).astype(np.float32), org + shift)])
    assert_bitwise(g, o)


def test_pointcloud2_layouts(scan0):
    """dlio::Point records (point_step 32, xyz at 0, dlio.h:85-106) and float64 xyz."""
    pts, org = scan0
    sub = decimate(pts, 8)
    rec = np.zeros(sub.shape[0], dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("pad", "<f4"),
                                         ("intensity", "<f4"), ("pad2", "<f4"), ("t", "<u4"),
                                         ("pad3", "<u4")])
    assert rec.dtype.itemsize == 32
    rec["x"], rec["y"], rec["z"] = sub[:, 0], sub[:, 1], sub[:, 2]
    a, b, c = hip(), hip(), hip()
    a.integrate(sub, org)
    b.integrate_cloud(rec.tobytes(), rec.shape[0], 32, 0, org)
    c.integrate(sub.astype(np.float64), org)
    ra = a.export_voxels()
    for v in (b, c):
        for x, y in zip(ra, v.export_voxels()):
            assert np.array_equal(x, y)


def test_device_resident_batch_matches_host_path(sim):
    import torch
    scans = [sim.scan(k) for k in range(3)]
    a = hip()
    for p, o in scans:
        a.integrate(p, o)
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    org = np.stack([o for _, o in scans])
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    b = hip()
    b.integrate_batch_device(d.data_ptr(), offs, org)
    b.sync()
    for x, y in zip(a.export_bricks(), b.export_bricks()):
        assert np.array_equal(x, y)


def test_query_dense_matches_oracle(scan0):
    g, o = run_both([(decimate(scan0[0], 4), scan0[1])])
    ijk, _, _ = o.export_voxels()
    lo = ijk[len(ijk) // 2] - np.array([32, 24, 12])  # a box around an observed voxel
    hi = lo + np.array([64, 48, 24])
    gs, gw = g.query_dense(lo, hi)
    os_, ow = o.query_dense(lo, hi)
    assert np.count_nonzero(gw) > 0
    assert np.array_equal(gw, ow)
    assert np.array_equal(gs.view(np.uint32), os_.view(np.uint32))


def test_export_import_roundtrip(scan0, tmp_path):
    a = hip()
    a.integrate(*scan0)
    path = str(tmp_path / "map.npz")
    a.save(path)
    b = hip()
    b.load(path)
    for x, y in zip(a.export_bricks(), b.export_bricks()):
        assert np.array_equal(x, y)


def test_sector_shards_merge_to_single_gpu_field(scan0):
    """Azimuth-sector sharding: per-sector partial fields merged by weighted mean equal the
    single-volume field — weights exact, sdf within 1e-5 m, non-border voxels bit-exact."""
    from tsdf_map import select_sector
    pts, org = scan0
    ref = hip()
    ref.integrate(pts, org)
    parts = []
    for s in range(4):
        v = hip()
        v.integrate(select_sector(pts, org, s, 4), org)
        parts.append(v)
    merged = hip()
    for v in parts:
        merged.import_bricks(*v.export_bricks())
    ri, rs, rw = ref.export_voxels()
    mi, ms, mw = merged.export_voxels()
    assert np.array_equal(ri, mi) and np.array_equal(rw, mw)
    assert np.max(np.abs(rs - ms)) <= 1e-5
    # voxels observed by one sector only are copied, hence bit-exact
    keys = [set(map(tuple, v.export_voxels()[0].tolist())) for v in parts]
    count = {}
    for k in keys:
        for t in k:
            count[t] = count.get(t, 0) + 1
    single = np.array([count[tuple(t)] == 1 for t in mi.tolist()])
    assert single.sum() > 0.5 * len(single)
    assert np.array_equal(rs[single].view(np.uint32), ms[single].view(np.uint32))


def test_pool_exhaustion_reports_enomem(scan0):
    from tsdf_map import TsdfError
    from tsdf_map import _abi
    g = hip(max_bricks=64, max_bricks_hard=64)  # fixed capacity: no growth
    g.integrate(*scan0)
    with pytest.raises(TsdfError) as e:
        g.sync()
    assert e.value.code == _abi.TSDF_ENOMEM
    g.sync()  # the flag is reported once
    assert g.num_bricks() == 64


def test_oversized_scan_rejected():
    from tsdf_map import TsdfError
    g = hip(max_points=1000)
    with pytest.raises(TsdfError):
        g.integrate(np.ones((1001, 3), np.float32), np.zeros(3))
