"""Capacity growth with batch replay (SURVEY §5 failure row): a context that starts
with a brick pool far too small grows its pool / hash table / work lists when a batch overflows and
re-runs the batches from the failed one, so the field ends BIT-EXACT to the oracle's and no
TSDF_ENOMEM is raised.  A fixed capacity (max_bricks_hard == max_bricks) keeps the old contract
(tests/test_gpu_parity.py::test_pool_exhaustion_reports_enomem)."""
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
    kw.pop("max_batch", None)
    kw.pop("pipeline", None)
    return oracle.OracleTSDFVolume(kw.pop("voxel_size", VS), kw.pop("sdf_trunc", TAU), **kw)


def bitwise(g, o):
    gi, gs, gw = g.export_voxels()
    oi, os_, ow = o.export_voxels()
    return (gi.shape == oi.shape and np.array_equal(gi, oi) and np.array_equal(gw, ow)
            and np.array_equal(gs.view(np.uint32), os_.view(np.uint32)))


def test_full_c1_scan_from_64_bricks(scan0):
    g = hip(max_bricks=64)
    g.integrate(*scan0)
    g.sync()  # no TSDF_ENOMEM
    o = ora()
    o.integrate(*scan0)
    assert bitwise(g, o)
    st = g.stats()
    assert st["n_grows"] >= 1 and st["n_replayed"] >= 1
    assert st["n_bricks"] == o.num_bricks() <= st["max_bricks"]
    assert st["n_rays_total"] == scan0[0].shape[0]  # replayed batches are counted once


@pytest.mark.parametrize("pipeline", [False, True, 2])
@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion", "voxblox"])
def test_host_path_sequence_grows(sim, pipeline, semantics):
    """Host-pointer scans in 2-scan batches: the staging checkpoint replays before overwriting."""
    kw = dict(max_bricks=128, max_batch=2, pipeline=pipeline, semantics=semantics)
    if semantics == "voxblox":
        kw.update(max_range=40.0)
    g, o = hip(**kw), ora(**kw)
    for k in (0, 1, 2, 3, 10, 20, 30):
        pts, org = sim.scan(k)
        pts = decimate(pts, 4)
        g.integrate(pts, org)
        o.integrate(pts, org)
    g.sync()
    assert bitwise(g, o)
    assert g.stats()["n_grows"] >= 2


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion"])
def test_device_batches_grow(sim, semantics):
    import torch
    scans = [sim.scan(k) for k in (0, 5, 9, 14, 22)]
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    org = np.stack([o for _, o in scans])
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    g = hip(max_bricks=1000, max_batch=2, semantics=semantics)
    g.integrate_batch_device(d.data_ptr(), offs, org)
    g.sync()
    o = ora(semantics=semantics)
    for p, q in scans:
        o.integrate(p, q)
    assert bitwise(g, o)
    assert g.stats()["n_grows"] >= 1


def test_growth_respects_hard_limit(scan0):
    from tsdf_map import TsdfError, _abi
    g = hip(max_bricks=64, max_bricks_hard=4096)
    g.integrate(*scan0)
    with pytest.raises(TsdfError) as e:
        g.sync()
    assert e.value.code == _abi.TSDF_ENOMEM
    st = g.stats()
    assert st["max_bricks"] == 4096 and st["n_bricks"] == 4096
    g.sync()  # reported once; the context stays usable
    g.integrate(decimate(scan0[0], 64), scan0[1])
    with pytest.raises(TsdfError):
        g.sync()


def test_import_grows(scan0):
    a = hip()
    a.integrate(*scan0)
    b = hip(max_bricks=16)
    b.import_bricks(*a.export_bricks())
    for x, y in zip(a.export_bricks(), b.export_bricks()):
        assert np.array_equal(x, y)


def test_large_batches_bitwise(sim):
    """Batches of up to 512 scans (the sector-sharded multi-GPU step is one batch): a 130-scan
    device batch is one launch, bit-exact to the oracle."""
    import torch
    scans = [(decimate(p, 16), o) for p, o in (sim.scan(k) for k in range(130))]
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    org = np.stack([o for _, o in scans])
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    g = hip(max_batch=512)
    g.integrate_batch_device(d.data_ptr(), offs, org)
    g.sync()
    assert g.stats()["n_batches"] == 1
    o = ora()
    for p, q in scans:
        o.integrate(p, q)
    assert bitwise(g, o)


@pytest.mark.parametrize("walk", ["two", "single"])
def test_sector_sample_list_grows(sim, walk):
    """A sharded context sizes its sample list (single walk: its k_walk regions) for 1 / n_sectors
    of the rays; scans whose points all lie in its world-frame sector (the world rule: an
    index-rule context takes 1 / n_sectors of every cloud by construction) overflow it, and it
    grows (OVF_SMP) without losing an update."""
    import torch
    from tsdf_map import sector_ids
    # two walks: 819 k sample slots for 8 x 2^15 points; single walk: 1184 regions of 512 rays for
    # 64 x 2^15 points, while the 64 scans' sector-0 points fill ~2200 of them
    n, kw = (6, dict(max_batch=8, max_points=1 << 15)) if walk == "two" else \
        (64, dict(max_batch=64, max_points=1 << 15))
    scans = []
    for k in range(n):
        p, o = sim.scan(k)
        p = p[sector_ids(p, o, 8, 0.0) == 0]
        scans.append((np.ascontiguousarray(p), o))
    allp = np.concatenate([p for p, _ in scans])
    offs = np.cumsum([0] + [p.shape[0] for p, _ in scans]).astype(np.uint64)
    org = np.stack([o for _, o in scans])
    d = torch.from_numpy(allp).to("cuda:0")
    torch.cuda.synchronize()
    g = hip(n_sectors=8, sector=0, walk=walk, sector_rule="world", **kw)
    g.integrate_batch_device(d.data_ptr(), offs, org)
    g.sync()
    assert g.stats()["n_grows"] >= 1
    o = ora(n_sectors=8, sector=0, sector_rule="world")
    for p, q in scans:
        o.integrate(p, q)
    assert bitwise(g, o)


@pytest.mark.parametrize("pipeline", [False, True, 2])
def test_metrics_drain_replay_keeps_staged_input(sim, tmp_path, pipeline):
    """the metrics-ring drain inside a launch can run a capacity replay while a host
    batch is already staged.  Hundreds of 1-scan batches with the metrics log on and a pool that
    keeps growing put overflows into that window; the field must still be the oracle's, bit for bit
    (each pending batch reads its own staging buffer, whatever the batch parity after a replay)."""
    g = hip(max_bricks=16, max_batch=1, pipeline=pipeline)
    g.set_metrics_log(tmp_path / "m.jsonl")
    o = ora()
    for k in range(600):
        pts, org = sim.scan(k % 300)
        pts = np.ascontiguousarray(pts[(k * 7) % 64::64])
        g.integrate(pts, org)
        o.integrate(pts, org)
    g.sync()
    st = g.stats()
    assert st["n_grows"] >= 3 and st["n_replayed"] >= 1
    assert bitwise(g, o)


def test_device_scans_queue_and_free_the_buffer(sim):
    """tsdf_integrate_device copies the scan into the pending batch before returning (ABI v6): the
    caller overwrites its buffer right after each call, and the field is still the oracle's."""
    import torch
    g = hip(max_bricks=64, max_batch=4)
    o = ora()
    buf = torch.empty((1 << 16, 3), dtype=torch.float32, device="cuda")
    for k in range(10):
        pts, org = sim.scan(k)
        pts = decimate(pts, 8)
        buf[:pts.shape[0]] = torch.from_numpy(pts).cuda()
        g.integrate_device(buf.data_ptr(), pts.shape[0], org)
        buf.fill_(1e9)  # the caller's buffer is free once the call returned
        o.integrate(pts, org)
    g.sync()
    assert bitwise(g, o)
    assert g.stats()["n_batches"] <= 4  # queued: 10 scans in batches of 4
