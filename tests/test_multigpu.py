"""The multi-GPU path on one MI355X: azimuth-sector filtering inside the walk kernels and the
device-resident border-brick reduce, against the oracle running the same ABI.

* sector filter: a context with n_sectors/sector integrates exactly the oracle's sector rays,
  bit for bit;
* border reduce, one process: the collective is emulated (all-gather = stack, all-to-all =
  slicing) over 3 GPU contexts and over 3 oracle contexts; after the reduce every GPU rank's field
  equals its oracle twin BIT FOR BIT, and the union equals the single-volume field (weights exact,
  |dSDF| <= 1e-5 m: fp32 weighted means of partial fields);
* border reduce, two processes: tsdf_map.distributed.border_reduce itself, gloo ranks sharing the
  GPU (tiles staged through host memory; RCCL needs one GPU per rank).
"""
import os
import socket

import numpy as np
import pytest
import torch

import oracle
from conftest import REPO

pytestmark = pytest.mark.gpu

VS, TAU = 0.05, 0.15
TILE = 1028


def hip(**kw):
    from tsdf_map import HipTSDFVolume
    return HipTSDFVolume(VS, TAU, **kw)


def ora(**kw):
    return oracle.OracleTSDFVolume(VS, TAU, **kw)


def voxels_equal_bitwise(a, b):
    ai, as_, aw = a
    bi, bs, bw = b
    return (ai.shape == bi.shape and np.array_equal(ai, bi) and np.array_equal(aw, bw)
            and np.array_equal(as_.view(np.uint32), bs.view(np.uint32)))


@pytest.mark.parametrize("n,yaw0,rule", [(4, 0.0, "world"), (3, 0.7, "world"), (4, 0.0, "index"),
                                         (3, 0.7, "index")])
def test_sector_filter_bitwise(sim, n, yaw0, rule):
    """Each sector context against its oracle twin, bit for bit, and the sectors partition the
    rays -- the world-frame azimuth filter in the walk kernels, and (ABI v10) the index rule's
    contiguous share of every cloud."""
    scans = [sim.scan(k) for k in (0, 5)]
    rays = 0
    for k in range(n):
        g = hip(n_sectors=n, sector=k, sector_yaw0=yaw0, sector_rule=rule)
        o = ora(n_sectors=n, sector=k, sector_yaw0=yaw0, sector_rule=rule)
        for pts, org in scans:
            g.integrate(pts, org)
            o.integrate(pts, org)
        g.sync()
        assert voxels_equal_bitwise(g.export_voxels(), o.export_voxels())
        rays += g.stats()["n_rays_total"]
    assert rays == sum(p.shape[0] for p, _ in scans)


def emulated_reduce(vols, dev):
    """border_reduce's four steps for all ranks of one process (the collective emulated)."""
    world = len(vols)
    keys, counts = [], []
    for v in vols:
        k = torch.empty(max(v.num_bricks(), 1), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        counts.append(v.brick_keys_into(k.data_ptr(), k.numel()))
        keys.append(k)
    stride = max(counts)
    allk = torch.full((world, stride), -1, dtype=torch.int64, device=dev)
    for r in range(world):
        allk[r, :counts[r]] = keys[r][:counts[r]]
    sends, splits = [], []
    for r, v in enumerate(vols):
        s = torch.empty((max(counts[r], 1), TILE), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        sc = v.border_pack(allk.data_ptr(), counts, stride, world, r, s.data_ptr(), s.shape[0])
        sends.append(s)
        splits.append(sc)
    for d, v in enumerate(vols):  # rank d receives block d of every source, sources ascending
        parts, rc = [], []
        for r in range(world):
            off = sum(splits[r][:d])
            parts.append(sends[r][off:off + splits[r][d]])
            rc.append(splits[r][d])
        recv = torch.cat(parts).contiguous() if sum(rc) else torch.empty((1, TILE), dtype=torch.int32,
                                                                          device=dev)
        torch.cuda.synchronize()
        v.border_merge(recv.data_ptr(), rc)
    for v in vols:  # every rank merged: commit (ABI v9)
        v.border_commit(True)
    return splits


def emulated_reduce_host(vols):
    """The same on host buffers for oracle contexts (numpy pointers)."""
    world = len(vols)
    keys = [np.empty(max(v.num_bricks(), 1), np.int64) for v in vols]
    counts = [v.brick_keys_into(k.ctypes.data, k.size) for v, k in zip(vols, keys)]
    stride = max(counts)
    allk = np.full((world, stride), -1, np.int64)
    for r in range(world):
        allk[r, :counts[r]] = keys[r][:counts[r]]
    sends, splits = [], []
    for r, v in enumerate(vols):
        s = np.empty((max(counts[r], 1), TILE), np.int32)
        splits.append(v.border_pack(allk.ctypes.data, counts, stride, world, r, s.ctypes.data,
                                    s.shape[0]))
        sends.append(s)
    for d, v in enumerate(vols):
        parts, rc = [], []
        for r in range(world):
            off = sum(splits[r][:d])
            parts.append(sends[r][off:off + splits[r][d]])
            rc.append(splits[r][d])
        recv = np.ascontiguousarray(np.concatenate(parts)) if sum(rc) else np.empty((1, TILE), np.int32)
        v.border_merge(recv.ctypes.data, rc)
    for v in vols:  # every rank merged: commit (ABI v9)
        v.border_commit(True)
    return splits


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion"])
def test_border_reduce_matches_oracle_bitwise(sim, semantics):
    from tsdf_map import bricks_to_voxels
    world, yaw0 = 3, 0.25
    dev = torch.device("cuda", 0)
    g = [hip(n_sectors=world, sector=r, sector_yaw0=yaw0, semantics=semantics) for r in range(world)]
    o = [ora(n_sectors=world, sector=r, sector_yaw0=yaw0, semantics=semantics) for r in range(world)]
    ref = ora(semantics=semantics)
    rounds = [(0, 1), (2, 40)]
    for i, ks in enumerate(rounds):
        for k in ks:
            pts, org = sim.scan(k)
            pts = np.ascontiguousarray(pts[::2])
            for v in g + o + [ref]:
                v.integrate(pts, org)
        gs = emulated_reduce(g, dev)
        os_ = emulated_reduce_host(o)
        assert sum(map(sum, gs)) > 100  # border bricks exist
        for r in range(world):
            assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), (i, r)
    # the union of the ranks' fields is the single-volume field
    parts = [v.export_bricks() for v in g]
    keep = [(w.reshape(len(c), -1) > 0).any(1) for c, _, w in parts]
    coords = np.concatenate([c[k] for (c, _, _), k in zip(parts, keep)])
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]  # each brick once
    mi, ms, mw = bricks_to_voxels(coords, np.concatenate([s[k] for (_, s, _), k in zip(parts, keep)]),
                                  np.concatenate([w[k] for (_, _, w), k in zip(parts, keep)]))
    ri, rs, rw = ref.export_voxels()
    assert np.array_equal(mi, ri) and np.array_equal(mw, rw)
    assert np.max(np.abs(ms - rs)) <= 1e-5


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion"])
def test_sharded_contexts_local_reduce_bitwise(sim, semantics):
    """tsdf_create_sharded + tsdf_integrate_sectors + tsdf_border_reduce_local: one process
    driving n sector contexts (here all on GPU 0; on a node, one per GPU, tiles between GPUs by
    peer copy) gives every context the oracle's reduced field bit for bit, twice over."""
    from tsdf_map import HipTSDFVolume, border_reduce_local, integrate_sectors
    world, yaw0 = 4, 0.6
    g = HipTSDFVolume.sharded(world, VS, TAU, device_ids=[0] * world, sector_yaw0=yaw0,
                              max_bricks=1 << 18, max_batch=4, semantics=semantics)
    assert [v.params.sector for v in g] == list(range(world))
    assert all(v.params.n_sectors == world and v.params.device_id == 0 for v in g)
    o = [ora(n_sectors=world, sector=r, sector_yaw0=yaw0, semantics=semantics) for r in range(world)]
    moved = 0
    for ks in ((0, 1, 2), (30,)):
        for k in ks:
            pts, org = sim.scan(k)
            pts = np.ascontiguousarray(pts[::2])
            integrate_sectors(g, pts, org)
            for v in o:
                v.integrate(pts, org)
        moved += border_reduce_local(g)
        splits = emulated_reduce_host(o)
        assert sum(map(sum, splits)) > 100
        for r in range(world):
            assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), (ks, r)
    assert moved > 100
    for v in g:
        v.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    for p in (os.path.join(REPO, "noetic-slam_amd"), os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from tsdf_map import HipTSDFVolume
    from tsdf_map.distributed import merged_bricks
    from tsdf_map.scan_gen import OusterSim

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sim = OusterSim()
    vol = HipTSDFVolume(VS, TAU, n_sectors=world, sector=rank, device_id=0)
    for k in (0, 3):
        vol.integrate(*sim.scan(k))
    c, s, w = merged_bricks(vol, device="cpu")
    # the sharded mesh over the collective (halo tiles through host memory here; RCCL on a node)
    from tsdf_map.distributed import mesh
    mv, _ = mesh(vol, comm_device="cpu", reduce=False)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), coords=c, sdf=s, weight=w, mesh=mv)
    dist.barrier()
    dist.destroy_process_group()


def test_border_reduce_two_processes(tmp_path, sim):
    import torch.multiprocessing as mp
    from tsdf_map import bricks_to_voxels
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    parts = [np.load(str(tmp_path / ("rank%d.npz" % r))) for r in range(world)]
    coords = np.concatenate([p["coords"] for p in parts])
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]
    mi, ms, mw = bricks_to_voxels(coords, np.concatenate([p["sdf"] for p in parts]),
                                  np.concatenate([p["weight"] for p in parts]))
    ref = ora()
    for k in (0, 3):
        ref.integrate(*sim.scan(k))
    ri, rs, rw = ref.export_voxels()
    assert np.array_equal(mi, ri) and np.array_equal(mw, rw)
    assert np.max(np.abs(ms - rs)) <= 1e-5
    # the ranks' meshes together: the mesh of the union field, triangle for triangle
    from test_distributed import tri_set
    union = ora()
    for p in parts:
        union.import_bricks(p["coords"], p["sdf"], p["weight"])
    got = tri_set(np.concatenate([p["mesh"] for p in parts]))
    assert got.shape[0] > 1000
    assert np.array_equal(got, tri_set(union.extract_triangle_mesh()[0]))


def test_border_abort_restores_bitwise(sim):
    """ABI v9 on the GPU: pack, merge, then abort (tsdf_border_commit_device(0)) -- the snapshot
    kernels write the merged bricks back and the sent bricks never lost their mass: every
    context's field is the one before, bit for bit; integration is refused while the reduce is
    open and accepted after."""
    world, yaw0 = 3, 0.25
    dev = torch.device("cuda", 0)
    g = [hip(n_sectors=world, sector=r, sector_yaw0=yaw0) for r in range(world)]
    for k in (0, 1):
        pts, org = sim.scan(k)
        for v in g:
            v.integrate(np.ascontiguousarray(pts[::2]), org)
    before = [v.export_voxels() for v in g]
    keys, counts = [], []
    for v in g:
        k = torch.empty(max(v.num_bricks(), 1), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        counts.append(v.brick_keys_into(k.data_ptr(), k.numel()))
        keys.append(k)
    stride = max(counts)
    allk = torch.full((world, stride), -1, dtype=torch.int64, device=dev)
    for r in range(world):
        allk[r, :counts[r]] = keys[r][:counts[r]]
    sends, splits = [], []
    for r, v in enumerate(g):
        s_ = torch.empty((max(counts[r], 1), TILE), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        splits.append(v.border_pack(allk.data_ptr(), counts, stride, world, r, s_.data_ptr(),
                                    s_.shape[0]))
        sends.append(s_)
    assert sum(map(sum, splits)) > 100
    for d, v in enumerate(g):
        parts = [sends[r][sum(splits[r][:d]):sum(splits[r][:d]) + splits[r][d]] for r in range(world)]
        rc = [splits[r][d] for r in range(world)]
        recv = torch.cat(parts).contiguous() if sum(rc) else torch.empty((1, TILE), dtype=torch.int32,
                                                                          device=dev)
        torch.cuda.synchronize()
        v.border_merge(recv.data_ptr(), rc)
    pts, org = sim.scan(3)
    with pytest.raises(Exception, match="border reduce is open"):
        g[0].integrate(np.ascontiguousarray(pts[::2]), org)
    assert not voxels_equal_bitwise(g[0].export_voxels(), before[0])  # the owner merged
    for v in g:
        v.border_commit(False)
    for v, b in zip(g, before):
        assert voxels_equal_bitwise(v.export_voxels(), b)
    g[0].integrate(np.ascontiguousarray(pts[::2]), org)


def test_sectors_bare_origin_voxblox_depth_weight(sim):
    """integrate_sectors with a bare (3,) origin takes
    tsdf_integrate_sectors_origin -- no orientation, so Voxblox's constant weight, exactly what
    integrate(points, origin) gives -- bit for bit against the oracle's sector volumes."""
    from tsdf_map import integrate_sectors
    n, yaw0 = 3, 0.5
    kw = dict(semantics="voxblox", use_const_weight=False, max_range=100.0)
    g = [hip(n_sectors=n, sector=r, sector_yaw0=yaw0, max_batch=2, **kw) for r in range(n)]
    o = [ora(n_sectors=n, sector=r, sector_yaw0=yaw0, **kw) for r in range(n)]
    for k in (0, 4):
        pts, org = sim.scan(k)
        pts = np.ascontiguousarray(pts[::2])
        integrate_sectors(g, pts, org)
        for v in o:
            v.integrate(pts, org)
    for r in range(n):
        g[r].sync()
        assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), r


@pytest.mark.parametrize("n,f64,mode,rule", [(3, False, "split", "world"), (4, True, "split", "world"),
                                              (8, False, "split", "world"),
                                              (3, False, "fanout", "world"),
                                              (4, True, "fanout", "world"), (8, False, "h2d", "world"),
                                              (3, False, "fanout", "index"),
                                              (4, True, "fanout", "index"),
                                              (8, False, "fanout", "index")])
def test_integrate_sectors_bitwise(sim, n, f64, mode, rule):
    """tsdf_integrate_sectors (the live N-GPU input) equals each context integrating
    the full cloud with its in-kernel sector filter (the oracle), bit for bit, for every transfer
    (tsdf_params.sector_input): split (host classification, each context gets its sector's
    points), fanout (one H2D, device-to-device copies to the other contexts) and h2d (one H2D per
    context from one packed buffer).  With the index rule (ABI v10) every context packs and copies
    only its contiguous share of the cloud, whatever sector_input says."""
    from tsdf_map import integrate_sectors
    yaw0 = 0.4
    g = [hip(n_sectors=n, sector=r, sector_yaw0=yaw0, max_batch=2, sector_input=mode,
             sector_rule=rule) for r in range(n)]
    o = [ora(n_sectors=n, sector=r, sector_yaw0=yaw0, sector_rule=rule) for r in range(n)]
    rays = total = 0
    for k in (0, 1, 9):
        pts, org = sim.scan(k)
        pts = np.ascontiguousarray(pts[::2])
        # rays along every sector start (boundary ties) and NaN rows (no sector: dropped)
        th = yaw0 + 2 * np.pi * np.arange(n) / n
        edge = org[None, :] + np.stack([7.0 * np.cos(th), 7.0 * np.sin(th), np.zeros(n)], 1)
        pts = np.concatenate([pts, edge.astype(np.float32),
                              np.full((3, 3), np.nan, np.float32)]).astype(np.float32)
        if f64:
            pts = pts.astype(np.float64)
        q = np.array([0.0, 0.0, np.sin(0.1 * k), np.cos(0.1 * k)])
        integrate_sectors(g, pts, np.concatenate([org, q]))
        for v in o:
            v.integrate(pts, org)
        rays += pts.shape[0] - 3
        total += pts.shape[0]
    for r in range(n):
        g[r].sync()
        assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), r
    if rule == "index":  # each context received exactly its share
        assert sum(v.stats()["n_points_in"] for v in g) == total
        assert max(v.stats()["n_points_in"] for v in g) <= -(-total // n) + 3
    elif mode == "split":
        assert sum(v.stats()["n_points_in"] for v in g) == rays  # each point went to one context
    else:
        assert all(v.stats()["n_points_in"] == total for v in g)  # every context got the cloud


def test_fanout_out_of_lockstep(sim):
    """The fan-out copies a follower's pending points from the leader's staging once per batch;
    partial flushes (a read-out of the leader alone), a follower's own scan in between, and the
    leader destroyed while its followers still hold uncopied points all leave every context equal
    to its oracle twin."""
    from tsdf_map import integrate_sectors
    n, yaw0 = 3, 0.3  # (the fan-out serves the world rule)
    g = [hip(n_sectors=n, sector=r, sector_yaw0=yaw0, max_batch=3, sector_rule="world")
         for r in range(n)]
    o = [ora(n_sectors=n, sector=r, sector_yaw0=yaw0, sector_rule="world") for r in range(n)]
    scans = []
    for k in (0, 1, 2, 5, 7, 9, 11):
        pts, org = sim.scan(k)
        scans.append((np.ascontiguousarray(pts[::4]), org))

    def both(i, only=None):
        pts, org = scans[i]
        if only is None:
            integrate_sectors(g, pts, np.concatenate([org, [0.0, 0.0, 0.0, 1.0]]))
            for v in o:
                v.integrate(pts, org)
        else:
            g[only].integrate(pts, org)
            o[only].integrate(pts, org)

    both(0)
    both(1)
    g[0].sync()              # the leader flushes alone; followers keep their pending range
    both(2)
    both(3, only=1)          # a follower's own scan between fan-out scans
    both(4)
    both(5)
    ref = [v.export_voxels() for v in o]
    for r in range(n):
        g[r].sync()
        assert voxels_equal_bitwise(g[r].export_voxels(), ref[r]), r
    both(6)                  # pending everywhere, then the leader goes first
    g[0].close()
    for r in (1, 2):
        assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), r


@pytest.mark.parametrize("rule", ["world", "index"])
def test_integrate_sectors_voxblox_merged(sim, rule):
    """MergedTsdfIntegrator: with the world rule each context bundles the whole scan before its
    sector filter, so the sectors take the fan-out (a requested host split is overridden); with the
    index rule each context bundles its own share.  Every context equals its oracle twin."""
    from tsdf_map import integrate_sectors
    n, yaw0 = 3, 0.2
    kw = dict(semantics="voxblox", method="merged", use_const_weight=False, sector_rule=rule)
    g = [hip(n_sectors=n, sector=r, sector_yaw0=yaw0, max_batch=2, sector_input="split", **kw)
         for r in range(n)]
    o = [ora(n_sectors=n, sector=r, sector_yaw0=yaw0, **kw) for r in range(n)]
    for k in (0, 4):
        pts, org = sim.scan(k)
        q = np.array([0.0, 0.05 * k, 0.0, 1.0])
        integrate_sectors(g, np.ascontiguousarray(pts[::2]), np.concatenate([org, q]))
        for v in o:
            v.integrate(np.ascontiguousarray(pts[::2]), np.concatenate([org, q]))
    for r in range(n):
        g[r].sync()
        assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), r


def test_sharded_contexts_report_peer_reach():
    """tsdf_create_sharded enables peer access between distinct devices; contexts on one device
    reach each other directly (peer_mask has every bit)."""
    from tsdf_map import HipTSDFVolume
    g = HipTSDFVolume.sharded(3, VS, TAU, device_ids=[0, 0, 0], max_bricks=1 << 12, max_batch=2)
    assert all(v.stats()["peer_mask"] == 0b111 for v in g)
    for v in g:
        v.close()


@pytest.mark.parametrize("kw", [dict(), dict(semantics="vdbfusion"),
                                dict(semantics="voxblox", method="merged", use_const_weight=False),
                                dict(semantics="voxblox", use_const_weight=False),
                                dict(walk="single")])
def test_index_rule_device_batches_bitwise(sim, kw):
    """ABI v10's index rule on resident device batches (the bench's path): each sector context
    reads only its contiguous share of every scan of the batch -- shares that are not contiguous
    in the batch buffer (ScanRec.xoff) -- and equals its oracle twin bit for bit; the shares
    partition the rays.  Covers both walks' point reads and the merged pre-pass's."""
    import torch
    n = 3
    scans = [sim.scan(k) for k in (0, 3, 6, 9)]
    pts = [np.ascontiguousarray(p[::3]) for p, _ in scans]
    offs = np.cumsum([0] + [p.shape[0] for p in pts]).astype(np.uint64)
    poses = np.stack([np.concatenate([o, [0.0, 0.0, np.sin(0.1 * k), np.cos(0.1 * k)]])
                      for k, (_, o) in enumerate(scans)])
    d = torch.from_numpy(np.concatenate(pts)).to("cuda:0")
    torch.cuda.synchronize()
    rays = 0
    for r in range(n):
        g = hip(n_sectors=n, sector=r, max_batch=4, **kw)
        o = ora(n_sectors=n, sector=r, **kw)
        g.integrate_batch_device(d.data_ptr(), offs, poses)
        for p, q in zip(pts, poses):
            o.integrate(p, q)
        g.sync()
        assert voxels_equal_bitwise(g.export_voxels(), o.export_voxels()), r
        assert g.stats()["n_points_in"] == o.stats()["n_points_in"]
        rays += g.stats()["n_points_in"]
    assert rays == int(offs[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(semantics="voxblox", method="merged", use_const_weight=False)])
def test_index_rule_tiny_and_empty_shares(sim, kw):
    """The index rule with scans of fewer points than sectors: a 2-point scan (one sector's share
    empty), an empty scan and a 1-point scan between full-size ones, as one device batch over 3
    sectors -- every context equals its oracle twin bit for bit and the shares partition the
    points (empty shares give zero-length ranges, ScanRec.xoff skips them)."""
    import torch
    n = 3
    full = [np.ascontiguousarray(sim.scan(k)[0][::5]) for k in (1, 4)]
    orgs = [sim.scan(k)[1] for k in (1, 2, 3, 4, 5)]
    pts = [full[0], full[0][100:102].copy(), np.zeros((0, 3), np.float32), full[1][7:8].copy(),
           full[1]]
    offs = np.cumsum([0] + [p.shape[0] for p in pts]).astype(np.uint64)
    poses = np.stack([np.concatenate([o, [0.0, 0.0, np.sin(0.2 * k), np.cos(0.2 * k)]])
                      for k, o in enumerate(orgs)])
    d = torch.from_numpy(np.concatenate(pts)).to("cuda:0")
    torch.cuda.synchronize()
    got = 0
    for r in range(n):
        g = hip(n_sectors=n, sector=r, max_batch=8, **kw)
        o = ora(n_sectors=n, sector=r, **kw)
        g.integrate_batch_device(d.data_ptr(), offs, poses)
        for p, q in zip(pts, poses):
            o.integrate(p, q)
        g.sync()
        assert voxels_equal_bitwise(g.export_voxels(), o.export_voxels()), r
        assert g.stats()["n_points_in"] == o.stats()["n_points_in"]
        got += g.stats()["n_points_in"]
    assert got == int(offs[-1])
