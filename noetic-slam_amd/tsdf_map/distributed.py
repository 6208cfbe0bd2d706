"""Multi-GPU border-brick reduce and mesh of azimuth-sector partial fields (SURVEY
§8e).

Integration shards each scan by azimuth sector (one sector per rank, one process per GPU; the
sector filter runs inside the walk kernels, tsdf_params.n_sectors/sector) and needs no collective:
VDBFusion's fused field is the weighted mean sum(w s) / sum(w) of all samples, so per-rank
partial fields combine exactly up to fp32 rounding.  A brick touched by rays of several sectors is
held by several ranks; `border_reduce` moves each such brick's mass to its owner, the lowest rank
holding it, entirely device-resident:

  1. all_gather of the brick keys (tsdf_brick_keys_device; ~8 B per brick);
  2. every rank packs its bricks owned by a lower rank into 4 KiB tiles, grouped by owner
     (tsdf_border_pack_device: kernels look the lower ranks' keys up in the rank's own hash
     table); the bricks keep their mass for now;
  3. ONE all_to_all_single of the tiles — RCCL over xGMI: point-to-point, so a direct all-to-all
     of the few-percent border set instead of a ring all-reduce of whole grids;
  4. the owner merges the received tiles, sources in ascending rank order
     (tsdf_border_merge_device: weighted mean, copy where W == 0; the touched bricks are
     snapshot first);
  5. the ranks agree (an all-reduce of their status) and commit -- the sent bricks are reset --
     or, if any rank failed anywhere, abort -- the merged bricks are restored -- so a failed
     reduce leaves every rank's field exactly as it was (tsdf_border_commit_device, ABI v9).

Every local step runs inside a try and every rank reaches the same collectives: a rank that
fails reports it at the next status vote instead of leaving the others blocked in a collective.

Afterwards the field is partitioned: every brick's full mass sits on exactly one rank, and
integration may continue (a later reduce moves only the new partial mass).  `mesh` then meshes
the partitioned field with a one-brick halo exchanged the same way (tsdf_halo_keys_device /
tsdf_halo_pack_device / tsdf_extract_mesh_halo): each rank meshes its own cubes, and the union of
the ranks' soups is the mesh of the union field.  The same code drives a CPU library (the oracle,
gloo) through the same ABI: `vol.tensor_device` says where the library's buffers live,
`comm_device` where the collective's do (they differ only in the one-GPU gloo rehearsal, which
stages the tiles through host memory).
"""
import time

import numpy as np

TILE_WORDS = 1028  # include/tsdf_hip.h TSDF_TILE_WORDS


class BorderReduceAborted(RuntimeError):
    """Another rank failed during the reduce; this rank rolled back (its field is unchanged)."""


class BorderReduceFatal(RuntimeError):
    """The reduce cannot end consistently: a collective raised on this rank (the process group
    must be taken as broken -- the other ranks may still wait in it until its timeout; this rank
    rolled back, its field is unchanged), or the commit failed here after every rank voted to
    commit (the peers committed: this rank's sent bricks still hold mass their owners now hold
    too, so the fields are inconsistent across ranks)."""


def _all_ok(ok, group, cdev):
    """Every rank's local status, agreed by an all-reduce (MIN)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def border_reduce(vol, group=None, comm_device=None, _fault=None):
    """Reduce the border bricks of this rank's `vol` with the other ranks of `group`.

    Returns {"bricks_sent", "bricks_received", "tile_bytes", "ms": {"keys", "pack", "exchange",
    "merge"}} for this rank (wall time of each step; "exchange" is the tile all-to-all).  On any
    rank's failure every rank rolls back and raises (BorderReduceAborted on the healthy ranks).
    `_fault` (tests): a step name ("keys", "pack", "exchange", "recv", "merge", "commit") at
    which this rank fails ("commit": its first commit attempts fail)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return {"bricks_sent": 0, "bricks_received": 0, "tile_bytes": 0}
    vdev = torch.device(vol.tensor_device)
    cdev = torch.device(comm_device) if comm_device is not None else vdev
    on_gpu = vdev.type == "cuda"

    def ready():  # torch's stream vs the library's: the ABI wants ready buffers
        if on_gpu:
            torch.cuda.synchronize(vdev)

    def fault(step):
        if _fault == step:
            raise RuntimeError("injected fault at %s on rank %d" % (step, rank))

    ms = {}
    t = time.perf_counter()

    def lap(name):
        nonlocal t
        now = time.perf_counter()
        ms[name] = round((now - t) * 1e3, 3)
        t = now

    err = None

    def guarded(fn):
        nonlocal err
        if err is not None:
            return None
        try:
            return fn()
        except Exception as e:  # reported at the next vote, re-raised after the roll-back
            err = e
            return None

    def vote_or_abort(opened):
        """All ranks healthy?  Otherwise roll this rank back and raise."""
        if _all_ok(err is None, group, cdev):
            return
        if opened:
            vol.border_commit(False)
        if err is not None:
            raise err
        raise BorderReduceAborted("border reduce aborted: another rank failed")

    # 1. keys
    def keys_step():
        fault("keys")
        n = vol.num_bricks()
        keys = torch.empty(max(n, 1), dtype=torch.int64, device=vdev)
        ready()
        return keys, vol.brick_keys_into(keys.data_ptr(), keys.numel())

    got = guarded(keys_step)
    vote_or_abort(False)
    keys, n = got
    cnt = torch.tensor([n], dtype=torch.int64, device=cdev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)  # (no transaction is open yet: nothing to undo)
    counts = [int(c.item()) for c in counts]
    stride = max(1, max(counts))

    def keys_stage():
        mine = torch.full((stride,), -1, dtype=torch.int64, device=cdev)
        mine[:n] = keys[:n].to(cdev)
        return mine

    mine = guarded(keys_stage)
    vote_or_abort(False)
    allk = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allk, mine, group=group)
    allk = guarded(lambda: torch.stack(allk).to(vdev).contiguous())
    vote_or_abort(False)
    lap("keys")

    # 2. pack the bricks owned elsewhere (rows grouped by destination rank); they keep their mass
    def pack_step():
        send = torch.empty((max(n, 1), TILE_WORDS), dtype=torch.int32, device=vdev)
        ready()
        sc = vol.border_pack(allk.data_ptr(), counts, stride, world, rank, send.data_ptr(),
                             send.shape[0])
        fault("pack")
        return send, sc

    got = guarded(pack_step)
    vote_or_abort(True)
    send, send_counts = got
    lap("pack")

    def collective(fn):
        """A collective every rank reaches; if it raises here, the group's state is unknown (the
        peers may be inside it): roll back and report the group broken."""
        try:
            return fn()
        except Exception as e:
            vol.border_commit(False)
            raise BorderReduceFatal("border reduce: a collective failed on rank %d (%s: %s); "
                                    "the process group must be re-created" %
                                    (rank, type(e).__name__, e)) from e

    # 3. one all-to-all of the tiles.  The local work around it (the count and tile buffers on the
    # collective's device, the received tiles back on the library's) runs guarded, with a vote
    # before each collective, so a local failure never leaves a peer alone in a collective.
    n_send = sum(send_counts)

    def exchange_prep():
        fault("exchange")
        return (torch.tensor(send_counts, dtype=torch.int64, device=cdev),
                send[:n_send].to(cdev).contiguous())

    got = guarded(exchange_prep)
    vote_or_abort(True)
    sc, send_c = got
    rc = torch.empty_like(sc)
    collective(lambda: dist.all_to_all_single(rc, sc, group=group))
    recv_counts = [int(x) for x in rc.tolist()]
    n_recv = sum(recv_counts)

    def recv_alloc():
        fault("recv")
        return torch.empty((max(n_recv, 1), TILE_WORDS), dtype=torch.int32, device=cdev)

    recv = guarded(recv_alloc)
    vote_or_abort(True)
    collective(lambda: dist.all_to_all_single(recv[:n_recv], send_c,
                                              output_split_sizes=recv_counts,
                                              input_split_sizes=send_counts, group=group))
    lap("exchange")

    # 4. merge on the owner, sources in ascending rank order (snapshot first)
    def merge_step():
        fault("merge")
        r = recv.to(vdev).contiguous()
        ready()
        vol.border_merge(r.data_ptr(), recv_counts)

    guarded(merge_step)
    # 5. commit only when every rank merged; else every rank restores
    vote_or_abort(True)
    # every rank voted to commit: a failure here cannot be rolled back (the peers commit), so the
    # commit is retried a bounded number of times before the fields are declared inconsistent
    last = None
    for attempt in range(3):
        try:
            if _fault == "commit" and attempt < 2:
                raise RuntimeError("injected fault at commit (attempt %d) on rank %d" % (attempt, rank))
            vol.border_commit(True)
            last = None
            break
        except Exception as e:
            last = e
    if last is not None:
        raise BorderReduceFatal("border reduce: rank %d could not commit after every rank voted "
                                "to (%s); its sent bricks' mass is now double-counted across "
                                "ranks" % (rank, last)) from last
    lap("merge")
    return {"bricks_sent": n_send, "bricks_received": n_recv,
            "tile_bytes": 4 * TILE_WORDS * (n_send + n_recv), "ms": ms}


def merged_bricks(vol, group=None, device=None):
    """Border-reduce, then return this rank's share of the merged map: (coords (n,3) int32,
    sdf (n,8,8,8), weight) — the bricks holding observed voxels here.  The union over ranks is
    the full map with every brick exactly once."""
    border_reduce(vol, group, comm_device=device)
    coords, S, W = vol.export_bricks()
    keep = (np.asarray(W).reshape(len(coords), -1) > 0).any(axis=1)
    return coords[keep], S[keep], W[keep]


def mesh(vol, group=None, comm_device=None, min_weight=0.0, table="generated", reduce=True):
    """This rank's share of the mesh of the sector-sharded field (C5: marching cubes on N GPUs).

    After a border reduce (run first unless `reduce` is False) every brick's mass sits on one
    rank.  Each rank asks every other rank for the neighbour bricks it needs and does not observe
    (an all_gather of the request lists), the holders pack those tiles (one all_to_all), and each
    rank meshes its own cubes with that halo.  Returns (vertices (3T, 3), triangles (T, 3)); the
    union over ranks is the mesh of the union field, each cube meshed once."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if world == 1:
        return vol.extract_triangle_mesh(min_weight=min_weight, table=table)
    if reduce:
        border_reduce(vol, group, comm_device)
    vdev = torch.device(vol.tensor_device)
    cdev = torch.device(comm_device) if comm_device is not None else vdev

    def ready():
        if vdev.type == "cuda":
            torch.cuda.synchronize(vdev)

    # requests: this rank's missing neighbour keys, gathered everywhere
    nreq = vol.halo_keys_into(0, 0)
    req = torch.empty(max(nreq, 1), dtype=torch.int64, device=vdev)
    ready()
    nreq = vol.halo_keys_into(req.data_ptr(), req.numel())
    cnt = torch.tensor([nreq], dtype=torch.int64, device=cdev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    stride = max(1, max(counts))
    mine = torch.full((stride,), -1, dtype=torch.int64, device=cdev)
    mine[:nreq] = req[:nreq].to(cdev)
    allreq = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allreq, mine, group=group)
    # holder side: for every other rank, the tiles of its requests observed here
    me = dist.get_rank(group)
    blocks, send_counts = [], []
    for r in range(world):
        if r == me or counts[r] == 0:
            send_counts.append(0)
            continue
        q = allreq[r][:counts[r]].to(vdev).contiguous()
        buf = torch.empty((counts[r], TILE_WORDS), dtype=torch.int32, device=vdev)
        ready()
        k = vol.halo_pack(q.data_ptr(), counts[r], buf.data_ptr(), counts[r])
        blocks.append(buf[:k])
        send_counts.append(k)
    send = (torch.cat(blocks) if blocks else torch.empty((0, TILE_WORDS), dtype=torch.int32,
                                                         device=vdev)).to(cdev).contiguous()
    sc = torch.tensor(send_counts, dtype=torch.int64, device=cdev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    n_recv = sum(recv_counts)
    recv = torch.empty((max(n_recv, 1), TILE_WORDS), dtype=torch.int32, device=cdev)
    dist.all_to_all_single(recv[:n_recv], send, output_split_sizes=recv_counts,
                           input_split_sizes=send_counts, group=group)
    recv = recv.to(vdev).contiguous()
    ready()
    return vol.extract_triangle_mesh(min_weight=min_weight, table=table,
                                     halo=(recv.data_ptr(), n_recv))
