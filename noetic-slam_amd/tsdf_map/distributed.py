"""Multi-GPU border-brick reduce of azimuth-sector partial fields.

Integration shards each scan by azimuth sector (one sector per rank, one process per GPU; the
sector filter runs inside the walk kernels, tsdf_params.n_sectors/sector) and needs no collective:
VDBFusion's fused field is the weighted mean sum(w s) / sum(w) of all samples, so per-rank
partial fields combine exactly up to fp32 rounding.  A brick touched by rays of several sectors is
held by several ranks; `border_reduce` moves each such brick's mass to its owner, the lowest rank
holding it, entirely device-resident:

  1. all_gather of the brick keys (tsdf_brick_keys_device; ~8 B per brick);
  2. every rank packs its bricks owned by a lower rank into 4 KiB tiles, grouped by owner, and
     resets them to the background (tsdf_border_pack_device: kernels look the lower ranks' keys up
     in the rank's own hash table);
  3. ONE all_to_all_single of the tiles — RCCL over xGMI: point-to-point, so a direct all-to-all
     of the few-percent border set instead of a ring all-reduce of whole grids;
  4. the owner merges the received tiles, sources in ascending rank order
     (tsdf_border_merge_device: weighted mean, copy where W == 0).

Afterwards the field is partitioned: every brick's full mass sits on exactly one rank, and
integration may continue (a later reduce moves only the new partial mass).  The same code drives a
CPU library (the oracle, gloo) through the same ABI: `vol.tensor_device` says where the library's
buffers live, `comm_device` where the collective's do (they differ only in the one-GPU gloo
rehearsal, which stages the tiles through host memory).
"""
import time

import numpy as np

TILE_WORDS = 1028  # include/tsdf_hip.h TSDF_TILE_WORDS


def border_reduce(vol, group=None, comm_device=None):
    """Reduce the border bricks of this rank's `vol` with the other ranks of `group`.

    Returns {"bricks_sent", "bricks_received", "tile_bytes", "ms": {"keys", "pack", "exchange",
    "merge"}} for this rank (wall time of each step; "exchange" is the tile all-to-all)."""
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

    ms = {}
    t = time.perf_counter()

    def lap(name):
        nonlocal t
        now = time.perf_counter()
        ms[name] = round((now - t) * 1e3, 3)
        t = now

    # 1. keys
    n = vol.num_bricks()
    keys = torch.empty(max(n, 1), dtype=torch.int64, device=vdev)
    ready()
    n = vol.brick_keys_into(keys.data_ptr(), keys.numel())
    cnt = torch.tensor([n], dtype=torch.int64, device=cdev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    stride = max(1, max(counts))
    mine = torch.full((stride,), -1, dtype=torch.int64, device=cdev)
    mine[:n] = keys[:n].to(cdev)
    allk = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allk, mine, group=group)
    allk = torch.stack(allk).to(vdev).contiguous()
    lap("keys")

    # 2. pack the bricks owned elsewhere (rows grouped by destination rank)
    send = torch.empty((max(n, 1), TILE_WORDS), dtype=torch.int32, device=vdev)
    ready()
    send_counts = vol.border_pack(allk.data_ptr(), counts, stride, world, rank, send.data_ptr(),
                                  send.shape[0])
    lap("pack")

    # 3. one all-to-all of the tiles
    sc = torch.tensor(send_counts, dtype=torch.int64, device=cdev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    n_send, n_recv = sum(send_counts), sum(recv_counts)
    recv = torch.empty((max(n_recv, 1), TILE_WORDS), dtype=torch.int32, device=cdev)
    dist.all_to_all_single(recv[:n_recv], send[:n_send].to(cdev), output_split_sizes=recv_counts,
                           input_split_sizes=send_counts, group=group)

    recv = recv.to(vdev)
    ready()
    lap("exchange")

    # 4. merge on the owner, sources in ascending rank order
    vol.border_merge(recv.data_ptr(), recv_counts)
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
