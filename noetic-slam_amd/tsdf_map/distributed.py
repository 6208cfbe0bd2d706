"""Multi-GPU read-out: reduce border bricks of azimuth-sector partial fields across ranks.

Integration shards each scan by azimuth sector (one sector per rank, one process per GPU) and
needs no collective: VDBFusion's fused field is the weighted mean sum(w s) / sum(w) of all
samples, so per-rank partial fields combine exactly up to fp32 rounding.  At read-out, bricks held
by more than one rank (the sector borders) are exchanged ONCE with a direct all-to-all to their
owner (the lowest holding rank) and merged there in rank order — no ring all-reduce of whole grids:
the border set is a few percent of the bricks, and xGMI is point-to-point.

Collectives run through torch.distributed: RCCL (backend "nccl") over xGMI on GPUs, gloo on CPU.
"""
import numpy as np


def _merge_into(S, W, s_in, w_in):
    """fp32 weighted-mean merge, the import rule of include/tsdf_hip.h (copy where W == 0)."""
    S = S.astype(np.float32, copy=True)
    W = W.astype(np.float32, copy=True)
    m = w_in > 0
    copy = m & (W == 0)
    mix = m & (W != 0)
    S[copy] = s_in[copy]
    W[copy] = w_in[copy]
    nw = (W[mix] + w_in[mix]).astype(np.float32)
    S[mix] = ((S[mix] * W[mix]).astype(np.float32) +
              (s_in[mix] * w_in[mix]).astype(np.float32)).astype(np.float32) / nw
    W[mix] = nw
    return S, W


def _keys(coords):
    c = coords.astype(np.int64) + (1 << 20)
    return c[:, 0] | (c[:, 1] << 21) | (c[:, 2] << 42)


def merged_bricks(vol, group=None, device=None):
    """Return this rank's share of the merged map: (coords (n,3) int32, sdf (n,512), weight).

    The union over ranks is the full map with every brick exactly once.  `vol` is any volume with
    export_bricks() (the GPU backend, or the oracle in CPU tests)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    coords, S, W = vol.export_bricks()
    coords = np.ascontiguousarray(coords, np.int32).reshape(-1, 3)
    S = np.ascontiguousarray(S, np.float32).reshape(-1, 512)
    W = np.ascontiguousarray(W, np.float32).reshape(-1, 512)
    if world == 1:
        return coords, S, W
    dev = device if device is not None else torch.device("cpu")

    # 1. who holds what: all-gather the brick keys
    n = torch.tensor([coords.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
    mine = torch.full((mx,), -1, dtype=torch.int64, device=dev)
    mine[:coords.shape[0]] = torch.from_numpy(_keys(coords)).to(dev)
    allk = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allk, mine, group=group)
    keys_of = [allk[r][:counts[r]].cpu().numpy() for r in range(world)]

    # 2. owner of each key = lowest holding rank
    owner = {}
    for r in range(world):
        for k in keys_of[r].tolist():
            if k not in owner:
                owner[k] = r
    my_keys = keys_of[rank]
    my_owner = np.array([owner[k] for k in my_keys.tolist()], np.int64)

    # 3. all-to-all: send my copies of bricks owned elsewhere to their owner
    send_idx = [np.flatnonzero(my_owner == r) if r != rank else np.zeros(0, np.int64)
                for r in range(world)]
    send_sizes = [len(i) for i in send_idx]
    order = np.concatenate(send_idx) if send_idx else np.zeros(0, np.int64)
    payload = np.concatenate([S[order], W[order]], axis=1) if len(order) else \
        np.zeros((0, 1024), np.float32)
    sizes = torch.tensor(send_sizes, dtype=torch.int64, device=dev)
    recv_sizes = torch.empty_like(sizes)
    dist.all_to_all_single(recv_sizes, sizes, group=group)
    recv_sizes = [int(x) for x in recv_sizes.cpu().tolist()]
    send_t = torch.from_numpy(np.ascontiguousarray(payload)).to(dev)
    recv_t = torch.empty((sum(recv_sizes), 1024), dtype=torch.float32, device=dev)
    dist.all_to_all_single(recv_t, send_t, output_split_sizes=recv_sizes,
                           input_split_sizes=send_sizes, group=group)
    # the keys travel beside the tiles (same split)
    ksend = torch.from_numpy(my_keys[order].astype(np.int64)).to(dev)
    krecv = torch.empty((sum(recv_sizes),), dtype=torch.int64, device=dev)
    dist.all_to_all_single(krecv, ksend, output_split_sizes=recv_sizes,
                           input_split_sizes=send_sizes, group=group)
    recv = recv_t.cpu().numpy()
    rkeys = krecv.cpu().numpy()

    # 4. merge on the owner, holders in ascending rank order (self first: self is the lowest)
    keep = my_owner == rank
    out_keys = my_keys[keep]
    oS, oW = S[keep].copy(), W[keep].copy()
    pos = {k: i for i, k in enumerate(out_keys.tolist())}
    src = np.repeat(np.arange(world), recv_sizes)
    for j in np.argsort(src, kind="stable"):
        i = pos[int(rkeys[j])]
        oS[i], oW[i] = _merge_into(oS[i], oW[i], recv[j, :512], recv[j, 512:])
    oc = coords[keep]
    return oc, oS, oW
