"""The N>1 path on CPU: world_size-2 gloo ranks, each integrating its azimuth sector into its own
partial field (the oracle stands in for the GPU volume here: same ABI, same sector filter), then
the border-brick reduce of tsdf_map.distributed (the GPU's code path, on host buffers), twice.  The union of the ranks' merged shares must equal the
single-volume field: same bricks/voxels, weights exact, |dSDF| <= 1e-5 m, single-owner voxels
bit-exact."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import REPO


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
    import oracle
    from tsdf_map.distributed import merged_bricks
    from tsdf_map.scan_gen import OusterSim

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sim = OusterSim()
    # the sector filter inside the integrate (tsdf_params.n_sectors / sector), as on the GPUs
    vol = oracle.OracleTSDFVolume(0.05, 0.15, n_sectors=world, sector=rank, sector_yaw0=0.3)
    for k in (0, 3):
        pts, org = sim.scan(k)
        vol.integrate(np.ascontiguousarray(pts[::8]), org)
    c, s, w = merged_bricks(vol)
    # a second reduce after more integration moves only the new partial mass
    pts, org = sim.scan(6)
    vol.integrate(np.ascontiguousarray(pts[::8]), org)
    c, s, w = merged_bricks(vol)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), coords=c, sdf=s, weight=w)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sector_sharded_merge_gloo(world, tmp_path):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    import oracle
    from tsdf_map import bricks_to_voxels
    from tsdf_map.scan_gen import OusterSim

    parts = [np.load(str(tmp_path / ("rank%d.npz" % r))) for r in range(world)]
    coords = np.concatenate([p["coords"] for p in parts])
    # every brick owned exactly once
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]
    mi, ms, mw = bricks_to_voxels(coords, np.concatenate([p["sdf"] for p in parts]),
                                  np.concatenate([p["weight"] for p in parts]))
    sim = OusterSim()
    ref = oracle.OracleTSDFVolume(0.05, 0.15)
    for k in (0, 3, 6):
        pts, org = sim.scan(k)
        ref.integrate(np.ascontiguousarray(pts[::8]), org)
    ri, rs, rw = ref.export_voxels()
    assert np.array_equal(mi, ri)
    assert np.array_equal(mw, rw)
    assert np.max(np.abs(ms - rs)) <= 1e-5
    assert np.mean(ms.view(np.uint32) == rs.view(np.uint32)) > 0.5
