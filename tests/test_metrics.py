"""The per-batch metrics log (tsdf_set_metrics_log; SURVEY §5 metrics row): one JSON line per
finished GPU batch, consistent with tsdf_get_stats and the oracle."""
import json

import numpy as np
import pytest

import oracle
from conftest import decimate

pytestmark = pytest.mark.gpu


def test_metrics_log_per_scan(sim, tmp_path):
    from tsdf_map import HipTSDFVolume
    log = tmp_path / "m.jsonl"
    g = HipTSDFVolume(0.05, 0.15, max_batch=1, max_bricks=256)  # one scan per batch; grows
    g.set_profiling(True)
    g.set_metrics_log(log)
    o = oracle.OracleTSDFVolume(0.05, 0.15)
    scans = [sim.scan(k) for k in (0, 1, 2, 3)]
    for p, q in scans:
        p = decimate(p, 2)
        g.integrate(p, q)
        o.integrate(p, q)
    g.sync()
    st = g.stats()
    lines = [json.loads(x) for x in log.read_text().splitlines()]
    ok = [r for r in lines if r["committed"]]
    assert len(ok) == 4 and all(r["scans"] == 1 for r in ok)
    assert any(not r["committed"] for r in lines)  # the pool grew: a batch was re-run
    assert sum(r["rays"] for r in ok) == st["n_rays_total"] == sum(p.shape[0] // 2 + p.shape[0] % 2
                                                                    for p, _ in scans)
    assert sum(r["voxel_updates"] for r in ok) == st["n_voxels_total"]
    # a failed batch's allocations stay in the pool (its replay finds them): the committed
    # records' new bricks add up to at most the pool, and the last record reports the pool
    assert sum(r["new_bricks"] for r in ok) <= st["n_bricks"] == o.num_bricks() == lines[-1]["bricks"]
    assert all(r["path_ms"] > 0 and r["gbs"] > 0 for r in ok)
    assert ok[0]["algorithmic_bytes"] == 12 * ok[0]["rays"] + 16 * ok[0]["voxel_updates"]
    g.set_metrics_log(None)
    g.integrate(*scans[0])
    g.sync()
    assert len(log.read_text().splitlines()) == len(lines)
