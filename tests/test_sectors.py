"""The azimuth-sector rule of the multi-GPU shards (include/tsdf_hip.h tsdf_sector_of): the numpy
restatement, the HIP library's host routine and the oracle's agree point for point, and the
sectors partition every scan.  CPU only (the host routines need no GPU)."""
import math

import numpy as np
import pytest

import oracle


def lib_sector_of(lib, pts, org, n, yaw0):
    from tsdf_map import _abi
    o = np.ascontiguousarray(org, np.float64)
    return np.array([lib.tsdf_sector_of(float(p[0]), float(p[1]), o.ctypes.data_as(_abi.D3),
                                        float(yaw0), n) for p in pts], np.int64)


@pytest.mark.parametrize("n,yaw0", [(2, 0.0), (3, 0.3), (4, 0.0), (8, -1.1), (5, 2.9)])
def test_sector_rule_agrees_and_partitions(scan0, n, yaw0):
    from tsdf_map import load_hip_library, sector_ids, select_sector
    pts, org = scan0
    pts = np.ascontiguousarray(pts[::37])
    sec = sector_ids(pts, org, n, yaw0)
    assert sec.min() >= 0 and sec.max() == n - 1
    hip = load_hip_library()
    assert np.array_equal(sec, lib_sector_of(hip, pts, org, n, yaw0))
    assert np.array_equal(sec, lib_sector_of(oracle.load(), pts, org, n, yaw0))
    total = 0
    for k in range(n):
        part = select_sector(pts, org, k, n, yaw0)
        assert np.array_equal(part, pts[sec == k])
        total += part.shape[0]
    assert total == pts.shape[0]


def test_sector_geometry():
    """Points at the true angles inside each sector land there (the pseudo-angle is monotone)."""
    from tsdf_map import sector_ids
    n, yaw0 = 6, 0.4
    th = yaw0 + 2 * math.pi * (np.arange(n * 10) + 0.5) / (n * 10)
    pts = np.stack([10 * np.cos(th), 10 * np.sin(th), np.zeros_like(th)], 1).astype(np.float32)
    sec = sector_ids(pts, np.zeros(3), n, yaw0)
    assert np.array_equal(sec, np.arange(n * 10) // 10)
    # axis directions and the origin itself
    o = np.zeros(3)
    axes = np.array([[1, 0, 0], [0, 1, 0], [-1, 0, 0], [0, -1, 0], [0, 0, 0]], np.float32)
    assert np.array_equal(sector_ids(axes, o, 4, 0.0), [0, 1, 2, 3, 0])


@pytest.mark.parametrize("rule", ["world", "index"])
def test_oracle_sector_filter_partitions_the_field(scan0, rule):
    """n sector-filtered oracle volumes together hold every ray of the scan exactly once (both
    rules: world-frame azimuth sectors, and the index rule's contiguous shares)."""
    pts, org = scan0
    pts = np.ascontiguousarray(pts[::16])
    full = oracle.OracleTSDFVolume(0.05, 0.15)
    full.integrate(pts, org)
    rays = 0
    for k in range(3):
        v = oracle.OracleTSDFVolume(0.05, 0.15, n_sectors=3, sector=k, sector_yaw0=1.0,
                                    sector_rule=rule)
        v.integrate(pts, org)
        rays += v.stats()["n_rays_total"]
    assert rays == full.stats()["n_rays_total"]
