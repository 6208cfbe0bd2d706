"""BASELINE.json configs C5 and C4 as GPU tests (both ran only as builder scripts).

* C5 (configs[4]): a synthetic DLIO bag (world-frame dlio::Point clouds of the OS-1-128 1024x10
  sensor + 100 Hz poses; no bag ships with the reference, `.gitignore:4,7`) ingested at 2 cm /
  6 cm, then marching cubes (`.gitignore:9,12-13`: the node's mesh outputs).  The GPU field and
  mesh equal the oracle's bit for bit; the field is compared with the literal upstream update:
  VDBFusion at its own precisions (same voxels and weights, |dS| <= 1e-5 m) and Voxblox's
  per-sample update (0 voxels over 0.1 tau).
* C4 (configs[3]): OS-1-128 2048x10 scans at 2 cm / 6 cm, azimuth-sharded over 4 contexts (the
  4 GPUs of C4, emulated on one: tests/test_multigpu.py's collective emulation), border bricks
  reduced; every rank's field equals the oracle's reduce bit for bit and the union equals the
  single-volume field.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from fieldcmp import _keys, compare
from test_multigpu import emulated_reduce, emulated_reduce_host, voxels_equal_bitwise

pytestmark = pytest.mark.gpu


def _write_dlio_bag(path, sim, n_scans):
    """Clouds at 10 Hz stamped on a pose sample, poses at 100 Hz (linear between the scans'
    origins): the pose at every cloud stamp is the scan's own origin."""
    from tsdf_map import ingest, rosbag
    from tsdf_map.scan_gen import pose_on_circle
    t0 = 1_000_000_000
    origins = [np.asarray(pose_on_circle(k, hz=sim.hz)[0], np.float64) for k in range(n_scans + 1)]
    with rosbag.BagWriter(path, compression="none", chunk_messages=64) as w:
        for k in range(n_scans):
            for j in range(10):
                a = j / 10.0
                pos = (1 - a) * origins[k] + a * origins[k + 1]
                t = t0 + (k * 10 + j) * 10_000_000
                w.write(ingest.DLIO_POSE, "geometry_msgs/PoseStamped", t,
                        rosbag.encode_pose_stamped(t, "robot/odom", tuple(pos), (0, 0, 0, 1)))
        t = t0 + n_scans * 100_000_000
        w.write(ingest.DLIO_POSE, "geometry_msgs/PoseStamped", t,
                rosbag.encode_pose_stamped(t, "robot/odom", tuple(origins[n_scans]), (0, 0, 0, 1)))
        for k in range(n_scans):
            pts, org = sim.scan(k)
            assert np.allclose(org, origins[k])
            t = t0 + k * 100_000_000
            w.write(ingest.DLIO_CLOUD, "sensor_msgs/PointCloud2", t,
                    rosbag.encode_pointcloud2(t, "robot/odom", pts))


C5_SCANS = 12
VOXBLOX_C5 = dict(semantics="voxblox", space_carving=False, max_range=100.0, min_range=0.1)


@pytest.fixture(scope="module")
def c5_bag(tmp_path_factory):
    from tsdf_map.scan_gen import OusterSim
    path = str(tmp_path_factory.mktemp("c5") / "c5_dlio.bag")
    _write_dlio_bag(path, OusterSim(), C5_SCANS)
    return path


@pytest.fixture(scope="module")
def c5_bag_sparse(tmp_path_factory):
    """Every 8th point of 6 clouds: Voxblox's carving defaults walk ~250 voxels per ray at 2 cm,
    which the per-sample CPU restatement must replay."""
    from tsdf_map.scan_gen import OusterSim

    class Sparse(OusterSim):
        def scan(self, k, *a, **kw):
            p, o = super().scan(k, *a, **kw)
            return np.ascontiguousarray(p[k % 8::8]), o

    path = str(tmp_path_factory.mktemp("c5s") / "c5_sparse.bag")
    _write_dlio_bag(path, Sparse(), 6)
    return path


def test_c5_voxblox_upstream_defaults(c5_bag_sparse):
    """C5's Voxblox comparison with voxblox's own defaults (TsdfIntegratorBase::Config: carving on,
    min / max ray 0.1 / 5 m, use_const_weight = false -> 1/z^2, dropoff, clearing rays, truncation
    0.1 m) at 2 cm: GPU == the oracle's scan-fused twin bit for bit; against the literal
    per-sample update the |dS| over 0.1 tau are counted (reported) and bounded."""
    from tsdf_map import HipTSDFVolume, TsdfIntegratorConfig, ingest
    cfg = TsdfIntegratorConfig()
    kw = dict(semantics="voxblox", space_carving=cfg.voxel_carving_enabled,
              min_range=cfg.min_ray_length_m, max_range=cfg.max_ray_length_m,
              use_const_weight=cfg.use_const_weight, allow_clear=cfg.allow_clear,
              use_weight_dropoff=cfg.use_weight_dropoff, max_weight=cfg.max_weight)
    vs, tau = 0.02, cfg.default_truncation_distance
    g = HipTSDFVolume(vs, tau, max_bricks=1 << 18, **kw)
    assert ingest.ingest_bag(g, c5_bag_sparse) == (6, 0)
    g.sync()
    gv = g.export_voxels()
    o = oracle.OracleTSDFVolume(vs, tau, threads=8, **kw)
    assert ingest.ingest_bag(o, c5_bag_sparse) == (6, 0)
    r = compare(gv, o.export_voxels())
    assert r["only_a"] == r["only_b"] == r["weight_mismatch"] == 0
    assert r["bitwise_equal"] == r["voxels_a"] > 100_000, r
    del o
    lit = oracle.OracleTSDFVolume(vs, tau, mode=oracle.MODE_SEQUENTIAL, **kw)
    assert ingest.ingest_bag(lit, c5_bag_sparse) == (6, 0)
    lv = lit.export_voxels()
    d = compare(gv, lv)
    _, ia, ib = np.intersect1d(_keys(gv[0]), _keys(lv[0]), assume_unique=True, return_indices=True)
    dd = np.abs(gv[1][ia].astype(np.float64) - lv[1][ib])
    over = int((dd > 0.1 * tau).sum())
    print("C5 voxblox upstream defaults vs literal:", d, "over 0.1 tau:", over,
          "p99.9:", float(np.quantile(dd, 0.999)))
    assert d["only_a"] == d["only_b"] == 0
    # carving puts far-field (clamped at tau) and near-surface samples of one scan on a voxel,
    # whose clamped per-sample order can differ by up to tau from the scan-fused sum
    assert over <= 1e-3 * dd.size and np.quantile(dd, 0.999) <= 0.1 * tau


def test_c5_voxblox_merged_upstream_defaults(c5_bag_sparse):
    """C5 against voxblox_ros's default integrator, MergedTsdfIntegrator, with
    voxblox's own config defaults at 2 cm: GPU == the oracle's scan-fused twin bit for bit; against
    the literal per-sample update of the same bundles the |dS| over 0.1 tau are counted and
    bounded; against SimpleTsdfIntegrator's field the differences are reported (bundling moves the
    rays' end points, so these differ by construction)."""
    from tsdf_map import HipTSDFVolume, TsdfIntegratorConfig, ingest
    cfg = TsdfIntegratorConfig()
    kw = dict(semantics="voxblox", space_carving=cfg.voxel_carving_enabled,
              min_range=cfg.min_ray_length_m, max_range=cfg.max_ray_length_m,
              use_const_weight=cfg.use_const_weight, allow_clear=cfg.allow_clear,
              use_weight_dropoff=cfg.use_weight_dropoff, max_weight=cfg.max_weight)
    vs, tau = 0.02, cfg.default_truncation_distance
    g = HipTSDFVolume(vs, tau, max_bricks=1 << 18, method="merged", **kw)
    assert ingest.ingest_bag(g, c5_bag_sparse) == (6, 0)
    g.sync()
    gv = g.export_voxels()
    o = oracle.OracleTSDFVolume(vs, tau, threads=8, method="merged", **kw)
    assert ingest.ingest_bag(o, c5_bag_sparse) == (6, 0)
    r = compare(gv, o.export_voxels())
    assert r["only_a"] == r["only_b"] == r["weight_mismatch"] == 0
    assert r["bitwise_equal"] == r["voxels_a"] > 100_000, r
    del o
    lit = oracle.OracleTSDFVolume(vs, tau, mode=oracle.MODE_SEQUENTIAL, method="merged", **kw)
    assert ingest.ingest_bag(lit, c5_bag_sparse) == (6, 0)
    lv = lit.export_voxels()
    d = compare(gv, lv)
    _, ia, ib = np.intersect1d(_keys(gv[0]), _keys(lv[0]), assume_unique=True, return_indices=True)
    dd = np.abs(gv[1][ia].astype(np.float64) - lv[1][ib])
    over = int((dd > 0.1 * tau).sum())
    simple = oracle.OracleTSDFVolume(vs, tau, threads=8, **kw)
    assert ingest.ingest_bag(simple, c5_bag_sparse) == (6, 0)
    vs_simple = compare(gv, simple.export_voxels())
    print("C5 voxblox merged vs literal:", d, "over 0.1 tau:", over,
          "p99.9:", float(np.quantile(dd, 0.999)), "| merged vs simple:", vs_simple)
    assert d["only_a"] == d["only_b"] == 0
    assert over <= 1e-3 * dd.size and np.quantile(dd, 0.999) <= 0.1 * tau


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "voxblox"])
def test_c5_bag_2cm_field_and_mesh(c5_bag, semantics):
    from tsdf_map import HipTSDFVolume, ingest
    vs, tau = 0.02, 0.06
    kw = dict(VOXBLOX_C5) if semantics == "voxblox" else dict(semantics=semantics)
    g = HipTSDFVolume(vs, tau, max_bricks=1 << 18, **kw)
    assert ingest.ingest_bag(g, c5_bag) == (C5_SCANS, 0)
    g.sync()
    gv = g.export_voxels()
    o = oracle.OracleTSDFVolume(vs, tau, threads=8, **kw)
    assert ingest.ingest_bag(o, c5_bag) == (C5_SCANS, 0)
    ov = o.export_voxels()
    r = compare(gv, ov)
    assert r["only_a"] == r["only_b"] == r["weight_mismatch"] == 0
    assert r["bitwise_equal"] == r["voxels_a"] > 1_000_000, r
    # the mesh of the field (VDBFusion extract_triangle_mesh's slot), bit for bit
    vg, _ = g.extract_triangle_mesh()
    o1 = oracle.OracleTSDFVolume(vs, tau, **kw)  # the oracle's mesh runs in its serial mode
    o1.import_bricks(*o.export_bricks())
    vo, _ = o1.extract_triangle_mesh()
    assert vg.shape[0] > 300_000 and vg.shape == vo.shape and np.array_equal(vg, vo)
    del o, o1
    # distance from the literal upstream update
    mode = oracle.MODE_VDB_LITERAL if semantics == "vdbfusion_f64" else oracle.MODE_SEQUENTIAL
    lit = oracle.OracleTSDFVolume(vs, tau, mode=mode, **kw)
    assert ingest.ingest_bag(lit, c5_bag) == (C5_SCANS, 0)
    lv = lit.export_voxels()
    d = compare(gv, lv)
    print("C5", semantics, "vs literal:", d)
    if semantics == "vdbfusion_f64":  # SURVEY §8c's per-voxel bar
        assert d["only_a"] == d["only_b"] == d["weight_mismatch"] == 0
        assert d["max_abs_dsdf"] <= 1e-5
    else:  # SURVEY §8c against Voxblox: |dS| <= 0.1 tau on every common voxel
        _, ia, ib = np.intersect1d(_keys(gv[0]), _keys(lv[0]), assume_unique=True,
                                   return_indices=True)
        dd = np.abs(gv[1][ia].astype(np.float64) - lv[1][ib])
        assert d["only_a"] == d["only_b"] == 0
        assert int((dd > 0.1 * tau).sum()) == 0, float(dd.max())


def test_c4_four_sector_border_reduce_2cm():
    from tsdf_map import HipTSDFVolume, bricks_to_voxels
    from tsdf_map.scan_gen import OusterSim
    vs, tau, world, yaw0 = 0.02, 0.06, 4, 0.3
    sim = OusterSim("os1_128_2048", hz=20.0)
    kw = dict(semantics="vdbfusion_f64", n_sectors=world, sector_yaw0=yaw0)
    dev = torch.device("cuda", 0)
    g = [HipTSDFVolume(vs, tau, sector=r, max_bricks=1 << 18, **kw) for r in range(world)]
    o = [oracle.OracleTSDFVolume(vs, tau, sector=r, **kw) for r in range(world)]
    ref = oracle.OracleTSDFVolume(vs, tau, semantics="vdbfusion_f64", threads=8)
    for ks in ((0, 1), (7,)):
        for k in ks:
            pts, org = sim.scan(k)
            for v in g + o + [ref]:
                v.integrate(pts, org)
        gs = emulated_reduce(g, dev)
        emulated_reduce_host(o)
        assert sum(map(sum, gs)) > 100  # border bricks exist
        for r in range(world):
            assert voxels_equal_bitwise(g[r].export_voxels(), o[r].export_voxels()), r
    parts = [v.export_bricks() for v in g]
    keep = [(w.reshape(len(c), -1) > 0).any(1) for c, _, w in parts]
    coords = np.concatenate([c[k] for (c, _, _), k in zip(parts, keep)])
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]  # each brick on one rank
    mi, ms, mw = bricks_to_voxels(coords, np.concatenate([s[k] for (_, s, _), k in zip(parts, keep)]),
                                  np.concatenate([w[k] for (_, _, w), k in zip(parts, keep)]))
    ri, rs, rw = ref.export_voxels()
    assert np.array_equal(mi, ri) and np.array_equal(mw, rw)
    assert np.max(np.abs(ms - rs)) <= 1e-5


@pytest.mark.parametrize("table", ["generated", "lorensen"])
def test_c5_sharded_mesh_four_contexts(c5_bag, table):
    """VERDICT r4 #3, C5's "2 cm + marching cubes, 8 GPUs": the 2 cm C5 bag into 4 sector contexts
    (one GPU standing in for four), border reduce, one-brick halo exchange, one mesh per context
    (tsdf_extract_mesh_local).  The union of the contexts' soups equals, triangle for triangle, the
    oracle's sharded mesh and the mesh of the union field; against the unsharded mesh only the
    border voxels' merge rounding differs."""
    from test_distributed import tri_set
    from tsdf_map import HipTSDFVolume, extract_mesh_local, ingest
    vs, tau, n = 0.02, 0.06, 4
    g = HipTSDFVolume.sharded(n, vs, tau, device_ids=[0] * n, sector_yaw0=0.4,
                              max_bricks=1 << 17, semantics="vdbfusion_f64")
    assert ingest.ingest_bag(g, c5_bag) == (C5_SCANS, 0)
    vg, _ = extract_mesh_local(g, table=table)
    o = [oracle.OracleTSDFVolume(vs, tau, n_sectors=n, sector=r, sector_yaw0=0.4,
                                 semantics="vdbfusion_f64") for r in range(n)]
    assert ingest.ingest_bag(o, c5_bag) == (C5_SCANS, 0)
    from tsdf_map import extract_mesh_local as eml
    vo, _ = eml(o, table=table)
    assert vg.shape[0] > 300_000
    assert vg.shape == vo.shape and np.array_equal(vg, vo)  # same soups, same order, same bits
    union = oracle.OracleTSDFVolume(vs, tau, semantics="vdbfusion_f64")
    for v in g:
        c, s, w = v.export_bricks()
        keep = (w.reshape(len(c), -1) > 0).any(1)
        union.import_bricks(c[keep], s[keep], w[keep])
    assert np.array_equal(tri_set(vg), tri_set(union.extract_triangle_mesh(table=table)[0]))
    one = HipTSDFVolume(vs, tau, max_bricks=1 << 18, semantics="vdbfusion_f64")
    assert ingest.ingest_bag(one, c5_bag) == (C5_SCANS, 0)
    v1, _ = one.extract_triangle_mesh(table=table)
    same = np.intersect1d(tri_set(vg).view(np.dtype((np.void, 36))).ravel(),
                          tri_set(v1).view(np.dtype((np.void, 36))).ravel()).shape[0]
    print("C5 sharded mesh (%s): %d triangles, unsharded %d, identical %d" %
          (table, vg.shape[0] // 3, v1.shape[0] // 3, same))
    assert abs(v1.shape[0] - vg.shape[0]) <= 1e-3 * v1.shape[0]
    assert same >= 0.99 * v1.shape[0] // 3
