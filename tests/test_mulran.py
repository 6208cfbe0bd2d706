"""MulRan scan files: the reader's record format and the reference
loader's quirks (ROSThread.cpp:470-559), and a MulRan-style scan sequence integrated through the
host path equal to the oracle's field.  No MulRan data ships with the reference, so the files are
synthetic scans of the analytic scene written in the MulRan record format."""
import os

import numpy as np
import pytest

from tsdf_map import mulran


def test_records_rings_and_reference_count(tmp_path):
    pts = np.random.default_rng(0).normal(size=(130, 3)).astype(np.float32)
    inten = np.arange(130, dtype=np.float32)
    f = tmp_path / "1561000444390857630.bin"
    mulran.write_bin(f, pts, inten)
    p, i, ring = mulran.read_bin(f)
    assert np.array_equal(p, pts) and np.array_equal(i, inten)
    assert ring[0] == 1 and ring[63] == 64 and ring[64] == 1 and ring[129] == 2
    assert mulran.reference_point_count(f) == 131  # the reference's trailing eof point
    with open(f, "ab") as fh:  # a partial record is dropped
        fh.write(b"\x00" * 7)
    assert mulran.read_bin(f)[0].shape[0] == 130


def test_list_scans_in_time_order(tmp_path):
    for s in (30, 4, 100):
        mulran.write_bin(tmp_path / ("%d.bin" % s), np.zeros((1, 3)))
    (tmp_path / "notes.txt").write_text("x")
    assert [s for s, _ in mulran.list_scans(tmp_path)] == [4, 30, 100]


def _sim64():
    from tsdf_map.scan_gen import OusterSim
    return OusterSim(columns=512)  # beam geometry is immaterial to the record format


def test_sequence_matches_oracle_cpu(tmp_path):
    import oracle
    sim = _sim64()
    poses = {}
    for k in range(3):
        pts_w, org = sim.scan(k)
        pose = np.eye(4)
        pose[:3, 3] = org
        mulran.write_bin(tmp_path / ("%d.bin" % (1000 + k)), pts_w[::8] - org)  # sensor frame
        poses[1000 + k] = pose
    o1 = oracle.OracleTSDFVolume(0.1, 0.3)
    assert mulran.integrate_sequence(o1, tmp_path, poses) == [1000, 1001, 1002]
    o2 = oracle.OracleTSDFVolume(0.1, 0.3)
    for s, path in mulran.list_scans(tmp_path):
        p, _, _ = mulran.read_bin(path)
        o2.integrate(mulran.to_world(p, poses[s]), poses[s][:3, 3])
    for x, y in zip(o1.export_voxels(), o2.export_voxels()):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_sequence_gpu_bitwise(tmp_path):
    import oracle
    from tsdf_map import HipTSDFVolume
    sim = _sim64()
    poses = {}
    for k in range(4):
        pts_w, org = sim.scan(k)
        pose = np.eye(4)
        pose[:3, 3] = org
        mulran.write_bin(tmp_path / ("%d.bin" % (2000 + k)), pts_w - org)
        poses[2000 + k] = pose
    o = oracle.OracleTSDFVolume(0.1, 0.3)
    g = HipTSDFVolume(0.1, 0.3)
    mulran.integrate_sequence(o, tmp_path, poses)
    mulran.integrate_sequence(g, tmp_path, poses)
    assert o.export_voxels()[0].shape[0] > 1000
    for x, y in zip(g.export_voxels(), o.export_voxels()):
        assert np.array_equal(x, y)
