"""ROS-free bag ingest.  No bag ships with the reference (the OS1-128 bag is
.gitignored), so bags are written here with the same record format and ROS1 message
encoding: round trips pin the reader; pose interpolation is checked in closed form; a DLIO-style
bag (world-frame dlio::Point clouds + 100 Hz poses) ingested through the host boundary must equal
integrating the same clouds from the interpolated origins (oracle; and the GPU, bitwise)."""
import struct

import numpy as np
import pytest

from tsdf_map import ingest, rosbag


def _quat_yaw(y):
    return (0.0, 0.0, np.sin(y / 2), np.cos(y / 2))


def _write_dlio_bag(path, sim, n_scans=4, compression="none", decim=4):
    truth = []
    with rosbag.BagWriter(path, compression=compression, chunk_messages=7) as w:
        for k in range(n_scans + 1):  # poses at 100 Hz around each 10 Hz scan
            for j in range(10):
                t = 1_000_000_000 + (k * 10 + j) * 10_000_000
                pos = (0.01 * (k * 10 + j), 0.002 * (k * 10 + j), 0.0)
                w.write(ingest.DLIO_POSE, "geometry_msgs/PoseStamped", t,
                        rosbag.encode_pose_stamped(t, "robot/odom", pos, _quat_yaw(0.01 * j)))
        for k in range(n_scans):
            pts, _ = sim.scan(k)
            pts = pts[::decim]
            t = 1_000_000_000 + k * 100_000_000 + 3_000_000  # between two pose samples
            w.write(ingest.DLIO_CLOUD, "sensor_msgs/PointCloud2", t,
                    rosbag.encode_pointcloud2(t, "robot/odom", pts))
            truth.append((t, pts))
    return truth


def test_roundtrip_and_decode(tmp_path, sim):
    for comp in ("none", "bz2"):
        p = tmp_path / ("b_%s.bag" % comp)
        truth = _write_dlio_bag(str(p), sim, n_scans=2, compression=comp)
        bag = rosbag.BagReader(str(p))
        clouds = list(bag.messages({ingest.DLIO_CLOUD}))
        assert [m.time_ns for m in clouds] == [t for t, _ in truth]
        c = rosbag.decode_pointcloud2(clouds[0].data)
        assert c.point_step == 32 and c.width == truth[0][1].shape[0] and c.height == 1
        xyz = np.frombuffer(c.data, np.float32).reshape(-1, 8)[:, :3]
        assert np.array_equal(xyz, truth[0][1])
        assert ingest.cloud_xyz_layout(c) == (0, False)
        poses = list(bag.messages({ingest.DLIO_POSE}))
        assert len(poses) == 30
        hd, pos, q = rosbag.decode_pose_stamped(poses[11].data)
        assert hd["stamp_ns"] == poses[11].time_ns and hd["frame_id"] == "robot/odom"
        assert np.allclose(pos, (0.11, 0.022, 0.0)) and np.allclose(q, _quat_yaw(0.01))


def test_lz4_chunks_are_rejected(tmp_path):
    p = tmp_path / "lz4.bag"
    rec = rosbag.BagWriter._rec({"op": bytes([rosbag.OP_CHUNK]), "compression": "lz4",
                                 "size": struct.pack("<I", 0)}, b"")
    p.write_bytes(rosbag.MAGIC + rec)
    with pytest.raises(NotImplementedError):
        list(rosbag.BagReader(str(p)).messages())


def test_pose_interpolation_closed_form():
    tr = ingest.PoseTrack()
    tr.add(100, (0, 0, 0), _quat_yaw(0.0))
    tr.add(200, (1, 2, 4), _quat_yaw(0.5))
    p, q = tr.at(125)
    assert np.allclose(p, (0.25, 0.5, 1.0)) and np.allclose(q, _quat_yaw(0.125))
    assert tr.at(99) is None and tr.at(201) is None
    assert tr.at(150, max_gap_ms=1e-5) is None  # 100 ns gap > 0.01 ns
    assert np.array_equal(tr.at(200)[0], (1, 2, 4))


def _expected(oracle_vol, bag_path, truth):
    track = ingest.load_poses(rosbag.BagReader(bag_path))
    for t, pts in truth:
        oracle_vol.integrate(pts, track.at(t)[0])


def test_ingest_matches_direct_integration(tmp_path, sim):
    import oracle
    p = str(tmp_path / "dlio.bag")
    truth = _write_dlio_bag(p, sim)
    o1 = oracle.OracleTSDFVolume(0.05, 0.15)
    assert ingest.ingest_bag(o1, p) == (4, 0)
    o2 = oracle.OracleTSDFVolume(0.05, 0.15)
    _expected(o2, p, truth)
    for x, y in zip(o1.export_voxels(), o2.export_voxels()):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_ingest_gpu_bitwise(tmp_path, sim):
    import oracle
    from tsdf_map import HipTSDFVolume
    p = str(tmp_path / "dlio.bag")
    truth = _write_dlio_bag(p, sim, compression="bz2", decim=2)
    g = HipTSDFVolume(0.05, 0.15)
    assert ingest.ingest_bag(g, p) == (4, 0)
    o = oracle.OracleTSDFVolume(0.05, 0.15)
    _expected(o, p, truth)
    for x, y in zip(g.export_voxels(), o.export_voxels()):
        assert np.array_equal(x, y)
