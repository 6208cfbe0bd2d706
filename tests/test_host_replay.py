"""The C-ABI driven from C++ the way tsdf_map_node drives it (noetic-slam_amd/host/tsdf_replay.cpp:
one PointCloud2 per scan through tsdf_integrate, then the map write-out through
tsdf_export_bricks).  On the CPU the same driver is linked against the oracle library, which
exports the same ABI; on the GPU the shipped binary (linked against libtsdf_hip.so) must write the
oracle's map bit for bit.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle
from conftest import REPO, decimate
from tsdf_map import bricks_to_voxels

HOST = os.path.join(REPO, "noetic-slam_amd", "host")


def dlio_records(xyz):
    """dlio::Point records (32 B: x y z 1 | intensity pad t pad; dlio.h:85-106)."""
    rec = np.zeros((xyz.shape[0], 8), np.float32)
    rec[:, :3] = xyz
    rec[:, 3] = 1.0
    rec[:, 4] = 7.0
    return rec


def write_stream(path, scans):
    with open(path, "wb") as f:
        for xyz, org in scans:
            rec = dlio_records(xyz)
            f.write(struct.pack("<QIIi3d", rec.shape[0], 32, 0, 0, *[float(v) for v in org]))
            f.write(rec.tobytes())


def read_bricks(path):
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        coords = np.frombuffer(f.read(12 * n), np.int32).reshape(n, 3)
        sdf = np.frombuffer(f.read(2048 * n), np.float32).reshape(n, 512)
        w = np.frombuffer(f.read(2048 * n), np.float32).reshape(n, 512)
    return coords, sdf, w


def scans_for_test(sim):
    return [(decimate(p, 16), org) for p, org in (sim.scan(k) for k in (0, 1, 5))]


def oracle_voxels(scans, **kw):
    o = oracle.OracleTSDFVolume(0.05, 0.15, **kw)
    for xyz, org in scans:
        o.integrate_cloud(dlio_records(xyz).tobytes(), xyz.shape[0], 32, 0, org)
    return bricks_to_voxels(*o.export_bricks())


@pytest.mark.parametrize("semantics", ["vdbfusion", "voxblox"])
def test_replay_driver_against_oracle_library(tmp_path, sim, semantics):
    lib = oracle.load()  # builds oracle/build/libtsdf_oracle.so if needed
    del lib
    exe = tmp_path / "tsdf_replay_oracle"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", str(exe),
                           os.path.join(HOST, "tsdf_replay.cpp"),
                           "-L" + os.path.dirname(oracle.LIB_PATH), "-ltsdf_oracle",
                           "-Wl,-rpath," + os.path.dirname(oracle.LIB_PATH)])
    scans = scans_for_test(sim)
    write_stream(tmp_path / "in.scans", scans)
    subprocess.check_call([str(exe), str(tmp_path / "in.scans"), str(tmp_path / "out.bricks"),
                           "0.05", "0.15", semantics])
    got = bricks_to_voxels(*read_bricks(tmp_path / "out.bricks"))
    # tsdf_default_params: Voxblox's 1/z^2 weight (upstream's default), the world z axis here
    ref = oracle_voxels(scans, semantics=semantics, use_const_weight=False)
    assert got[0].shape[0] > 1000
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("semantics", ["vdbfusion", "voxblox"])
def test_replay_driver_on_gpu_bitwise(tmp_path, sim, semantics):
    exe = os.path.join(REPO, "noetic-slam_amd", "lib", "tsdf_replay")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    scans = scans_for_test(sim)
    write_stream(tmp_path / "in.scans", scans)
    out = subprocess.run([exe, str(tmp_path / "in.scans"), str(tmp_path / "out.bricks"), "0.05",
                          "0.15", semantics], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = bricks_to_voxels(*read_bricks(tmp_path / "out.bricks"))
    ref = oracle_voxels(scans, semantics=semantics, use_const_weight=False)
    assert got[0].shape[0] > 1000
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[2], ref[2])
    assert np.array_equal(got[1].view(np.uint32), ref[1].view(np.uint32))


# ---- the node's two subscriptions: clouds paired with the 100 Hz pose track (host/tsdf_map_core.h)

def topic_stream(sim, tilt=0.0):
    """(records, expected clouds with their origins): DLIO-like arrival order — poses at 100 Hz,
    each cloud stamped 3 ms after a pose sample and arriving before the sample that brackets it;
    one cloud older than the track and one inside a 60 ms pose gap are dropped."""
    from tsdf_map.ingest import PoseTrack
    t0 = 1_000_000_000
    track = PoseTrack()
    recs, want = [], []

    def pose(t):
        a = (t - t0) * 1e-9
        # tilt: the sensor pitches and yaws over time (its z axis matters for Voxblox's 1/z^2)
        h, r = 0.5 * tilt * a, 0.5 * (0.3 * a)
        q = (np.sin(h) * np.cos(r), np.sin(h) * np.sin(r), np.cos(h) * np.sin(r), np.cos(h) * np.cos(r))
        return (2.0 + 3.0 * np.cos(0.3 * a), -1.0 + 3.0 * np.sin(0.3 * a), 0.05 * a), q

    clouds = {0: 0, 1: 1, 2: 5, 3: 9}
    recs.append(("C", t0 - 5_000_000, decimate(sim.scan(7)[0], 16)))  # before the track: dropped
    for k in range(4):
        for j in range(10):
            t = t0 + (k * 10 + j) * 10_000_000
            if k == 2 and j in (4, 5, 6, 7, 8):
                continue  # a 60 ms gap in the pose stream
            p, q = pose(t)
            track.add(t, p, q)
            recs.append(("P", t, (p, q)))
            if j == 9 or (k == 2 and j == 3):
                tc = t + 3_000_000 if j == 9 else t + 33_000_000  # the latter falls in the gap
                pts = decimate(sim.scan(clouds[k])[0], 16)
                recs.append(("C", tc, pts))
                if j == 9:
                    want.append((tc, pts))
    t = t0 + 40 * 10_000_000
    p, q = pose(t)
    track.add(t, p, q)
    recs.append(("P", t, (p, q)))
    return recs, [(pts, np.concatenate(track.at(tc))) for tc, pts in want]


def write_topics(path, recs):
    with open(path, "wb") as f:
        f.write(b"TSDFSTR2")
        for kind, t, v in recs:
            if kind == "P":
                f.write(b"P" + struct.pack("<q3d4d", t, *v[0], *v[1]))
            else:
                rec = dlio_records(v)
                f.write(b"C" + struct.pack("<qQIIi", t, rec.shape[0], 32, 0, 0) + rec.tobytes())


def test_topic_stream_pairs_poses_like_ingest(tmp_path, sim):
    """MapCore (the node's logic, C++) pairs every cloud with the pose track at its stamp exactly
    as tsdf_map.ingest.PoseTrack does: the replay, linked against the oracle library, writes the
    map of integrating the clouds from those origins."""
    lib = oracle.load()
    del lib
    exe = tmp_path / "tsdf_replay_oracle"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", str(exe),
                           os.path.join(HOST, "tsdf_replay.cpp"),
                           "-L" + os.path.dirname(oracle.LIB_PATH), "-ltsdf_oracle",
                           "-Wl,-rpath," + os.path.dirname(oracle.LIB_PATH)])
    recs, want = topic_stream(sim)
    write_topics(tmp_path / "in.topics", recs)
    out = subprocess.run([str(exe), str(tmp_path / "in.topics"), str(tmp_path / "out.bricks")],
                         capture_output=True, text=True, check=True)
    assert "paired 4 clouds, dropped 1 (outside the track) 1 (gap)" in out.stdout
    got = bricks_to_voxels(*read_bricks(tmp_path / "out.bricks"))
    ref = oracle_voxels(want)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


def test_topic_stream_voxblox_depth_weight_pairs_orientation(tmp_path, sim):
    """The slerped orientation reaches the library (tsdf_integrate_pose): Voxblox's 1/z^2 weights
    of a tilting sensor equal integrating the clouds with ingest's poses (the same slerp)."""
    lib = oracle.load()
    del lib
    exe = tmp_path / "tsdf_replay_oracle"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", str(exe),
                           os.path.join(HOST, "tsdf_replay.cpp"),
                           "-L" + os.path.dirname(oracle.LIB_PATH), "-ltsdf_oracle",
                           "-Wl,-rpath," + os.path.dirname(oracle.LIB_PATH)])
    recs, want = topic_stream(sim, tilt=0.7)
    write_topics(tmp_path / "in.topics", recs)
    subprocess.run([str(exe), str(tmp_path / "in.topics"), str(tmp_path / "out.bricks"), "0.05",
                    "0.15", "voxblox"], capture_output=True, text=True, check=True)
    got = bricks_to_voxels(*read_bricks(tmp_path / "out.bricks"))
    ref = oracle_voxels(want, semantics="voxblox", use_const_weight=False)
    assert np.unique(got[2]).size > 50  # depth weights, not counts
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("semantics", ["vdbfusion", "voxblox"])
def test_topic_stream_on_gpu_bitwise(tmp_path, sim, semantics):
    exe = os.path.join(REPO, "noetic-slam_amd", "lib", "tsdf_replay")
    recs, want = topic_stream(sim, tilt=0.7)
    write_topics(tmp_path / "in.topics", recs)
    out = subprocess.run([exe, str(tmp_path / "in.topics"), str(tmp_path / "out.bricks"), "0.05",
                          "0.15", semantics], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = bricks_to_voxels(*read_bricks(tmp_path / "out.bricks"))
    ref = oracle_voxels(want, semantics=semantics, use_const_weight=False)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[2], ref[2])
    assert np.array_equal(got[1].view(np.uint32), ref[1].view(np.uint32))
