"""Ouster sensor input, pinned by the reference's own golden digests.

tests/golden/ouster/ holds five of the reference's recorded frames (src/ouster/ouster-sdk/tests/
pcaps: four UDP lidar profiles, 32 and 128 beams) with the SDK's metadata and *_digest.json — md5
of every LidarScan field of the decoded frame (_digest.py:75-88).  The numpy restatement
(oracle/ouster_ref.py) must reproduce every digest; the GPU decoder must equal it bit for bit (and
so hit the digests itself); the GPU points must equal the fp32 restatement of r dir + off and the
pose; and a frame decoded, projected and integrated on the GPU must give the oracle's field.
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import ouster_ref as R
from conftest import GOLDEN

FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "ouster", "*[0-9].json")))


def load(js):
    from tsdf_map.ouster import OusterFormat, read_pcap
    meta = json.load(open(js))
    fmt = OusterFormat(meta)
    digest = json.load(open(js.replace(".json", "_digest.json")))
    packets = read_pcap(js.replace(".json", ".pcap"), fmt.port)
    return meta, fmt, digest, packets


def pose(k=0):
    c, s = np.cos(0.3 + k), np.sin(0.3 + k)
    return np.array([[c, -s, 0.0, 3.25 + k], [s, c, 0.0, -1.5], [0.0, 0.0, 1.0, 0.8],
                     [0.0, 0.0, 0.0, 1.0]])


def test_fixtures_present():
    assert len(FIXTURES) == 5


@pytest.mark.parametrize("js", FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_reference_decoder_matches_golden_digests(js):
    meta, fmt, digest, packets = load(js)
    ph = R.layout(fmt.profile_name, fmt.h, fmt.columns_per_packet)[5]
    scans = R.decode_frames([p for p in packets if len(p) == ph], fmt.profile_name, fmt.h, fmt.w,
                            fmt.columns_per_packet)
    got, want = R.scan_digest(scans[0]), digest["scans"][0]
    keys = [k for k in want if k in got]
    assert "RANGE" in keys and "FRAME_ID" in keys
    for k in keys:
        assert got[k] == want[k], k


@pytest.mark.parametrize("js", FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_packet_size_and_frames(js):
    from tsdf_map import load_hip_library
    from tsdf_map.ouster import split_frames
    import ctypes as C
    meta, fmt, digest, packets = load(js)
    n = C.c_uint32()
    assert load_hip_library().tsdf_os_packet_bytes(C.byref(fmt.c), C.byref(n)) == 0
    assert n.value == R.layout(fmt.profile_name, fmt.h, fmt.columns_per_packet)[5]
    frames = split_frames(packets, fmt, n.value)
    assert len(frames) == 1 and len(frames[0][1]) == 64
    assert str(frames[0][0]) == digest["scans"][0]["FRAME_ID"]


def _frontend(meta):
    from tsdf_map import HipTSDFVolume
    from tsdf_map.ouster import OusterFrontend
    vol = HipTSDFVolume(0.05, 0.15, max_points=1 << 18, max_bricks=1 << 18, min_range=1e-3)
    return vol, OusterFrontend(vol, meta)


@pytest.mark.gpu
@pytest.mark.parametrize("js", FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_gpu_decode_bitwise_and_digests(js):
    meta, fmt, digest, packets = load(js)
    vol, fe = _frontend(meta)
    (fid, pk), = fe.frames(packets)
    imgs = fe.decode(pk)
    fe.sync()
    ref = R.decode_frames(pk, fmt.profile_name, fmt.h, fmt.w, fmt.columns_per_packet)[0]
    want = digest["scans"][0]
    for f, img in imgs.items():
        g = img.cpu().numpy().view(np.uint32)
        if f not in ref:
            assert not g.any(), f  # field absent from this profile
            continue
        assert np.array_equal(g, ref[f].astype(np.uint32)), f
        md5 = hashlib.md5(g.astype(ref[f].dtype).tobytes()).hexdigest()
        assert md5 == want[f], f


@pytest.mark.gpu
def test_gpu_points_and_field_bitwise():
    import oracle
    js = [f for f in FIXTURES if "OS-2-128" in f][0]
    meta, fmt, digest, packets = load(js)
    vol, fe = _frontend(meta)
    (fid, pk), = fe.frames(packets)
    o = oracle.OracleTSDFVolume(0.05, 0.15, min_range=1e-3)
    ref = R.decode_frames(pk, fmt.profile_name, fmt.h, fmt.w, fmt.columns_per_packet)[0]
    lut_d = fe.lut_dir.cpu().numpy()
    lut_o = fe.lut_off.cpu().numpy()
    for k in range(3):
        P = pose(k)
        imgs, xyz = fe.integrate_frame(pk, P)
        fe.sync()
        # fp32 restatement: r dir + off (0 where r = 0), then ((m0 x + m1 y) + m2 z) + m3
        s = R.cartesian_f32(ref["RANGE"], lut_d, lut_o)
        m = P[:3, :4].astype(np.float32)
        w = np.stack([m[i, 0] * s[:, 0] + m[i, 1] * s[:, 1] + m[i, 2] * s[:, 2] + m[i, 3]
                      for i in range(3)], 1).astype(np.float32)
        g = xyz.cpu().numpy()
        assert np.array_equal(g, w), k
        o.integrate(w, P[:3, 3])
    fe.sync()
    assert o.export_voxels()[0].shape[0] > 10000
    for x, y in zip(vol.export_voxels(), o.export_voxels()):
        assert np.array_equal(x, y)


def test_destaggered_cloud_layout_and_order():
    """48-B ouster_ros::Point records (os_point.h:20-44) in copy_scan_to_cloud_destaggered order."""
    from tsdf_map.ouster import OUSTER_POINT, destaggered_cloud
    assert OUSTER_POINT.itemsize == 48
    assert [OUSTER_POINT.fields[k][1] for k in ("x", "intensity", "t", "reflectivity", "ring",
                                                "ambient", "range")] == [0, 16, 20, 24, 26, 28, 32]
    h, w = 4, 8
    rng = np.arange(h * w, dtype=np.uint32).reshape(h, w) + 100
    xyz = np.stack([rng.reshape(-1)] * 3, 1).astype(np.float32)
    shift = [3, 1, 0, 5]
    ts = np.arange(w, dtype=np.uint64) * 10 + 1000
    c = destaggered_cloud(xyz, rng, rng, rng, rng, shift, ts, scan_ts=1020)
    for u in range(h):
        for v in range(w):
            vs = (v + w - shift[u]) % w
            r = c[u * w + v]
            assert r["range"] == rng[u, vs] and r["x"] == rng[u, vs] and r["ring"] == u
            assert r["t"] == max(int(ts[vs]) - 1020, 0) and r["w"] == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("semantics,min_range", [("vdbfusion_f64", 1.0), ("vdbfusion_f64", 0.0),
                                                 ("vdbfusion", 0.0)])
def test_gpu_destaggered_48b_cloud_bitwise(semantics, min_range):
    """An organized 48-B cloud of the pinned OS-2-128 frame (destaggered, world frame) integrates
    through tsdf_integrate(point_step 48) to the same field, bit for bit, as the staggered packed
    xyz: the per-scan fuse sums each voxel's samples exactly, so point order does not matter.
    In the default mode (vdbfusion_f64) with DLIO's crop box as min_range (odom.cc:114-116: what
    the node receives) and without it, and in the fp32 restatement.  The r = 0 pixels are the
    sensor origin rounded to float: test_oracle_kat.py::test_zero_range_point_is_origin_ray pins
    which modes keep that ray."""
    from tsdf_map import HipTSDFVolume
    from tsdf_map.ouster import destaggered_cloud
    js = [f for f in FIXTURES if "OS-2-128" in f][0]
    meta, fmt, digest, packets = load(js)
    vol, fe = _frontend(meta)
    (fid, pk), = fe.frames(packets)
    ref = R.decode_frames(pk, fmt.profile_name, fmt.h, fmt.w, fmt.columns_per_packet)[0]
    P = pose(1)
    imgs = fe.decode(pk)
    xyz = fe.points(imgs["RANGE"], P)
    fe.sync()
    x = xyz.cpu().numpy()
    cloud = destaggered_cloud(x, ref["RANGE"], ref["SIGNAL"], ref["REFLECTIVITY"], ref["NEAR_IR"],
                              meta["data_format"]["pixel_shift_by_row"])
    kw = dict(max_points=1 << 18, semantics=semantics, min_range=min_range)
    a = HipTSDFVolume(0.05, 0.15, **kw)
    a.integrate_cloud(cloud.tobytes(), cloud.shape[0], 48, 0, P[:3, 3])
    b = HipTSDFVolume(0.05, 0.15, **kw)
    b.integrate(x, P[:3, 3])
    a.sync()
    b.sync()
    ai, as_, aw = a.export_voxels()
    bi, bs, bw = b.export_voxels()
    assert ai.shape[0] > 10000
    assert np.array_equal(ai, bi) and np.array_equal(aw, bw)
    assert np.array_equal(as_.view(np.uint32), bs.view(np.uint32))
    o = oracle.OracleTSDFVolume(0.05, 0.15, semantics=semantics, min_range=min_range)
    o.integrate(x, P[:3, 3])
    oi, os_, ow = o.export_voxels()
    assert np.array_equal(ai, oi) and np.array_equal(aw, ow)
    assert np.array_equal(as_.view(np.uint32), os_.view(np.uint32))
    # which rays count: every pixel at least min_range from the origin; an r = 0 pixel (the origin
    # rounded to float) is dropped by the crop, and kept without it only in the double-precision
    # mode, where it sits a rounding error from the double origin (the KAT's rule)
    nz = int(np.count_nonzero(ref["RANGE"]))
    zero_kept = semantics == "vdbfusion_f64" and min_range == 0.0
    d = np.linalg.norm(x.astype(np.float64) - P[:3, 3], axis=1).astype(np.float32)
    far = int(np.count_nonzero(d >= min_range))
    want = x.shape[0] if zero_kept else (nz if min_range == 0.0 else far)
    assert a.stats()["n_rays_total"] == b.stats()["n_rays_total"] == want
