"""Ouster sensor input for the MI355X backend.

The reference's sensor driver is the Ouster SDK (src/ouster/ouster-sdk): UDP lidar packets are
batched into a LidarScan (ouster_client/src/lidar_scan.cpp:540-633 ScanBatcher) and turned into
points with the xyz LUT (lidar_scan.cpp:297-382 make_xyz_lut, ouster/impl/cartesian.h).  Here the
raw packets of a frame go to the GPU as bytes (the same 1.6 MB per 128 x 1024 frame as its xyz),
are decoded there (tsdf_os_decode_device), turned into world points with the scan pose
(tsdf_os_cartesian_device) and integrated, without a host-side point cloud.

`read_pcap` / `split_frames` are the host side of a recorded stream (libpcap container, UDP
payloads on the lidar port; frames grouped by frame_id, reordered packets of the previous frame
dropped, as the SDK's batcher does).
"""
import ctypes as C
import struct

import numpy as np

from . import _abi
from .scan_gen import make_xyz_lut


def read_pcap(path, port=7502):
    """UDP payloads sent to `port` in a classic libpcap file (Ethernet / IPv4 / UDP), in order."""
    with open(path, "rb") as f:
        b = f.read()
    magic = struct.unpack_from("<I", b, 0)[0]
    if magic not in (0xA1B2C3D4, 0xA1B23C4D):
        raise ValueError("%s: not a little-endian libpcap file" % path)
    out, off = [], 24
    while off + 16 <= len(b):
        incl = struct.unpack_from("<I", b, off + 8)[0]
        d = b[off + 16: off + 16 + incl]
        off += 16 + incl
        if len(d) < 42 or d[12:14] != b"\x08\x00" or d[23] != 17:  # IPv4 / UDP only
            continue
        ihl = (d[14] & 15) * 4
        _, dport, ulen = struct.unpack_from(">HHH", d, 14 + ihl)
        if dport == port:
            out.append(bytes(d[14 + ihl + 8: 14 + ihl + ulen]))
    return out


class OusterFormat:
    """Sensor metadata (the SDK's metadata JSON) -> tsdf_os_format, LUT inputs."""

    def __init__(self, meta):
        df = meta["data_format"]
        self.profile_name = df.get("udp_profile_lidar") or "LEGACY"
        if self.profile_name not in _abi.OS_PROFILES:
            raise ValueError("unsupported Ouster lidar profile %s" % self.profile_name)
        self.h = int(df["pixels_per_column"])
        self.w = int(df["columns_per_frame"])
        self.columns_per_packet = int(df["columns_per_packet"])
        self.port = int(meta.get("udp_port_lidar", 7502))
        self.altitude = np.asarray(meta["beam_altitude_angles"], np.float64)
        self.azimuth = np.asarray(meta["beam_azimuth_angles"], np.float64)
        self.beam_origin_mm = float(meta["lidar_origin_to_beam_origin_mm"])
        self.c = _abi.OsFormat(_abi.OS_PROFILES[self.profile_name], self.h,
                               self.columns_per_packet, self.w)

    @property
    def legacy(self):
        return self.profile_name == "LEGACY"

    def frame_id(self, packet):
        """parsing.cpp:281-288: packet header @2, or the first column's header @10 (legacy)."""
        return struct.unpack_from("<H", packet, 10 if self.legacy else 2)[0]


def split_frames(packets, fmt, packet_bytes):
    """Lidar packets -> [[packets of one frame], ...] in stream order (ScanBatcher's grouping)."""
    frames, cur, fid = [], [], None
    for p in packets:
        if len(p) != packet_bytes:
            continue
        f = fmt.frame_id(p)
        if fid is not None and f != fid:
            if fid == (f + 1) & 0xFFFF:
                continue  # reordered packet of the previous frame
            frames.append((fid, cur))
            cur = []
        fid = f
        cur.append(p)
    if cur:
        frames.append((fid, cur))
    return frames


# ouster_ros::Point (reference include/ouster_ros/os_point.h:20-44): PCL_ADD_POINT4D (x, y, z, 1),
# intensity, t (ns since the scan), reflectivity, ring, ambient, range (mm); EIGEN_ALIGN16 -> 48 B.
OUSTER_POINT = np.dtype({
    "names": ["x", "y", "z", "w", "intensity", "t", "reflectivity", "ring", "ambient", "range"],
    "formats": [np.float32, np.float32, np.float32, np.float32, np.float32, np.uint32, np.uint16,
                np.uint16, np.uint16, np.uint32],
    "offsets": [0, 4, 8, 12, 16, 20, 24, 26, 28, 32],
    "itemsize": 48})


def destaggered_cloud(xyz, rng, signal, reflectivity, near_ir, pixel_shift_by_row,
                      timestamps=None, scan_ts=0):
    """The organized cloud of ouster_ros' copy_scan_to_cloud_destaggered (reference
    src/ouster/src/os_ros.cpp:195-229): point (u, v) of the h x w cloud (row u = beam, tgt index
    u w + v) takes pixel v_shift = (v + w - pixel_shift_by_row[u]) % w of the staggered images and
    of `xyz` (h w x 3, staggered row-major, as the LUT projection gives it); t = column
    timestamp - scan_ts (0 if earlier); ring = u.  Host arrays in, a 48-B OUSTER_POINT array out
    (tsdf_integrate with point_step 48, xyz_offset 0 takes it as is)."""
    rng = np.asarray(rng)
    h, w = rng.shape
    shift = np.asarray(pixel_shift_by_row, np.int64).reshape(h)
    v = np.arange(w)
    v_shift = (v[None, :] + w - shift[:, None]) % w           # (h, w)
    src = (np.arange(h)[:, None] * w + v_shift).reshape(-1)   # staggered source of each target
    out = np.zeros(h * w, OUSTER_POINT)
    p = np.asarray(xyz, np.float32).reshape(h * w, 3)[src]
    out["x"], out["y"], out["z"], out["w"] = p[:, 0], p[:, 1], p[:, 2], 1.0
    out["intensity"] = np.asarray(signal).reshape(-1)[src].astype(np.float32)
    if timestamps is not None:
        ts = np.asarray(timestamps, np.uint64)[v_shift].reshape(-1)
        out["t"] = np.where(ts > scan_ts, ts - np.uint64(scan_ts), 0).astype(np.uint32)
    out["reflectivity"] = np.asarray(reflectivity).reshape(-1)[src].astype(np.uint16)
    out["ring"] = np.repeat(np.arange(h, dtype=np.uint16), w)
    out["ambient"] = np.asarray(near_ir).reshape(-1)[src].astype(np.uint16)
    out["range"] = rng.reshape(-1)[src].astype(np.uint32)
    return out


class OusterFrontend:
    """Packets of one frame -> device field images -> world points -> the volume, on the GPU.
    `volume` is a HipTSDFVolume; the work runs on its context's stream, so call sync() before
    reading the returned tensors with torch."""

    FIELDS = ("RANGE", "SIGNAL", "REFLECTIVITY", "NEAR_IR")

    def __init__(self, volume, meta):
        import torch
        self.vol = volume
        self.fmt = OusterFormat(meta)
        n = C.c_uint32()
        rc = volume._lib.tsdf_os_packet_bytes(C.byref(self.fmt.c), C.byref(n))
        if rc != _abi.TSDF_OK:
            raise ValueError("bad Ouster format")
        self.packet_bytes = n.value
        self.device = torch.device("cuda", volume.params.device_id)
        d, o = make_xyz_lut(self.fmt.w, self.fmt.h, self.fmt.beam_origin_mm, self.fmt.altitude,
                            self.fmt.azimuth)
        self.lut_dir = torch.from_numpy(d.astype(np.float32)).to(self.device)
        self.lut_off = torch.from_numpy(o.astype(np.float32)).to(self.device)
        self._alive = []  # device buffers the library's stream may still read (until sync())
        torch.cuda.synchronize(self.device)  # the LUT upload ran on torch's stream

    def frames(self, packets):
        return split_frames(packets, self.fmt, self.packet_bytes)

    def decode(self, packets):
        """dict field -> (h, w) uint32 torch tensor on the device (staggered, SDK field values)."""
        import torch
        buf = torch.from_numpy(np.frombuffer(b"".join(packets), np.uint8).copy()).to(self.device)
        torch.cuda.current_stream(self.device).synchronize()  # upload (torch's stream) done
        imgs = {f: torch.empty((self.fmt.h, self.fmt.w), dtype=torch.int32, device=self.device)
                for f in self.FIELDS}
        ptr = [C.c_void_p(imgs[f].data_ptr()) for f in self.FIELDS]
        self.vol._check(self.vol._lib.tsdf_os_decode_device(
            self.vol._ctx, C.byref(self.fmt.c), C.c_void_p(buf.data_ptr()), len(packets), *ptr),
            "os_decode")
        self._alive += [buf] + list(imgs.values())
        return imgs

    def points(self, range_img, pose):
        """World points (h*w, 3) float32 on the device; pose: (4, 4) (or (3, 4)) sensor -> world."""
        import torch
        m = np.ascontiguousarray(np.asarray(pose, np.float64)[:3, :4]).reshape(12)
        xyz = torch.empty((range_img.numel(), 3), dtype=torch.float32, device=self.device)
        self.vol._check(self.vol._lib.tsdf_os_cartesian_device(
            self.vol._ctx, C.c_void_p(range_img.data_ptr()), range_img.numel(),
            C.c_void_p(self.lut_dir.data_ptr()), C.c_void_p(self.lut_off.data_ptr()),
            m.ctypes.data_as(C.POINTER(C.c_double)), C.c_void_p(xyz.data_ptr())), "os_cartesian")
        self._alive.append(xyz)
        return xyz

    def integrate_frame(self, packets, pose):
        """Decode, project and integrate one frame seen from the pose's translation."""
        imgs = self.decode(packets)
        xyz = self.points(imgs["RANGE"], pose)
        self.vol.integrate_device(xyz.data_ptr(), xyz.shape[0], np.asarray(pose, np.float64)[:3, 3])
        return imgs, xyz

    def sync(self):
        """Wait for the volume's queued work; the frontend's device buffers are released."""
        self.vol.sync()
        self._alive.clear()
