"""CPU restatement of Ouster lidar-packet decoding — TEST INFRASTRUCTURE ONLY (the checker for
noetic-slam_amd/csrc/tsdf_ouster.hip).

Restates, in numpy, what the reference's Ouster SDK does from UDP lidar packets to a LidarScan:
  * packet layouts per UDP profile (src/ouster/ouster-sdk/ouster_client/src/parsing.cpp:42-125:
    legacy / single / dual / low-bandwidth field tables; :150-175 header, column, footer sizes),
  * column header fields (parsing.cpp:370-420: timestamp @0, measurement_id @8, status @10 or the
    legacy footer, frame_id in the packet header @2 or the legacy column header @10),
  * ScanBatcher (ouster_client/src/lidar_scan.cpp:540-633): columns of one frame are placed at
    their measurement_id, invalid columns (status bit 0 clear) are dropped, missing ones stay 0,
  * scan field dtypes (lidar_scan.cpp:52-102).
It is pinned by the reference's own golden digests (tests/pcaps/*_digest.json, md5 of each scan
field's bytes, python/src/ouster/client/_digest.py:75-88), see tests/test_ouster.py.
"""
import hashlib

import numpy as np

# field -> (source bytes, byte offset in the pixel, mask, shift)  [parsing.cpp:42-99]
_LEGACY = {"RANGE": (4, 0, 0x000FFFFF, 0), "REFLECTIVITY": (2, 4, 0, 0), "SIGNAL": (2, 6, 0, 0),
           "NEAR_IR": (2, 8, 0, 0)}
_SINGLE = {"RANGE": (4, 0, 0x0007FFFF, 0), "REFLECTIVITY": (1, 4, 0, 0), "SIGNAL": (2, 6, 0, 0),
           "NEAR_IR": (2, 8, 0, 0)}
_DUAL = {"RANGE": (4, 0, 0x0007FFFF, 0), "REFLECTIVITY": (1, 3, 0, 0),
         "RANGE2": (4, 4, 0x0007FFFF, 0), "REFLECTIVITY2": (1, 7, 0, 0), "SIGNAL": (2, 8, 0, 0),
         "SIGNAL2": (2, 10, 0, 0), "NEAR_IR": (2, 12, 0, 0)}
_LB = {"RANGE": (2, 0, 0x7FFF, -3), "REFLECTIVITY": (1, 2, 0, 0), "NEAR_IR": (1, 3, 0, -4)}

# profile -> (pixel bytes, field table, scan dtypes)  [parsing.cpp:107-118, lidar_scan.cpp:52-102]
PROFILES = {
    "LEGACY": (12, _LEGACY, {"RANGE": np.uint32, "SIGNAL": np.uint32, "NEAR_IR": np.uint32,
                             "REFLECTIVITY": np.uint32}),
    "RNG19_RFL8_SIG16_NIR16": (12, _SINGLE, {"RANGE": np.uint32, "SIGNAL": np.uint16,
                                             "REFLECTIVITY": np.uint16, "NEAR_IR": np.uint16}),
    "RNG19_RFL8_SIG16_NIR16_DUAL": (16, _DUAL, {"RANGE": np.uint32, "RANGE2": np.uint32,
                                                "SIGNAL": np.uint16, "SIGNAL2": np.uint16,
                                                "REFLECTIVITY": np.uint8,
                                                "REFLECTIVITY2": np.uint8, "NEAR_IR": np.uint16}),
    "RNG15_RFL8_NIR8": (4, _LB, {"RANGE": np.uint32, "REFLECTIVITY": np.uint16,
                                 "NEAR_IR": np.uint16}),
}


def layout(profile, pixels_per_column, columns_per_packet):
    """(packet header, column header, column footer, packet footer, column bytes, packet bytes)."""
    legacy = profile == "LEGACY"
    ph, ch, cf, pf = (0, 16, 4, 0) if legacy else (32, 12, 0, 32)
    col = ch + pixels_per_column * PROFILES[profile][0] + cf
    return ph, ch, cf, pf, col, ph + columns_per_packet * col + pf


def _u(buf, off, nbytes):
    return int.from_bytes(bytes(buf[off:off + nbytes]), "little")


def decode_frames(packets, profile, h, w, columns_per_packet):
    """LidarScans (dict field -> (h, w) array, plus FRAME_ID) batched from lidar packets, in
    order; the last frame is returned even if incomplete (as the SDK's scan iterator does)."""
    pixel_bytes, fields, dtypes = PROFILES[profile]
    ph, ch, cf, pf, col, pkt = layout(profile, h, columns_per_packet)
    legacy = profile == "LEGACY"
    scans, cur = [], None
    for p in packets:
        p = np.frombuffer(p, np.uint8)
        assert p.size == pkt
        fid = _u(p, ph + 10, 2) if legacy else _u(p, 2, 2)
        if cur is not None and fid != cur["FRAME_ID"]:
            if cur["FRAME_ID"] == (fid + 1) & 0xFFFF:
                continue  # reordered packet of the previous frame: dropped
            scans.append(cur)
            cur = None
        if cur is None:
            cur = {"FRAME_ID": fid}
            cur.update({f: np.zeros((h, w), dt) for f, dt in dtypes.items()})
        for icol in range(columns_per_packet):
            cb = ph + icol * col
            m_id = _u(p, cb + 8, 2)
            status = _u(p, cb + col - cf, 4) if legacy else (_u(p, cb + 10, 2) & 0xFFFF)
            if m_id >= w or not (status & 1):
                continue
            px = p[cb + ch: cb + ch + h * pixel_bytes].reshape(h, pixel_bytes)
            for f, (nb, off, mask, shift) in fields.items():
                v = np.zeros(h, np.uint64)
                for k in range(nb):
                    v |= px[:, off + k].astype(np.uint64) << np.uint64(8 * k)
                if mask:
                    v &= np.uint64(mask)
                if shift > 0:
                    v >>= np.uint64(shift)
                elif shift < 0:
                    v <<= np.uint64(-shift)
                cur[f][:, m_id] = v.astype(dtypes[f])
    if cur is not None:
        scans.append(cur)
    return scans


def scan_digest(scan):
    """md5 of each field's bytes, the reference's FieldDigest.from_scan (_digest.py:75-88)."""
    out = {"FRAME_ID": str(scan["FRAME_ID"])}
    for f, a in scan.items():
        if f != "FRAME_ID":
            out[f] = hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()
    return out


def cartesian_f32(rng, direction, offset):
    """xyz = r * dir + off per pixel, zero where r = 0 (ouster/impl/cartesian.h:55-70), in fp32
    (the GPU path's precision; the SDK's default is double)."""
    r = rng.reshape(-1).astype(np.float32)
    xyz = r[:, None] * direction.astype(np.float32) + offset.astype(np.float32)
    xyz[r == 0] = 0.0
    return xyz.astype(np.float32)
