"""MulRan Ouster scans (`sensor_data/Ouster/<stamp_ns>.bin`), the input of the reference's config 3
(the reader is src/file_player_mulran/src/ROSThread.cpp:470-559).

Each file is a flat array of 16-byte records (x, y, z, intensity as float32, OS1-64 lidar frame).
The reference's loader has three quirks this reader makes explicit instead of copying:
  * it loops `while (!file.eof())`, so the failing read after the last record still pushes one
    point whose fields were never written (ROSThread.cpp:507-516) — here that point is not
    produced; `reference_point_count` reports the count the reference publishes (records + 1);
  * ring = (k % 64) + 1 for the k-th record (:514), whatever the sensor's real beam order is;
  * the per-point time `t` is never set (PointXYZIRT.t uninitialised) — no time is produced.
A trailing partial record (file size not a multiple of 16) is dropped.
"""
import os

import numpy as np

RECORD = 16  # x, y, z, intensity (float32)


def read_bin(path):
    """(points (n, 3) float32, intensity (n,) float32, ring (n,) int32) of one MulRan scan."""
    raw = np.fromfile(path, dtype=np.float32)
    n = raw.size // 4
    rec = raw[:4 * n].reshape(n, 4)
    ring = (np.arange(n, dtype=np.int64) % 64 + 1).astype(np.int32)
    return np.ascontiguousarray(rec[:, :3]), np.ascontiguousarray(rec[:, 3]), ring


def reference_point_count(path):
    """Points the reference's loader publishes for this file: whole records + the eof one."""
    return os.path.getsize(path) // RECORD + 1


def list_scans(folder):
    """[(stamp_ns, path)] of a MulRan `sensor_data/Ouster` folder, in time order."""
    out = []
    for name in os.listdir(folder):
        stem, ext = os.path.splitext(name)
        if ext == ".bin" and stem.isdigit():
            out.append((int(stem), os.path.join(folder, name)))
    return sorted(out)


def write_bin(path, points, intensity=None):
    """Write points (n, 3) (+ intensity) as a MulRan record file (test fixtures, converters)."""
    p = np.asarray(points, np.float32).reshape(-1, 3)
    i = np.zeros(p.shape[0], np.float32) if intensity is None else np.asarray(intensity, np.float32)
    np.concatenate([p, i[:, None]], 1).astype(np.float32).tofile(path)


def to_world(points, pose):
    """Sensor-frame points -> world, pose (4, 4) (or (3, 4)), fp32: ((r0 x + r1 y) + r2 z) + t."""
    m = np.asarray(pose, np.float64)[:3, :4].astype(np.float32)
    p = np.asarray(points, np.float32)
    return np.stack([m[i, 0] * p[:, 0] + m[i, 1] * p[:, 1] + m[i, 2] * p[:, 2] + m[i, 3]
                     for i in range(3)], 1).astype(np.float32)


def integrate_sequence(volume, folder, poses):
    """Integrate a MulRan scan folder; poses: {stamp_ns: (4, 4) sensor -> world} (e.g. DLIO's).
    Scans without a pose are skipped.  Returns the stamps integrated."""
    done = []
    for stamp, path in list_scans(folder):
        if stamp not in poses:
            continue
        pts, _, _ = read_bin(path)
        P = np.asarray(poses[stamp], np.float64)
        volume.integrate(to_world(pts, P), P[:3, 3])
        done.append(stamp)
    return done
