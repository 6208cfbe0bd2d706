"""Synthetic Ouster scans in DLIO's output contract (world-frame xyz + scan origin).

Geometry follows the reference's Ouster SDK projection:
  * XYZ LUT — `make_xyz_lut` (src/ouster/ouster-sdk/ouster_client/src/lidar_scan.cpp:297-382):
    encoder angle  theta_e = 2*pi - v*2*pi/W,  azimuth theta_a = -az[u],  altitude phi = alt[u];
    direction = (cos(theta_e+theta_a) cos(phi), sin(theta_e+theta_a) cos(phi), sin(phi));
    offset    = (cos(theta_e) b - dir_x n, sin(theta_e) b - dir_y n, -dir_z n)   (b = n =
    lidar_origin_to_beam_origin_mm since beam_to_lidar(2,3) = 0, types.cpp:254-262);
    both scaled by range_unit = 0.001 (types.h:42); transform = identity (lidar frame).
  * projection — `cartesianT` (.../include/ouster/impl/cartesian.h:35-72): xyz = r*dir + offset for
    r != 0, and (0,0,0) for r == 0.
Ranges are integer millimetres (uint32), as the sensor reports them.

Scene: ground plane z = -1.8 m, a vertical cylinder wall of radius 25 m around
the world origin (every ray returns), plus four pillars so the map has interior structure.  The
sensor drives a circle of radius 8 m at 1 m/s (10 Hz -> 0.1 m per scan), heading tangent.

Points are emitted column-major (all beams of column 0, then column 1, ...), i.e. in scan-time
order as DLIO's deskew leaves them (odom.cc:635-636); zero-range returns are dropped as DLIO's
crop box does (odom.cc:114-116).  Output is float32 world-frame xyz, the dlio::Point x,y,z.
"""
import json
import math
import os

import numpy as np

_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden")

GROUND_Z = -1.8
WALL_R = 25.0
PILLARS = ((6.0, 14.0, 0.6), (-12.0, 3.0, 0.8), (2.0, -15.0, 0.5), (-16.0, -10.0, 1.0))
CIRCLE_R = 8.0


def load_beams(name="os1_128_1024", path=None):
    path = path or os.path.join(_GOLDEN, "ouster_beams.json")
    with open(path) as f:
        return json.load(f)[name]


def make_xyz_lut(w, h, lidar_origin_to_beam_origin_mm, altitude_deg, azimuth_deg):
    """LUT per lidar_scan.cpp:297-382, identity transform. Returns (direction, offset) as
    (h*w, 3) float64 arrays in row-major pixel order i = u*w + v; direction is per millimetre."""
    v = np.arange(w, dtype=np.float64)[None, :]
    alt = np.asarray(altitude_deg, dtype=np.float64)[:, None] * math.pi / 180.0
    az = -np.asarray(azimuth_deg, dtype=np.float64)[:, None] * math.pi / 180.0
    enc = 2.0 * math.pi - v * (2.0 * math.pi / w)
    enc = np.broadcast_to(enc, (h, w))
    alt = np.broadcast_to(alt, (h, w))
    az = np.broadcast_to(az, (h, w))
    d = np.stack([np.cos(enc + az) * np.cos(alt), np.sin(enc + az) * np.cos(alt), np.sin(alt)], -1)
    b = float(lidar_origin_to_beam_origin_mm)
    n = b  # beam_to_lidar(2,3) == 0 -> euclidean distance is the x offset
    off = np.stack([np.cos(enc) * b - d[..., 0] * n, np.sin(enc) * b - d[..., 1] * n,
                    -d[..., 2] * n], -1)
    return (d * 0.001).reshape(-1, 3), (off * 0.001).reshape(-1, 3)


def cartesian(range_mm, direction, offset):
    """cartesian.h:35-72: r*dir + offset, r == 0 -> 0."""
    r = range_mm.reshape(-1).astype(np.float64)[:, None]
    xyz = r * direction + offset
    xyz[r[:, 0] == 0] = 0.0
    return xyz


def pose_on_circle(k, hz=10.0, speed=1.0, radius=CIRCLE_R):
    """Scan k's pose: position on the circle, yaw tangent to it."""
    ang = speed * (k / hz) / radius
    pos = np.array([radius * math.cos(ang), radius * math.sin(ang), 0.0])
    yaw = ang + math.pi / 2.0
    return pos, yaw


def _rot_z(yaw):
    c, s = math.cos(yaw), math.sin(yaw)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def _intersect(o, d):
    """Nearest positive hit of rays o + t d (world frame, (n,3)) with the scene; inf if none."""
    t = np.full(o.shape[0], np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        tg = (GROUND_Z - o[:, 2]) / d[:, 2]
        t = np.where((tg > 0) & np.isfinite(tg), np.minimum(t, tg), t)

        def cyl(cx, cy, r, inside):
            ox, oy = o[:, 0] - cx, o[:, 1] - cy
            a = d[:, 0] ** 2 + d[:, 1] ** 2
            b = 2 * (ox * d[:, 0] + oy * d[:, 1])
            c = ox * ox + oy * oy - r * r
            disc = b * b - 4 * a * c
            sq = np.sqrt(np.maximum(disc, 0))
            t_far = (-b + sq) / (2 * a)
            t_near = (-b - sq) / (2 * a)
            th = t_far if inside else np.where(t_near > 0, t_near, np.inf)
            return np.where((disc >= 0) & (a > 0) & (th > 0), th, np.inf)

        t = np.minimum(t, cyl(0.0, 0.0, WALL_R, True))
        for (cx, cy, r) in PILLARS:
            t = np.minimum(t, cyl(cx, cy, r, False))
    return t


class OusterSim:
    """Synthetic spinning LiDAR (OS-1-128 beams) over the analytic scene."""

    def __init__(self, beams="os1_128_1024", columns=None, noise_m=0.01, hz=10.0):
        meta = load_beams(beams)
        self.w = int(columns or meta["columns_per_frame"])
        self.h = int(meta["pixels_per_column"])
        self.dir, self.off = make_xyz_lut(self.w, self.h, meta["lidar_origin_to_beam_origin_mm"],
                                          meta["beam_altitude_angles"],
                                          meta["beam_azimuth_angles"])
        # unit directions for intersection (dir is per-mm)
        self.udir = self.dir / np.linalg.norm(self.dir, axis=1, keepdims=True)
        self.noise_m = float(noise_m)
        self.hz = float(hz)
        # column-major emission order: pixel i = u*w + v, emit v outer, u inner
        self.order = (np.arange(self.h)[None, :] * self.w + np.arange(self.w)[:, None]).reshape(-1)

    def range_image(self, pos, yaw, seed=None):
        """(h, w) uint32 millimetre ranges for the sensor at pos/yaw."""
        R = _rot_z(yaw)
        o = self.off @ R.T + pos
        d = self.udir @ R.T
        t = _intersect(o, d)
        if self.noise_m > 0 and seed is not None:
            t = t + np.random.default_rng(seed).normal(0.0, self.noise_m, t.shape)
        # range measured along dir from the beam origin, in mm (same unit the LUT expects)
        r = np.where(np.isfinite(t) & (t > 0), np.rint(t * 1000.0), 0.0)
        r = np.minimum(r, 2 ** 20 - 1)  # 20-bit range field (RNG19 profiles are narrower)
        return r.astype(np.uint32).reshape(self.h, self.w)

    def scan(self, k):
        """Scan k of the circular trajectory: (float32 (n,3) world xyz, float64 origin (3,))."""
        pos, yaw = pose_on_circle(k, hz=self.hz)
        rng = self.range_image(pos, yaw, seed=k)
        xyz = cartesian(rng, self.dir, self.off)  # lidar frame
        keep = rng.reshape(-1) != 0
        sel = self.order[keep[self.order]]
        pts = xyz[sel] @ _rot_z(yaw).T + pos
        return pts.astype(np.float32), pos.astype(np.float64)

    def scans(self, k0, n):
        return [self.scan(k) for k in range(k0, k0 + n)]


class TorchOusterSim:
    """The same sensor, scene and trajectory evaluated in torch float64 on a device — used by
    bench.py to synthesise thousands of scans in seconds.  Same equations as OusterSim (the noise
    stream differs: torch's generator instead of numpy's), so parity tests use OusterSim."""

    def __init__(self, device, beams="os1_128_1024", noise_m=0.01, hz=10.0):
        import torch
        self.torch = torch
        base = OusterSim(beams, noise_m=noise_m, hz=hz)
        self.w, self.h, self.hz, self.noise_m = base.w, base.h, base.hz, base.noise_m
        self.device = device
        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=device)  # noqa: E731
        self.dir, self.off, self.udir = t(base.dir), t(base.off), t(base.udir)
        self.order = torch.as_tensor(base.order, device=device)

    def _intersect(self, o, d):
        torch = self.torch
        inf = torch.full_like(o[:, 0], float("inf"))
        tg = (GROUND_Z - o[:, 2]) / d[:, 2]
        t = torch.where((tg > 0) & torch.isfinite(tg), tg, inf)

        def cyl(cx, cy, r, inside):
            ox, oy = o[:, 0] - cx, o[:, 1] - cy
            a = d[:, 0] ** 2 + d[:, 1] ** 2
            b = 2 * (ox * d[:, 0] + oy * d[:, 1])
            c = ox * ox + oy * oy - r * r
            disc = b * b - 4 * a * c
            sq = torch.sqrt(torch.clamp(disc, min=0))
            th = (-b + sq) / (2 * a) if inside else (-b - sq) / (2 * a)
            return torch.where((disc >= 0) & (a > 0) & (th > 0), th, inf)

        t = torch.minimum(t, cyl(0.0, 0.0, WALL_R, True))
        for (cx, cy, r) in PILLARS:
            t = torch.minimum(t, cyl(cx, cy, r, False))
        return t

    def scan(self, k):
        """(float32 (n,3) world xyz on device, float64 origin (3,) numpy)."""
        torch = self.torch
        pos, yaw = pose_on_circle(k, hz=self.hz)
        R = torch.as_tensor(_rot_z(yaw), dtype=torch.float64, device=self.device)
        P = torch.as_tensor(pos, dtype=torch.float64, device=self.device)
        t = self._intersect(self.off @ R.T + P, self.udir @ R.T)
        if self.noise_m > 0:
            g = torch.Generator(device=self.device)
            g.manual_seed(int(k))
            t = t + self.noise_m * torch.randn(t.shape, generator=g, dtype=torch.float64,
                                               device=self.device)
        r = torch.where(torch.isfinite(t) & (t > 0), torch.round(t * 1000.0),
                        torch.zeros_like(t)).clamp(max=2 ** 20 - 1)
        xyz = r[:, None] * self.dir + self.off
        keep = (r != 0)[self.order]
        sel = self.order[keep]
        pts = xyz[sel] @ R.T + P
        return pts.to(torch.float32), pos.astype(np.float64)


def single_ray_scan(points, origin=(0.0, 0.0, 0.0)):
    """Helper for KATs: float32 points + float64 origin."""
    return np.asarray(points, np.float32).reshape(-1, 3), np.asarray(origin, np.float64)
