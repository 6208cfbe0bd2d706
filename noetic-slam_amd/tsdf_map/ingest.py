"""Bag ingest for the TSDF node slot: DLIO's deskewed world-frame clouds
(robot/dlio/odom_node/pointcloud/deskewed, dliomapping.cpp:44) integrated from the sensor
position at each cloud's stamp.

DLIO stamps the cloud with the scan time (odom.cc:447) but publishes /pose and /odom at the IMU
rate stamped with imu_stamp (odom.cc:318,383), so a cloud's origin is the pose track evaluated at
its stamp: linear in position, slerp in orientation, between the bracketing pose samples; clouds
outside the track or next to a gap wider than `max_gap_ms` are skipped (and counted).
"""
import bisect
import math

import numpy as np

from . import rosbag

DLIO_CLOUD = "/robot/dlio/odom_node/pointcloud/deskewed"
DLIO_POSE = "/robot/dlio/odom_node/pose"


def _slerp(q0, q1, a):
    """Shortest-arc slerp (normalised lerp above a dot of 0.9995), op for op the C++ twin's
    (host/tsdf_map_core.h PoseTrack::slerp: sequential sums, libm acos / sin), so the node and the
    ingest give the same bits."""
    q0 = [float(v) for v in q0]
    q1 = [float(v) for v in q1]
    d = 0.0
    for k in range(4):
        d += q0[k] * q1[k]
    sg = -1.0 if d < 0.0 else 1.0
    q1 = [sg * v for v in q1]
    d *= sg
    if d > 0.9995:
        q = [q0[k] + a * (q1[k] - q0[k]) for k in range(4)]
    else:
        th = math.acos(d)
        x, y, z = math.sin((1.0 - a) * th), math.sin(a * th), math.sin(th)
        q = [(x * q0[k] + y * q1[k]) / z for k in range(4)]
    n = 0.0
    for k in range(4):
        n += q[k] * q[k]
    n = math.sqrt(n)
    return np.array([v / n for v in q], np.float64)


class PoseTrack:
    """Time-stamped poses (position, quaternion x y z w), queried at arbitrary stamps."""

    def __init__(self):
        self.t, self.p, self.q = [], [], []

    def add(self, t_ns, position, quaternion):
        i = bisect.bisect(self.t, t_ns)
        self.t.insert(i, int(t_ns))
        self.p.insert(i, np.asarray(position, np.float64))
        self.q.insert(i, np.asarray(quaternion, np.float64))

    def __len__(self):
        return len(self.t)

    def at(self, t_ns, max_gap_ms=50.0):
        """(position, quaternion) at t_ns, or None outside the track / across a gap."""
        if not self.t or t_ns < self.t[0] or t_ns > self.t[-1]:
            return None
        i = bisect.bisect_left(self.t, t_ns)
        if self.t[i] == t_ns:
            return self.p[i], self.q[i]
        t0, t1 = self.t[i - 1], self.t[i]
        if (t1 - t0) > max_gap_ms * 1e6:
            return None
        a = (t_ns - t0) / float(t1 - t0)
        return self.p[i - 1] + a * (self.p[i] - self.p[i - 1]), _slerp(self.q[i - 1], self.q[i], a)


def load_poses(bag, topic=DLIO_POSE):
    """PoseTrack of a pose topic (geometry_msgs/PoseStamped, nav_msgs/Odometry or nav_msgs/Path,
    whose last message's poses are used)."""
    track, last_path = PoseTrack(), None
    for m in bag.messages({topic}):
        if m.type == "geometry_msgs/PoseStamped":
            hd, p, q = rosbag.decode_pose_stamped(m.data)
            track.add(hd["stamp_ns"], p, q)
        elif m.type == "nav_msgs/Odometry":
            hd, p, q = rosbag.decode_odometry(m.data)
            track.add(hd["stamp_ns"], p, q)
        elif m.type == "nav_msgs/Path":
            last_path = m.data
        else:
            raise ValueError("pose topic %s has type %s" % (topic, m.type))
    if last_path is not None:
        for hd, p, q in rosbag.decode_path(last_path):
            track.add(hd["stamp_ns"], p, q)
    return track


def cloud_xyz_layout(cloud):
    """(xyz_offset, is_f64) of a PointCloud2 whose x, y, z are consecutive float32 or float64."""
    f = {name: (off, dt) for name, off, dt, _ in cloud.fields}
    if not all(k in f for k in "xyz"):
        raise ValueError("cloud has no x, y, z fields")
    (ox, dx), (oy, dy), (oz, dz) = f["x"], f["y"], f["z"]
    size = {7: 4, 8: 8}.get(dx)
    if size is None or dy != dx or dz != dx or oy != ox + size or oz != ox + 2 * size:
        raise ValueError("x, y, z must be consecutive float32 or float64")
    if cloud.is_bigendian:
        raise ValueError("big-endian clouds are not supported")
    return ox, dx == 8


def ingest_bag(volume, path, cloud_topic=DLIO_CLOUD, pose_topic=DLIO_POSE, max_gap_ms=50.0):
    """Integrate every cloud of `cloud_topic` (world frame) from the pose track's pose at its stamp
    (position: the ray origin; orientation: the sensor axes).  `volume` may be a list of sector
    volumes (volume k = sector k of len(volume)): each cloud then goes to all of them through
    tsdf_integrate_sectors (the N-GPU node's path).  Returns (integrated, skipped) cloud counts."""
    from .volume import integrate_sectors_cloud
    sectors = isinstance(volume, (list, tuple))
    bag = rosbag.BagReader(path)
    track = load_poses(bag, pose_topic)
    done = skipped = 0
    for m in bag.messages({cloud_topic}):
        c = rosbag.decode_pointcloud2(m.data)
        pose = track.at(c.header["stamp_ns"], max_gap_ms)
        if pose is None:
            skipped += 1
            continue
        off, f64 = cloud_xyz_layout(c)
        # the full pose (x, y, z, qx, qy, qz, qw): the position is the ray origin, the
        # orientation gives Voxblox's sensor z axis (tsdf_integrate_pose)
        if sectors:
            integrate_sectors_cloud(volume, c.data, c.width * c.height, c.point_step, off,
                                    np.concatenate([pose[0], pose[1]]), xyz_is_f64=f64)
        else:
            volume.integrate_cloud(c.data, c.width * c.height, c.point_step, off,
                                   np.concatenate([pose[0], pose[1]]), xyz_is_f64=f64)
        done += 1
    return done, skipped
