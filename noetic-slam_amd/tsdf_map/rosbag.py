"""ROS-free ROS1 bag (v2.0) reading, so the reference's bag pipelines (BASELINE configs C2 / C5:
an OS1-128 bag through DLIO into the TSDF node) run headless on a GPU box.

Implements the public rosbag 2.0 record format — "#ROSBAG V2.0\\n", then records of
(u32 header length, header fields `name=value`, u32 data length, data); op 0x03 bag header,
0x05 chunk (compression none / bz2; lz4 raises, no lz4 module here), 0x07 connection, 0x02 message
data, 0x04 index, 0x06 chunk info — and the ROS1 wire encoding of the messages this path uses:
sensor_msgs/PointCloud2 (the DLIO deskewed cloud, dliomapping.cpp:44,64-81; dlio::Point layout
dlio.h:85-106), geometry_msgs/PoseStamped (odom.cc:315-356), nav_msgs/Odometry and nav_msgs/Path.
`BagWriter` writes the same format (tests and converters).
"""
import bz2
import struct
from collections import namedtuple

MAGIC = b"#ROSBAG V2.0\n"
OP_MSG, OP_BAG_HEADER, OP_INDEX, OP_CHUNK, OP_CHUNK_INFO, OP_CONNECTION = 2, 3, 4, 5, 6, 7

Connection = namedtuple("Connection", "conn topic type md5sum")
Message = namedtuple("Message", "topic type time_ns data")


def _fields(buf):
    out, i = {}, 0
    while i < len(buf):
        n = struct.unpack_from("<I", buf, i)[0]
        k, _, v = buf[i + 4: i + 4 + n].partition(b"=")
        out[k.decode()] = v
        i += 4 + n
    return out


def _records(buf, pos=0):
    while pos + 4 <= len(buf):
        hl = struct.unpack_from("<I", buf, pos)[0]
        h = _fields(buf[pos + 4: pos + 4 + hl])
        pos += 4 + hl
        dl = struct.unpack_from("<I", buf, pos)[0]
        yield h, buf[pos + 4: pos + 4 + dl]
        pos += 4 + dl


class BagReader:
    """Messages of a bag in file order (chunks are decompressed as met)."""

    def __init__(self, path):
        with open(path, "rb") as f:
            self.buf = f.read()
        if not self.buf.startswith(MAGIC):
            raise ValueError("%s: not a ROS bag v2.0" % path)
        self.connections = {}

    def _conn(self, h, data):
        c = _fields(data)
        cid = struct.unpack("<I", h["conn"])[0]
        self.connections[cid] = Connection(cid, h["topic"].decode(), c.get("type", b"").decode(),
                                           c.get("md5sum", b"").decode())

    def messages(self, topics=None):
        for h, data in _records(self.buf, len(MAGIC)):
            op = h.get("op", b"\x00")[0]
            if op == OP_CONNECTION:
                self._conn(h, data)
            elif op == OP_CHUNK:
                comp = h.get("compression", b"none").decode()
                if comp == "bz2":
                    data = bz2.decompress(data)
                elif comp != "none":
                    raise NotImplementedError("bag chunk compression %r" % comp)
                for h2, d2 in _records(data):
                    op2 = h2.get("op", b"\x00")[0]
                    if op2 == OP_CONNECTION:
                        self._conn(h2, d2)
                    elif op2 == OP_MSG:
                        m = self._msg(h2, d2)
                        if topics is None or m.topic in topics:
                            yield m
            elif op == OP_MSG:
                m = self._msg(h, data)
                if topics is None or m.topic in topics:
                    yield m

    def _msg(self, h, data):
        c = self.connections[struct.unpack("<I", h["conn"])[0]]
        sec, nsec = struct.unpack("<II", h["time"])
        return Message(c.topic, c.type, sec * 1000000000 + nsec, data)


# ---- ROS1 message encoding -------------------------------------------------------------------

class _R:
    def __init__(self, b):
        self.b, self.i = b, 0

    def u(self, fmt):
        v = struct.unpack_from("<" + fmt, self.b, self.i)
        self.i += struct.calcsize("<" + fmt)
        return v if len(v) > 1 else v[0]

    def s(self):
        n = self.u("I")
        v = self.b[self.i: self.i + n]
        self.i += n
        return v


def _header(r):
    seq, sec, nsec = r.u("III")
    return {"seq": seq, "stamp_ns": sec * 1000000000 + nsec, "frame_id": r.s().decode()}


PointCloud2 = namedtuple("PointCloud2", "header height width fields is_bigendian point_step "
                                        "row_step data is_dense")


def decode_pointcloud2(b):
    r = _R(b)
    hd = _header(r)
    h, w = r.u("II")
    fields = []
    for _ in range(r.u("I")):
        name = r.s().decode()
        off = r.u("I")
        dt = r.u("B")
        cnt = r.u("I")
        fields.append((name, off, dt, cnt))
    big = r.u("B")
    step, row = r.u("II")
    data = r.s()
    dense = r.u("B")
    return PointCloud2(hd, h, w, fields, big, step, row, data, dense)


def decode_pose_stamped(b):
    """geometry_msgs/PoseStamped -> (header, position (3,), quaternion (x, y, z, w))."""
    r = _R(b)
    hd = _header(r)
    p = r.u("3d")
    q = r.u("4d")
    return hd, p, q


def decode_odometry(b):
    """nav_msgs/Odometry -> (header, position, quaternion) (child frame, covariances, twist
    skipped)."""
    r = _R(b)
    hd = _header(r)
    r.s()  # child_frame_id
    p = r.u("3d")
    q = r.u("4d")
    return hd, p, q


def decode_path(b):
    """nav_msgs/Path -> [(header, position, quaternion)] of its poses."""
    r = _R(b)
    _header(r)
    out = []
    for _ in range(r.u("I")):
        hd = _header(r)
        out.append((hd, r.u("3d"), r.u("4d")))
    return out


def _w_header(stamp_ns, frame_id, seq=0):
    f = frame_id.encode()
    return struct.pack("<III", seq, stamp_ns // 1000000000, stamp_ns % 1000000000) + \
        struct.pack("<I", len(f)) + f


def encode_pointcloud2(stamp_ns, frame_id, xyz, point_step=32, xyz_offset=0):
    """A PointCloud2 of float32 x, y, z (dlio::Point layout by default: 32-B points)."""
    import numpy as np
    xyz = np.asarray(xyz, np.float32)
    n = xyz.shape[0]
    rec = np.zeros((n, point_step), np.uint8)
    rec[:, xyz_offset: xyz_offset + 12] = xyz.view(np.uint8).reshape(n, 12)
    fields = [("x", xyz_offset, 7, 1), ("y", xyz_offset + 4, 7, 1), ("z", xyz_offset + 8, 7, 1)]
    out = _w_header(stamp_ns, frame_id) + struct.pack("<II", 1, n) + struct.pack("<I", len(fields))
    for name, off, dt, cnt in fields:
        out += struct.pack("<I", len(name)) + name.encode() + struct.pack("<IBI", off, dt, cnt)
    data = rec.tobytes()
    return out + struct.pack("<BII", 0, point_step, point_step * n) + \
        struct.pack("<I", len(data)) + data + struct.pack("<B", 1)


def encode_pose_stamped(stamp_ns, frame_id, position, quaternion):
    return _w_header(stamp_ns, frame_id) + struct.pack("<3d", *position) + \
        struct.pack("<4d", *quaternion)


class BagWriter:
    """Minimal rosbag v2.0 writer: one chunk per `chunk_messages` messages (none or bz2)."""

    TYPES = {"sensor_msgs/PointCloud2": "1158d486dd51d683ce2f1be655c3c181",
             "geometry_msgs/PoseStamped": "d3812c3cbc69362b77dc0b19b345f8f5"}

    def __init__(self, path, compression="none", chunk_messages=16):
        self.f = open(path, "wb")
        self.comp, self.per = compression, chunk_messages
        self.conns, self.pending = {}, []
        self.f.write(MAGIC)
        self._record({"op": bytes([OP_BAG_HEADER]), "index_pos": struct.pack("<Q", 0),
                      "conn_count": struct.pack("<I", 0), "chunk_count": struct.pack("<I", 0)},
                     b" " * (4096 - 69))

    @staticmethod
    def _hdr(fields):
        out = b""
        for k, v in fields.items():
            item = k.encode() + b"=" + (v if isinstance(v, bytes) else v.encode())
            out += struct.pack("<I", len(item)) + item
        return out

    @classmethod
    def _rec(cls, fields, data):
        h = cls._hdr(fields)
        return struct.pack("<I", len(h)) + h + struct.pack("<I", len(data)) + data

    def _record(self, fields, data):
        self.f.write(self._rec(fields, data))

    def write(self, topic, msg_type, time_ns, data):
        if topic not in self.conns:
            self.conns[topic] = (len(self.conns), msg_type)
        self.pending.append((topic, time_ns, data))
        if len(self.pending) >= self.per:
            self._flush()

    def _flush(self):
        if not self.pending:
            return
        body = b""
        for topic in sorted({t for t, _, _ in self.pending}):
            cid, typ = self.conns[topic]
            body += self._rec({"op": bytes([OP_CONNECTION]), "conn": struct.pack("<I", cid),
                               "topic": topic},
                              self._hdr({"topic": topic, "type": typ,
                                         "md5sum": self.TYPES.get(typ, "*")}))
        for topic, t, data in self.pending:
            body += self._rec({"op": bytes([OP_MSG]), "conn": struct.pack("<I", self.conns[topic][0]),
                               "time": struct.pack("<II", t // 1000000000, t % 1000000000)}, data)
        payload = bz2.compress(body) if self.comp == "bz2" else body
        self._record({"op": bytes([OP_CHUNK]), "compression": self.comp,
                      "size": struct.pack("<I", len(body))}, payload)
        self.pending = []

    def close(self):
        self._flush()
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
