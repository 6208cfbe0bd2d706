"""ctypes binding of the CPU oracle (oracle/build/libtsdf_oracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, as the
checker or the timed CPU baseline; nothing in noetic-slam_amd/ imports it.  The library exports the
same C-ABI as libtsdf_hip.so (include/tsdf_hip.h, minus the device-pointer entry points), so the
oracle is driven through the very same host wrapper class as the GPU backend.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "noetic-slam_amd"))

from tsdf_map import _abi  # noqa: E402
from tsdf_map.volume import TSDFVolume  # noqa: E402

LIB_PATH = os.path.join(HERE, "build", "libtsdf_oracle.so")
MODE_SCAN_FUSED = 0
MODE_SEQUENTIAL = 1
MODE_VDB_LITERAL = 2  # VDBFusion's own precisions (double sdf, Ray<float> DDA), per-sample update
HOST_ONLY = ("tsdf_integrate_device", "tsdf_integrate_batch_device",
             "tsdf_integrate_batch_device_pose", "tsdf_set_profiling",
             "tsdf_set_metrics_log",
             "tsdf_os_packet_bytes", "tsdf_os_decode_device", "tsdf_os_cartesian_device")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = _abi.declare(C.CDLL(LIB_PATH), optional=HOST_ONLY)
        lib.tsdf_oracle_set_mode.restype = C.c_int
        lib.tsdf_oracle_set_mode.argtypes = [C.c_void_p, C.c_int]
        lib.tsdf_oracle_set_threads.restype = C.c_int
        lib.tsdf_oracle_set_threads.argtypes = [C.c_void_p, C.c_int]
        lib.tsdf_oracle_num_voxels.restype = C.c_uint64
        lib.tsdf_oracle_num_voxels.argtypes = [C.c_void_p]
        lib.tsdf_oracle_export_voxels.restype = C.c_int
        lib.tsdf_oracle_export_voxels.argtypes = [C.c_void_p, _abi.I3, _abi.FP, _abi.FP,
                                                  C.c_uint64, _abi.U64P]
        lib.tsdf_oracle_ray_voxels.restype = C.c_int64
        lib.tsdf_oracle_ray_voxels.argtypes = [C.c_void_p, _abi.FP, _abi.D3, _abi.I3, _abi.FP,
                                               C.c_uint64]
        _lib = lib
    return _lib


class OracleTSDFVolume(TSDFVolume):
    """The CPU restatement behind the same host interface as HipTSDFVolume."""

    def __init__(self, voxel_size, sdf_trunc, space_carving=False, mode=MODE_SCAN_FUSED, threads=1,
                 **kw):
        super().__init__(load(), voxel_size, sdf_trunc, space_carving, **kw)
        self._check(self._lib.tsdf_oracle_set_mode(self._ctx, mode), "set_mode")
        # threads > 1: the partitioned multi-threaded scan-fused mode (same field, bit for bit)
        self._check(self._lib.tsdf_oracle_set_threads(self._ctx, int(threads)), "set_threads")

    def export_voxels(self):
        n = int(self._lib.tsdf_oracle_num_voxels(self._ctx))
        ijk = np.empty((n, 3), np.int32)
        s = np.empty(n, np.float32)
        w = np.empty(n, np.float32)
        out = C.c_uint64()
        self._check(self._lib.tsdf_oracle_export_voxels(self._ctx, ijk.ctypes.data_as(_abi.I3),
                                                        s.ctypes.data_as(_abi.FP),
                                                        w.ctypes.data_as(_abi.FP), n,
                                                        C.byref(out)), "export_voxels")
        return ijk, s, w

    def ray_voxels(self, point, origin, cap=1 << 16):
        """Gated voxels of one ray in DDA order: (ijk (k,3), sdf (k,)); None if filtered out."""
        p = np.ascontiguousarray(point, np.float32).reshape(3)
        o = np.ascontiguousarray(origin, np.float64).reshape(3)
        ijk = np.empty((cap, 3), np.int32)
        s = np.empty(cap, np.float32)
        k = self._lib.tsdf_oracle_ray_voxels(self._ctx, p.ctypes.data_as(_abi.FP),
                                             o.ctypes.data_as(_abi.D3),
                                             ijk.ctypes.data_as(_abi.I3), s.ctypes.data_as(_abi.FP),
                                             cap)
        if k < 0:
            return None
        return ijk[:min(k, cap)], s[:min(k, cap)]
