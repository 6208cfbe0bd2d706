"""Loader for the in-tree HIP library (noetic-slam_amd/lib/libtsdf_hip.so)."""
import ctypes
import os

from . import _abi

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_ROOT, "lib")
HIP_LIB = os.path.join(LIB_DIR, "libtsdf_hip.so")

ABI_VERSION = 10  # TSDF_ABI_VERSION of include/tsdf_hip.h

_hip = None


def load_hip_library(path=None):
    """Load and declare libtsdf_hip.so; raises (never falls back) when it is missing."""
    global _hip
    if _hip is not None and path is None:
        return _hip
    # TSDF_HIP_LIB: load another build of the same ABI (A/B kernel experiments, profiles/)
    p = path or os.environ.get("TSDF_HIP_LIB") or HIP_LIB
    if not os.path.exists(p):
        raise RuntimeError("libtsdf_hip.so not built (%s); run `python -c 'import __graft_entry__ "
                           "as g; g.build()'` or `make -C noetic-slam_amd/csrc`" % p)
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7, but
    # needed as "libamdhip64.so"), so it is loaded first and the library's libamdhip64.so.7 then
    # resolves to that copy.  Loaded the other way round, the process holds two runtimes and
    # torch finds no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = _abi.declare(ctypes.CDLL(p))
    if lib.tsdf_abi_version() != ABI_VERSION:
        raise RuntimeError("libtsdf_hip.so ABI version mismatch")
    if path is None:
        _hip = lib
    return lib
