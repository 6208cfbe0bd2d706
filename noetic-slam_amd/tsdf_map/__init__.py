"""tsdf_map — host side of the MI355X TSDF backend (MAP_BACKEND_IDX = 4) for noetic-slam.

Named after the reference's mapping package (src/tsdf_map, README.md:44-50).  The backend table
mirrors the node's compile-time switch; indices 0-3 are the reference's CPU backends, which are not
in the reference snapshot and so are listed but not constructible here.
"""
from ._abi import BRICK_SIDE, BRICK_VOX  # noqa: F401
from ._lib import HIP_LIB, load_hip_library  # noqa: F401
from .volume import (HipTSDFVolume, MergedTsdfIntegrator, SimpleTsdfIntegrator,  # noqa: F401
                     TSDFVolume,
                     TsdfError, TsdfIntegratorConfig, border_reduce_local, bricks_to_voxels,
                     extract_mesh_local, integrate_sectors, integrate_sectors_cloud,
                     sector_ids, select_sector)

MAP_BACKENDS = {
    0: "CHAD TSDF (absent from the reference snapshot)",
    1: "Octomap (absent from the reference snapshot)",
    2: "Voxblox (absent from the reference snapshot)",
    3: "VDBFusion (absent from the reference snapshot)",
    4: "MI355X HIP TSDF (this package)",
}
MAP_BACKEND_IDX = 4


def make_backend(idx=MAP_BACKEND_IDX, **kw):
    """Construct backend `idx` the way tsdf_map_node's switch does."""
    if idx == 4:
        return HipTSDFVolume(**kw)
    if idx in (2, 3) and kw.pop("on_gpu", False):
        # the MI355X backend restating CPU backend idx 2 (Voxblox) or 3 (VDBFusion) semantics
        return HipTSDFVolume(semantics="voxblox" if idx == 2 else "vdbfusion_f64", **kw)
    if idx in MAP_BACKENDS:
        raise NotImplementedError("MAP_BACKEND_IDX=%d: %s" % (idx, MAP_BACKENDS[idx]))
    raise ValueError("unknown MAP_BACKEND_IDX %r" % idx)
