"""ctypes declarations of the C-ABI in include/tsdf_hip.h (shared by every library exporting it)."""
import ctypes as C
import math

TSDF_OK = 0
TSDF_EINVAL = -1
TSDF_ENOMEM = -2
TSDF_EHIP = -3
TSDF_ENODEV = -4
TSDF_EOVERFLOW = -5
BRICK_SIDE = 8
BRICK_VOX = 512

STATUS_NAMES = {
    TSDF_OK: "TSDF_OK", TSDF_EINVAL: "TSDF_EINVAL", TSDF_ENOMEM: "TSDF_ENOMEM",
    TSDF_EHIP: "TSDF_EHIP", TSDF_ENODEV: "TSDF_ENODEV", TSDF_EOVERFLOW: "TSDF_EOVERFLOW",
}

ABI_VERSION = 10
TILE_WORDS = 1028  # TSDF_TILE_WORDS: u32 words of one border-brick tile
MAX_WORLD = 64
SEM_VDBFUSION = 0
SEM_VOXBLOX = 1
SEM_VDBFUSION_F64 = 2
SEMANTICS = {"vdbfusion": SEM_VDBFUSION, "voxblox": SEM_VOXBLOX,
             "vdbfusion_f64": SEM_VDBFUSION_F64}

# k_<kind>, KernelKind order: the two-walk front end (count, place) or the single walk (walk, spans)
KERNEL_KINDS = ("count", "compact", "place", "integrate", "walk", "spans")
WALK_TWO = 0     # tsdf_params.walk: k_count + k_place (default)
WALK_SINGLE = 1  # k_walk + k_spans when the band allows it
MC_TABLES = {"generated": 0, "lorensen": 1, "lorensen_rule": 2}  # TSDF_MC_*
VB_METHODS = {"simple": 0, "merged": 1}  # tsdf_params.voxblox_method (TSDF_VB_*)
SECTOR_INPUTS = {"fanout": 0, "h2d": 1, "split": 2}  # tsdf_params.sector_input
SECTOR_RULES = {"world": 0, "index": 1}  # tsdf_params.sector_rule (TSDF_SECTOR_RULE_*, ABI v10)


class TsdfParams(C.Structure):
    _fields_ = [
        ("voxel_size", C.c_double),
        ("sdf_trunc", C.c_double),
        ("space_carving", C.c_int32),
        ("weight_mode", C.c_int32),
        ("min_range", C.c_double),
        ("max_range", C.c_double),
        ("max_bricks", C.c_uint64),
        ("max_points", C.c_uint64),
        ("max_pairs", C.c_uint64),
        ("device_id", C.c_int32),
        ("brick_side", C.c_int32),
        ("max_batch", C.c_uint32),
        ("pipeline", C.c_uint32),
        # ABI v3
        ("semantics", C.c_int32),
        ("allow_clear", C.c_int32),
        ("use_weight_dropoff", C.c_int32),
        ("max_weight", C.c_float),
        # ABI v4
        ("n_sectors", C.c_uint32),
        ("sector", C.c_uint32),
        ("sector_yaw0", C.c_double),
        ("max_bricks_hard", C.c_uint64),
        # ABI v5
        ("walk", C.c_int32),
        # ABI v6
        ("depth_weight", C.c_int32),
        # ABI v8
        ("voxblox_method", C.c_int32),
        ("sector_input", C.c_int32),
        # ABI v10
        ("sector_rule", C.c_int32),
    ]


class TsdfStats(C.Structure):
    _fields_ = [
        ("n_scans", C.c_uint64),
        ("n_points_in", C.c_uint64),
        ("n_bricks", C.c_uint64),
        ("n_pairs_last", C.c_uint64),
        ("n_active_last", C.c_uint64),
        ("n_voxels_last", C.c_uint64),
        ("n_voxels_total", C.c_uint64),
        ("n_rays_total", C.c_uint64),
        ("n_dirty_total", C.c_uint64),
        ("n_batches", C.c_uint64),
        ("kernel_ms", C.c_double * 8),
        ("kernel_launches", C.c_uint64 * 8),
        # ABI v4
        ("n_grows", C.c_uint64),
        ("n_replayed", C.c_uint64),
        ("max_bricks", C.c_uint64),
        # ABI v8
        ("peer_mask", C.c_uint64),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("kernel_ms", "kernel_launches")}
        d["kernel_ms"] = {KERNEL_KINDS[i]: self.kernel_ms[i] for i in range(len(KERNEL_KINDS))}
        d["kernel_launches"] = {KERNEL_KINDS[i]: self.kernel_launches[i]
                                for i in range(len(KERNEL_KINDS))}
        return d


# every symbol include/tsdf_hip.h declares, with its signature
P = C.c_void_p
D3 = C.POINTER(C.c_double)
I3 = C.POINTER(C.c_int32)
L3 = C.POINTER(C.c_int64)
FP = C.POINTER(C.c_float)
U64P = C.POINTER(C.c_uint64)
class OsFormat(C.Structure):
    """tsdf_os_format (include/tsdf_hip.h)."""
    _fields_ = [("profile", C.c_uint32), ("pixels_per_column", C.c_uint32),
                ("columns_per_packet", C.c_uint32), ("columns_per_frame", C.c_uint32)]


OS_PROFILES = {"LEGACY": 0, "RNG19_RFL8_SIG16_NIR16": 1, "RNG19_RFL8_SIG16_NIR16_DUAL": 2,
               "RNG15_RFL8_NIR8": 3}


SIGNATURES = {
    "tsdf_default_params": (None, [C.POINTER(TsdfParams)]),
    "tsdf_abi_version": (C.c_int, []),
    "tsdf_create": (C.c_int, [C.POINTER(TsdfParams), C.POINTER(P)]),
    "tsdf_destroy": (None, [P]),
    "tsdf_last_error": (C.c_char_p, [P]),
    "tsdf_integrate": (C.c_int, [P, P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int32, D3]),
    "tsdf_integrate_pose": (C.c_int, [P, P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int32, D3]),
    "tsdf_integrate_sectors": (C.c_int, [C.POINTER(P), C.c_uint32, P, C.c_uint64, C.c_uint32,
                                         C.c_uint32, C.c_int32, D3]),
    "tsdf_integrate_device": (C.c_int, [P, P, C.c_uint64, D3]),
    "tsdf_integrate_batch_device": (C.c_int, [P, P, U64P, C.c_uint32, D3]),
    "tsdf_integrate_batch_device_pose": (C.c_int, [P, P, U64P, C.c_uint32, D3]),
    "tsdf_sync": (C.c_int, [P]),
    "tsdf_query_dense": (C.c_int, [P, L3, L3, FP, FP]),  # ABI v10: int64 bounds
    "tsdf_num_bricks": (C.c_int, [P, U64P]),
    "tsdf_export_bricks": (C.c_int, [P, I3, FP, FP, C.c_uint64, U64P]),
    "tsdf_import_bricks": (C.c_int, [P, I3, FP, FP, C.c_uint64]),
    "tsdf_get_stats": (C.c_int, [P, C.POINTER(TsdfStats)]),
    "tsdf_reset_stats": (C.c_int, [P]),
    "tsdf_set_profiling": (C.c_int, [P, C.c_int32]),
    "tsdf_set_profiling_period": (C.c_int, [P, C.c_uint32, C.c_uint32]),
    "tsdf_create_sharded": (C.c_int, [C.POINTER(TsdfParams), C.c_uint32, C.POINTER(C.c_int32),
                                      C.POINTER(P)]),
    "tsdf_border_reduce_local": (C.c_int, [C.POINTER(P), C.c_uint32, U64P]),
    "tsdf_set_metrics_log": (C.c_int, [P, C.c_char_p]),
    "tsdf_select_sector": (C.c_int, [FP, C.c_uint64, D3, C.c_double, C.c_uint32, C.c_uint32, FP,
                                     U64P]),
    "tsdf_sector_of": (C.c_int32, [C.c_float, C.c_float, D3, C.c_double, C.c_uint32]),
    "tsdf_brick_keys_device": (C.c_int, [P, P, C.c_uint64, U64P]),
    "tsdf_border_pack_device": (C.c_int, [P, P, U64P, C.c_uint64, C.c_uint32, C.c_uint32, P,
                                          C.c_uint64, U64P]),
    "tsdf_border_merge_device": (C.c_int, [P, P, U64P, C.c_uint32]),
    # ABI v9
    "tsdf_border_commit_device": (C.c_int, [P, C.c_int32]),
    "tsdf_integrate_sectors_origin": (C.c_int, [C.POINTER(P), C.c_uint32, P, C.c_uint64,
                                                C.c_uint32, C.c_uint32, C.c_int32, D3]),
    "tsdf_halo_keys_device": (C.c_int, [P, P, C.c_uint64, U64P]),
    "tsdf_halo_pack_device": (C.c_int, [P, P, C.c_uint64, P, C.c_uint64, U64P]),
    "tsdf_extract_mesh_halo": (C.c_int, [P, C.c_float, C.c_int32, P, C.c_uint64, FP, C.c_uint64,
                                         U64P]),
    "tsdf_extract_mesh_local": (C.c_int, [C.POINTER(P), C.c_uint32, C.c_float, C.c_int32, FP,
                                          C.c_uint64, U64P]),
    "tsdf_extract_mesh": (C.c_int, [P, C.c_float, FP, C.c_uint64, U64P]),
    "tsdf_mc_table": (C.c_int, [C.POINTER(C.c_uint8)]),
    "tsdf_extract_mesh_table": (C.c_int, [P, C.c_float, C.c_int32, FP, C.c_uint64, U64P]),
    "tsdf_mc_table_of": (C.c_int, [C.c_int32, C.POINTER(C.c_uint8)]),
    "tsdf_os_packet_bytes": (C.c_int, [C.POINTER(OsFormat), C.POINTER(C.c_uint32)]),
    "tsdf_os_decode_device": (C.c_int, [P, C.POINTER(OsFormat), P, C.c_uint32, P, P, P, P]),
    "tsdf_os_cartesian_device": (C.c_int, [P, P, C.c_uint64, P, P, C.POINTER(C.c_double), P]),
}


def declare(lib, names=None, optional=()):
    """Attach restype/argtypes for the ABI symbols present in `lib`; raise if a required one is
    missing."""
    missing = []
    for name, (res, args) in SIGNATURES.items():
        if names is not None and name not in names:
            continue
        fn = getattr(lib, name, None)
        if fn is None:
            if name not in optional:
                missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing:
        raise RuntimeError("library %s lacks ABI symbols: %s" % (lib._name, ", ".join(missing)))
    return lib


def default_params(lib=None, **kw):
    p = TsdfParams()
    if lib is not None:
        lib.tsdf_default_params(C.byref(p))
    else:
        p.voxel_size, p.sdf_trunc, p.space_carving, p.weight_mode = 0.05, 0.15, 0, 0
        p.min_range, p.max_range = 0.0, math.inf
        p.max_bricks, p.max_points, p.max_pairs = 1 << 20, 1 << 18, 0
        p.device_id, p.brick_side, p.max_batch = 0, BRICK_SIDE, 32
        p.semantics, p.allow_clear, p.use_weight_dropoff, p.max_weight = SEM_VDBFUSION_F64, 1, 1, 1e4
        p.n_sectors, p.sector, p.sector_yaw0, p.max_bricks_hard = 0, 0, 0.0, 0
        p.walk = WALK_TWO
        p.depth_weight, p.voxblox_method, p.sector_input = 1, 0, 0
        p.sector_rule = SECTOR_RULES["index"]
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError("unknown tsdf_params field %r" % k)
        setattr(p, k, v)
    return p
