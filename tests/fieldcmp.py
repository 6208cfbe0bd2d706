"""Per-voxel comparison of two exported fields (test helper): touched-set differences, weight
mismatches and |dSDF| statistics over the common voxels whose weights agree."""
import numpy as np


def _keys(ijk):
    k = np.asarray(ijk, np.int64) + (1 << 20)
    return k[:, 0] | (k[:, 1] << 21) | (k[:, 2] << 42)


def compare(a, b):
    """a, b: (ijk, sdf, weight) as export_voxels() returns them."""
    ai, as_, aw = a
    bi, bs, bw = b
    ka, kb = _keys(ai), _keys(bi)
    common, ia, ib = np.intersect1d(ka, kb, assume_unique=True, return_indices=True)
    d = np.abs(as_[ia].astype(np.float64) - bs[ib].astype(np.float64))
    weq = aw[ia] == bw[ib]
    de = d[weq]
    return {
        "voxels_a": int(ka.size), "voxels_b": int(kb.size),
        "only_a": int(ka.size - common.size), "only_b": int(kb.size - common.size),
        "weight_mismatch": int((~weq).sum()),
        "max_abs_dsdf": float(de.max()) if de.size else 0.0,
        "p999_abs_dsdf": float(np.quantile(de, 0.999)) if de.size else 0.0,
        "over_1e-5": int((de > 1e-5).sum()),
        "bitwise_equal": int((as_[ia][weq].view(np.uint32) == bs[ib][weq].view(np.uint32)).sum()),
    }
