"""The oracle keeps reproducing the committed golden vectors bit for bit (CPU)."""
import os

import numpy as np

import oracle
from conftest import GOLDEN


def _make_golden():
    import sys
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    import make_golden
    return make_golden


def make_golden_semantics():
    return _make_golden().SEMANTICS


def test_oracle_reproduces_golden():
    digest = _make_golden().digest
    z = np.load(os.path.join(GOLDEN, "golden_c1_decimated.npz"), allow_pickle=False)
    v = oracle.OracleTSDFVolume(float(z["voxel_size"]), float(z["sdf_trunc"]),
                                semantics=make_golden_semantics())
    offs = z["scan_offsets"]
    for s in range(len(offs) - 1):
        v.integrate(z["points"][offs[s]:offs[s + 1]], z["origins"][s])
    ijk, s_, w = v.export_voxels()
    assert np.array_equal(ijk, z["ijk"])
    assert np.array_equal(w, z["weight"])
    assert np.array_equal(s_.view(np.uint32), z["sdf"].view(np.uint32))
    want = open(os.path.join(GOLDEN, "golden_c1_decimated.sha256")).read().split()[0]
    assert digest(ijk, s_, w) == want


def test_golden_inputs_follow_the_generator():
    """The stored inputs are the generator's (regression of the Ouster LUT / scene code)."""
    make_golden = _make_golden()
    from tsdf_map.scan_gen import OusterSim
    z = np.load(os.path.join(GOLDEN, "golden_c1_decimated.npz"), allow_pickle=False)
    p, o = OusterSim().scan(make_golden.SCANS[0])
    n0 = int(z["scan_offsets"][1])
    assert np.array_equal(z["points"][:n0], p[::make_golden.DECIMATE])
    assert np.array_equal(z["origins"][0], o)
