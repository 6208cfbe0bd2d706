"""Generate the committed golden vectors (run in the build container):

    python tests/golden/make_golden.py

golden_c1_decimated.npz — inputs and expected outputs of a 3-scan sequence of the C1 synthetic
OS-1-128 1024x10 stream (every 16th point of each scan, column-major scan order), 5 cm voxels,
15 cm truncation, no carving, integrated by the CPU oracle in its scan-fused mode.  The GPU must
reproduce the output bit for bit (tests/test_gpu_parity.py::test_golden_fixture); the oracle must
keep reproducing it (tests/test_golden.py), which pins the restatement against silent drift.
golden_c1_decimated.sha256 holds the digest of the expected outputs.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "noetic-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

SCANS = (0, 1, 40)
DECIMATE = 16
SEMANTICS = "vdbfusion"  # the fp32 restatement (the golden file predates the ABI v8 default)
VS, TAU = 0.05, 0.15


def digest(ijk, sdf, w):
    h = hashlib.sha256()
    for a in (ijk, sdf, w):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    import oracle
    from tsdf_map.scan_gen import OusterSim

    sim = OusterSim()
    pts, org = [], []
    for k in SCANS:
        p, o = sim.scan(k)
        pts.append(np.ascontiguousarray(p[::DECIMATE]))
        org.append(o)
    offs = np.cumsum([0] + [p.shape[0] for p in pts]).astype(np.int64)
    v = oracle.OracleTSDFVolume(VS, TAU, semantics=SEMANTICS)
    for p, o in zip(pts, org):
        v.integrate(p, o)
    ijk, s, w = v.export_voxels()
    np.savez_compressed(os.path.join(HERE, "golden_c1_decimated.npz"),
                        points=np.concatenate(pts), origins=np.stack(org), scan_offsets=offs,
                        voxel_size=VS, sdf_trunc=TAU, ijk=ijk, sdf=s, weight=w)
    with open(os.path.join(HERE, "golden_c1_decimated.sha256"), "w") as f:
        f.write(digest(ijk, s, w) + "\n")
    print("voxels", ijk.shape[0], "digest", digest(ijk, s, w))


if __name__ == "__main__":
    main()
