"""k_integrate's fuse chains divide with the reciprocal off the chain (tsdf_ray.h div_rn: y = RN(1/d)
from the hardware reciprocal and one Newton step, Markstein's correction), and redo a chain with
IEEE division when a step leaves the checked ranges.  Both must give the oracle's IEEE quotients bit
for bit: ordinary chains (every parity test), and chains that start from imported extreme states —
|S W| past 2^100, subnormal S, +0 and -0, weights past 2^24 and past 2^40."""
import numpy as np
import pytest

import oracle
from conftest import decimate

pytestmark = pytest.mark.gpu


def hip(**kw):
    from tsdf_map import HipTSDFVolume
    return HipTSDFVolume(0.05, 0.15, **kw)


def ora(**kw):
    return oracle.OracleTSDFVolume(0.05, 0.15, **kw)


def bitwise(a, b):
    ai, as_, aw = a.export_voxels()
    bi, bs, bw = b.export_voxels()
    return (ai.shape == bi.shape and np.array_equal(ai, bi)
            and np.array_equal(aw.view(np.uint32), bw.view(np.uint32))
            and np.array_equal(as_.view(np.uint32), bs.view(np.uint32)))


@pytest.mark.parametrize("semantics", ["vdbfusion", "voxblox"])
def test_extreme_starting_states(sim, semantics):
    (p0, o0), (p1, o1) = sim.scan(0), sim.scan(1)
    base = ora(semantics=semantics)
    base.integrate(decimate(p0, 4), o0)
    c, s, w = base.export_bricks()
    sf, wf = s.reshape(-1), w.reshape(-1)
    idx = np.flatnonzero(wf > 0)
    rng = np.random.default_rng(7)
    pick = rng.choice(idx, size=min(30000, idx.size), replace=False)
    kind = np.arange(pick.size) % 6
    sf[pick[kind == 0]], wf[pick[kind == 0]] = 1e35, 1e4       # |S W| > 2^100
    sf[pick[kind == 1]], wf[pick[kind == 1]] = -3e-41, 2.0     # subnormal S
    sf[pick[kind == 2]], wf[pick[kind == 2]] = 0.0, 7.0
    sf[pick[kind == 3]], wf[pick[kind == 3]] = -0.0, 5.0
    wf[pick[kind == 4]] = 3e7                                   # weights past 2^24
    wf[pick[kind == 5]] = 2e12                                  # a divisor past 2^40
    g, o = hip(semantics=semantics), ora(semantics=semantics)
    g.import_bricks(c, s, w)
    o.import_bricks(c, s, w)
    for p, org in ((p1, o1), (decimate(p0, 2), o0)):
        g.integrate(p, org)
        o.integrate(p, org)
    assert bitwise(g, o)
