import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "noetic-slam_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtsdf_hip.so)")


@pytest.fixture(scope="session")
def sim():
    from tsdf_map.scan_gen import OusterSim
    return OusterSim()


@pytest.fixture(scope="session")
def scan0(sim):
    return sim.scan(0)


def decimate(points, k):
    """Every k-th point (keeps the DLIO column-major order)."""
    return np.ascontiguousarray(points[::k])
