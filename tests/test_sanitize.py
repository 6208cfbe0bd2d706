"""VERDICT r4 #8 / SURVEY §5 "Race detection / sanitizers": the multi-threaded C oracle built with
AddressSanitizer + UndefinedBehaviorSanitizer (any report aborts: -fno-sanitize-recover=all) and
with ThreadSanitizer (oracle/Makefile `sanitize`), driven through its whole C-ABI by
tests/cpp/oracle_sanitize.c on real scans: every semantics in serial and in the partitioned
multi-threaded scan-fused mode (bit for bit), Voxblox's capped 1/z^2 weights on thousands of
points in one voxel (the exact int64 fixed-point sums at their extremes, where ADVICE r3 found an
overflow), rays onto voxel faces and far from the origin, read-out, marching cubes, the
border-reduce transaction (commit and abort), the sharded calls and the sharded mesh.  Host code
only: GPU sanitizers are not available on this pool."""
import os
import struct
import subprocess

import numpy as np
import pytest

from conftest import REPO

ORACLE = os.path.join(REPO, "oracle")


@pytest.fixture(scope="module")
def sanitized():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "sanitize"])
    return {k: os.path.join(ORACLE, "build", "oracle_" + k) for k in ("asan", "tsan")}


def write_scans(path, sim, ks, step):
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(ks)))
        for k in ks:
            pts, org = sim.scan(k)
            pts = np.ascontiguousarray(pts[::step], np.float32)
            f.write(struct.pack("<Q3d", pts.shape[0], *org))
            f.write(pts.tobytes())


def run(exe, args, timeout):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    return subprocess.run([exe] + args, capture_output=True, text=True, timeout=timeout, env=env)


def test_oracle_address_and_undefined_sanitizer(tmp_path, sim, sanitized):
    write_scans(tmp_path / "scans.bin", sim, (0, 1, 4), 8)
    r = run(sanitized["asan"], [str(tmp_path / "scans.bin"), "4", "all"], 900)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.stdout + r.stderr)[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_oracle_thread_sanitizer(tmp_path, sim, sanitized):
    """The partitioned multi-threaded mode (tsdf_oracle_set_threads > 1: ray threads bucket samples
    per brick-hash partition, partition threads fuse) on a full C1 scan under TSan."""
    write_scans(tmp_path / "scans.bin", sim, (0,), 1)
    r = run(sanitized["tsan"], [str(tmp_path / "scans.bin"), "8", "threads"], 900)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.stdout + r.stderr)[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr
