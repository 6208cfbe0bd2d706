"""k_count's gate skip (noetic-slam_amd/csrc/tsdf_ray.h gate_skip_bound): a voxel whose DDA exit time
is at most the ray's tsafe must pass the gate, since its centre is provably in front of the hit.
tests/csrc/gate_skip_check.c restates the fp32 walk (SEM 0) and the double-precision one (SEM 2)
with the bound and checks the claim on 2 M random and adversarial rays (origins up to 10 km from
zero, depths just past the band, axis-aligned and diagonal directions); the GPU parity tests then
hold the kernels bit-exact with the skip on."""
import os
import subprocess

from conftest import REPO


def test_gate_skip_bound_holds(tmp_path):
    exe = tmp_path / "gate_skip_check"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                           os.path.join(REPO, "tests", "csrc", "gate_skip_check.c"), "-lm"])
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    vox, skip, fail = (int(x) for x in out.stdout.split())
    assert out.returncode == 0 and fail == 0, out.stdout
    assert vox > 10_000_000 and skip > 0.25 * vox  # the bound is not vacuous
