"""The host staging thread pool (noetic-slam_amd/csrc/pack_pool.h: spin-then-sleep workers, pools
run side by side with part offsets for tsdf_integrate_sectors) built with g++ and stressed on the
CPU: every part of every job runs exactly once, also after the workers went to sleep."""
import os
import subprocess

from conftest import REPO


def test_pack_pool_stress(tmp_path):
    exe = tmp_path / "pack_pool_stress"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", "-o", str(exe),
                           os.path.join(REPO, "tests", "cpp", "pack_pool_stress.cpp")])
    out = subprocess.run([str(exe), "3000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")


def test_pack_pool_thread_sanitizer(tmp_path):
    """The same stress under ThreadSanitizer (host code only): no data race on the job, the
    generation counter or the busy count."""
    exe = tmp_path / "pack_pool_tsan"
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=thread",
                           "-o", str(exe), os.path.join(REPO, "tests", "cpp", "pack_pool_stress.cpp")])
    out = subprocess.run([str(exe), "300"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "WARNING: ThreadSanitizer" not in out.stderr, out.stderr[-3000:]
