"""The insert staging pool (flink-skyline-qos_amd/csrc/stage_pool.h) on its own, without HIP:
thousands of back-to-back jobs of varying size, every item exactly once, nothing touched after
run() returns -- once plain and once under ThreadSanitizer (tests/stage_pool_stress.cc)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "stage_pool_stress.cc")
INC = os.path.join(ROOT, "flink-skyline-qos_amd", "csrc")


def _build(tmp_path, extra):
    exe = str(tmp_path / ("stress" + ("_tsan" if extra else "")))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-I", INC, SRC, "-o", exe] + extra
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("threads", [2, 4, 8])
def test_stage_pool_plain(tmp_path, threads):
    exe = _build(tmp_path, [])
    r = subprocess.run([exe, "20000", str(threads)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_stage_pool_tsan(tmp_path):
    try:
        exe = _build(tmp_path, ["-fsanitize=thread"])
    except subprocess.CalledProcessError as e:       # no libtsan in the image
        pytest.skip("ThreadSanitizer unavailable: " + e.stderr[-200:])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([exe, "5000", "4"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr
