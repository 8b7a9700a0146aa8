"""host_parallel's persistent worker pool (siddhi_amd/csrc/runtime.hpp HostPool), host code only: every thread range
runs once per call over thousands of calls, nested and concurrent callers fall back to their own threads, and a
forked child gets a working pool (tools/micro/host_pool_check.cpp, built here with hipcc; no GPU call)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not on PATH")
def test_host_pool(tmp_path):
    exe = str(tmp_path / "host_pool_check")
    subprocess.run(["hipcc", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools/micro/host_pool_check.cpp"),
                    "-lpthread"], check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host pool ok" in r.stdout
