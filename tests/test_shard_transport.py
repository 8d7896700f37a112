"""Host unit test of the row-sharded plan's transport selection and its fallback when RCCL
cannot start (csrc/shard_transport.hpp, tests/shard_transport_test.cpp): g++ on the CPU,
no device."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_shard_transport_selection(tmp_path):
    exe = tmp_path / "shard_transport_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "celestia-app_amd", "csrc"),
                    os.path.join(ROOT, "tests", "shard_transport_test.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ok" in out.stdout
