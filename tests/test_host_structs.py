"""Host-side data structures of the product library (no GPU): the feature database's per-camera measurement
storage with its cached first / last times, the in-object track set and the host work pool
(uvio_amd/csrc/engine.h, pool.h), driven by tests/cpp/meas_list_test.cpp against plain models."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_meas_list_track_set_and_pool(tmp_path):
    exe = tmp_path / "meas_list_test"
    subprocess.check_call([HIPCC, "-x", "c++", "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
                           "-I", os.path.join(ROOT, "uvio_amd", "csrc"), os.path.join(ROOT, "tests", "cpp", "meas_list_test.cpp"),
                           "-o", str(exe), "-pthread"], timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, timeout=300)
    assert out.returncode == 0, out.stdout.decode() + out.stderr.decode()
    assert b"meas_list_test: ok" in out.stdout
