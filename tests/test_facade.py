"""The C++ facade header (include/uvio_hp.hpp) compiles with g++ against the C ABI, links
against libuvio_hp.so and behaves on a host without a GPU: options load, construction throws
uvio_amd::Error with UVIO_HP_E_DEVICE (the product has no CPU fallback)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_facade_compiles_links_and_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("checks the no-device behaviour")
    lib = os.path.join(ROOT, "uvio_amd", "libuvio_hp.so")
    if not os.path.exists(lib):
        from uvio_amd import build
        build.build_product()
    exe = str(tmp_path / "facade_check")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "facade_check.cpp"), "-o", exe, lib,
           "-Wl,-rpath," + os.path.dirname(lib), "-Wl,--allow-shlib-undefined"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    cfg = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")
    r = subprocess.run([exe, cfg], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, LD_LIBRARY_PATH="/opt/rocm/lib:" + os.environ.get("LD_LIBRARY_PATH", "")))
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "code -3" in r.stdout
