"""The C-ABI boundary: the library loads, exports every entry point include/uvio_hp.h declares, the
option loader reads the reference's YAML keys, and the product fails loudly without a GPU (no CPU
fallback exists).  No compute calls: these run on the CPU-only CI box."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "uvio_hp.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(uvio_hp_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding_list():
    from uvio_amd import _native as N
    assert _declared() == sorted(N.EXPORTED)


def test_library_exports_every_declared_symbol():
    from uvio_amd import _native as N
    lib = N.load()
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_struct_layouts_match_header_sizes():
    """sizeof of the C structs, computed by the C compiler, equals the ctypes mirrors."""
    import subprocess
    import tempfile
    from uvio_amd import _native as N
    src = ('#include "uvio_hp.h"\n#include <stdio.h>\nint main(){printf("%zu %zu %zu %zu\\n", sizeof(uvio_hp_options_t),'
           ' sizeof(uvio_hp_camera_t), sizeof(uvio_hp_anchor_t), sizeof(uvio_hp_timing_t));return 0;}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "s")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        sizes = [int(x) for x in subprocess.check_output([exe]).split()]
    assert sizes == [C.sizeof(N.Options), C.sizeof(N.Camera), C.sizeof(N.Anchor), C.sizeof(N.Timing)]


def test_options_load_euroc(euroc_yaml):
    import numpy as np
    import uvio_amd as U
    from uvio_amd.sim import quat_2_rot
    o = U.load_options(euroc_yaml)
    assert o.num_cameras == 2 and o.use_stereo == 1
    assert o.max_clone_size == 11
    assert o.integration == 1  # rk4
    assert o.feat_rep_slam == 4  # ANCHORED_MSCKF_INVERSE_DEPTH
    c0 = o.cams[0]
    assert (c0.width, c0.height) == (752, 480)
    assert np.allclose(c0.intrinsics[:4], [458.654, 457.296, 367.215, 248.375])
    assert np.allclose(c0.intrinsics[4:], [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05])
    # T_imu_cam (T_CtoI) of cam0 in kalibr_imucam_chain.yaml -> q_ItoC = R_CtoI^T, p_IinC = -R_CtoI^T p_CinI
    T = np.array([[0.0148655429818, -0.999880929698, 0.00414029679422, -0.0216401454975],
                  [0.999557249008, 0.0149672133247, 0.025715529948, -0.064676986768],
                  [-0.0257744366974, 0.00375618835797, 0.999660727178, 0.00981073058949]])
    R_ItoC = quat_2_rot(np.array(c0.q_ItoC[:]))
    assert np.allclose(R_ItoC, T[:, :3].T, atol=1e-9)
    assert np.allclose(np.array(c0.p_IinC[:]), -T[:, :3].T @ T[:, 3], atol=1e-9)
    assert abs(o.sigma_w - 1.6968e-04) < 1e-12 and abs(o.sigma_ab - 3.0e-03) < 1e-12


def test_options_missing_file_is_config_error():
    import uvio_amd as U
    with pytest.raises(RuntimeError, match="E_CONFIG"):
        U.load_options("/nonexistent/estimator_config.yaml")


def test_overrides_reject_unknown_keys(euroc_yaml):
    import uvio_amd as U
    with pytest.raises(KeyError):
        U.load_options(euroc_yaml, not_a_key=1)


def test_product_fails_loudly_without_gpu(euroc_yaml):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import uvio_amd as U
    o = U.load_options(euroc_yaml)
    with pytest.raises(RuntimeError, match="E_DEVICE"):
        U.VioManager(o)
    P = [[1.0]]
    with pytest.raises(RuntimeError, match="E_DEVICE"):
        U.ekf_update(P, [0], [[1.0]], [0.5], 1.0)
