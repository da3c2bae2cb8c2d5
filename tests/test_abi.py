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


def test_undistort_arguments_and_no_gpu(euroc_yaml):
    """uvio_hp_undistort: argument errors before any device work, an empty batch is a no-op, and points on a
    CPU-only box fail loudly (E_DEVICE; the host never undistorts a batch by itself)."""
    import numpy as np
    import torch
    import uvio_amd as U
    from uvio_amd import _native as N
    lib = N.load()
    cam = np.zeros(8)
    fp = C.POINTER(C.c_float)
    uv = np.zeros(2, np.float32)
    out = np.zeros(2, np.float32)
    args = (cam.ctypes.data_as(C.POINTER(C.c_double)), 1, uv.ctypes.data_as(fp), out.ctypes.data_as(fp), None)
    assert lib.uvio_hp_undistort(2, *args) == N.E_ARG  # no such camera model
    assert lib.uvio_hp_undistort(0, None, 1, args[2], args[3], None) == N.E_ARG
    assert lib.uvio_hp_undistort(0, args[0], -1, args[2], args[3], None) == N.E_ARG
    assert lib.uvio_hp_undistort(1, args[0], 1, None, args[3], None) == N.E_ARG
    assert lib.uvio_hp_undistort(0, args[0], 0, None, None, None) == 0
    o = U.load_options(euroc_yaml)
    assert U.undistort(o.cams[0], np.zeros((0, 2), np.float32)).shape == (0, 2)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="E_DEVICE"):
            U.undistort(o.cams[0], np.ones((3, 2), np.float32))


def _cfg(name):
    return os.path.join(ROOT, "configs", name, "estimator_config.yaml")


def test_options_load_tum_vi_t_cam_imu():
    """TUM-VI's kalibr chain gives T_cam_imu = [R_ItoC | p_IinC]; the parser falls back to it when T_imu_cam
    is absent and inverts it (YamlParser::parse(Matrix4d), opencv_yaml_parse.h:487-530)."""
    import numpy as np
    import uvio_amd as U
    from uvio_amd.sim import quat_2_rot
    o = U.load_options(_cfg("tum_vi"))
    assert o.num_cameras == 2 and o.use_stereo == 1 and o.min_px_dist == 15
    c0 = o.cams[0]
    assert c0.model == 1 and (c0.width, c0.height) == (512, 512)
    T = np.array([[-0.9995250378696743, 0.029615343885863205, -0.008522328211654736, 0.04727988224914392],
                  [0.0075019185074052044, -0.03439736061393144, -0.9993800792498829, -0.047443232143367084],
                  [-0.02989013031643309, -0.998969345370175, 0.03415885127385616, -0.0681999605066297]])
    assert np.allclose(quat_2_rot(np.array(c0.q_ItoC[:])), T[:, :3], atol=1e-9)
    assert np.allclose(np.array(c0.p_IinC[:]), T[:, 3], atol=1e-9)
    assert abs(o.gravity_mag - 9.80766) < 1e-12 and abs(o.sigma_a - 0.0028) < 1e-12


def test_options_load_uzhfpv_and_rpng_sim_uwb():
    import uvio_amd as U
    o = U.load_options(_cfg("uzhfpv_outdoor_45"))
    assert o.do_calib_camera_pose == 0 and o.do_calib_camera_intrinsics == 1
    assert o.cams[1].model == 1 and (o.cams[1].width, o.cams[1].height) == (640, 480)
    assert abs(o.msckf_sigma_pix - 1.5) < 1e-12 and o.fast_threshold == 50 and o.track_frequency == 31.0
    assert abs(o.calib_camimu_dt - (-0.008637511810764048)) < 1e-15
    o = U.load_options(_cfg("rpng_sim_uwb"))
    assert o.num_cameras == 4 and o.use_stereo == 0
    assert o.do_calib_imu_intrinsics == 1 and o.do_calib_imu_g_sensitivity == 1
    assert o.use_uwb == 1 and o.n_anchors == 6 and o.n_anchors_to_fix == 2
    assert [o.anchors[i].fix for i in range(6)] == [1, 1, 0, 0, 0, 0]
    assert list(o.anchors[4].p_AinG) == [0.0, 7.0, 1.5]
    assert list(o.p_IinU) == [-0.01, 0.01, 0.05]  # uwb_extrinsics p_UinI -> p_IinU = -p_UinI
    assert abs(o.cams[2].p_IinC[0] - o.cams[0].p_IinC[0]) > 0.1  # the second pair is shifted
