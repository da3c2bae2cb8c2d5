"""ctypes mirror of include/uvio_hp.h (structs + loader).

The product library ``uvio_amd/libuvio_hp.so`` is built in-tree (``python -m uvio_amd.build``).
There is no fallback: if the library cannot be loaded the import of the facade raises.
"""
import ctypes as C
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("UVIO_HP_LIB", os.path.join(ROOT, "uvio_amd", "libuvio_hp.so"))  # override: A/B runs

MAX_CAMS = 4
MAX_ANCHORS = 16

OK = 0
E_ARG, E_STATE, E_DEVICE, E_NUMERIC, E_CONFIG, E_ORDER, E_CAPACITY, E_INTERNAL = -1, -2, -3, -4, -5, -6, -7, -8
ERRNAMES = {0: "OK", -1: "E_ARG", -2: "E_STATE", -3: "E_DEVICE", -4: "E_NUMERIC", -5: "E_CONFIG", -6: "E_ORDER",
            -7: "E_CAPACITY", -8: "E_INTERNAL"}


class Camera(C.Structure):
    _fields_ = [("model", C.c_int), ("width", C.c_int), ("height", C.c_int), ("intrinsics", C.c_double * 8),
                ("q_ItoC", C.c_double * 4), ("p_IinC", C.c_double * 3)]


class Anchor(C.Structure):
    _fields_ = [("id", C.c_uint64), ("fix", C.c_int), ("p_AinG", C.c_double * 3), ("const_bias", C.c_double),
                ("dist_bias", C.c_double), ("cov_diag", C.c_double * 5)]


class Options(C.Structure):
    _fields_ = [
        ("do_fej", C.c_int), ("integration", C.c_int), ("num_cameras", C.c_int), ("use_stereo", C.c_int),
        ("do_calib_camera_pose", C.c_int), ("do_calib_camera_intrinsics", C.c_int),
        ("do_calib_camera_timeoffset", C.c_int), ("do_calib_imu_intrinsics", C.c_int),
        ("do_calib_imu_g_sensitivity", C.c_int), ("imu_model", C.c_int), ("max_clone_size", C.c_int),
        ("max_slam_features", C.c_int), ("max_slam_in_update", C.c_int), ("max_msckf_in_update", C.c_int),
        ("max_aruco_features", C.c_int), ("feat_rep_msckf", C.c_int), ("feat_rep_slam", C.c_int),
        ("dt_slam_delay", C.c_double), ("gravity_mag", C.c_double), ("calib_camimu_dt", C.c_double),
        ("msckf_sigma_pix", C.c_double), ("msckf_chi2_multipler", C.c_double),
        ("slam_sigma_pix", C.c_double), ("slam_chi2_multipler", C.c_double),
        ("sigma_w", C.c_double), ("sigma_a", C.c_double), ("sigma_wb", C.c_double), ("sigma_ab", C.c_double),
        ("imu_dw", C.c_double * 6), ("imu_da", C.c_double * 6), ("imu_tg", C.c_double * 9),
        ("q_GYROtoIMU", C.c_double * 4), ("q_ACCtoIMU", C.c_double * 4),
        ("fi_triangulate_1d", C.c_int), ("fi_refine_features", C.c_int), ("fi_max_runs", C.c_int),
        ("fi_init_lamda", C.c_double), ("fi_max_lamda", C.c_double), ("fi_min_dx", C.c_double),
        ("fi_min_dcost", C.c_double), ("fi_lam_mult", C.c_double), ("fi_min_dist", C.c_double),
        ("fi_max_dist", C.c_double), ("fi_max_baseline", C.c_double), ("fi_max_cond_number", C.c_double),
        ("cams", Camera * MAX_CAMS),
        ("num_pts", C.c_int), ("fast_threshold", C.c_int), ("grid_x", C.c_int), ("grid_y", C.c_int),
        ("min_px_dist", C.c_int), ("histogram_method", C.c_int), ("downsample_cameras", C.c_int),
        ("track_frequency", C.c_double),
        ("use_uwb", C.c_int), ("do_calib_uwb_extrinsics", C.c_int), ("prior_uwb_imu_cov", C.c_double),
        ("uwb_sigma_range", C.c_double), ("uwb_chi2_multipler", C.c_double), ("min_dist_to_use_uwb", C.c_double),
        ("p_IinU", C.c_double * 3), ("n_anchors_to_fix", C.c_int), ("n_anchors", C.c_int),
        ("anchors", Anchor * MAX_ANCHORS),
        ("record_timing", C.c_int), ("init_max_features", C.c_int),
        ("try_zupt", C.c_int), ("zupt_chi2_multipler", C.c_double), ("zupt_max_velocity", C.c_double),
        ("zupt_noise_multiplier", C.c_double), ("zupt_max_disparity", C.c_double),
        ("zupt_only_at_beginning", C.c_int), ("use_klt", C.c_int), ("use_aruco", C.c_int),
        ("record_timing_information", C.c_int), ("record_timing_filepath", C.c_char * 256),
        ("init_window_time", C.c_double), ("init_imu_thresh", C.c_double), ("init_max_disparity", C.c_double),
        ("init_dyn_use", C.c_int),
    ]


class Timing(C.Structure):
    _fields_ = [("timestamp", C.c_double), ("tracking", C.c_double), ("propagation", C.c_double),
                ("msckf_update", C.c_double), ("slam_update", C.c_double), ("slam_delayed", C.c_double),
                ("marg", C.c_double), ("total", C.c_double), ("n_msckf", C.c_int), ("n_slam", C.c_int),
                ("n_slam_delayed", C.c_int), ("n_clones", C.c_int), ("cov_dim", C.c_int),
                ("msckf_rows", C.c_int), ("msckf_cols", C.c_int), ("k_feat_launches", C.c_int),
                ("k_feat_s", C.c_double), ("k_feat_flops", C.c_double), ("device_syncs", C.c_int),
                ("sync_wait", C.c_double), ("zupt", C.c_int), ("n_anchor_change", C.c_int),
                ("chain_wait", C.c_double), ("stage_restarts", C.c_int), ("chain_blob_old_epoch", C.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class KStat(C.Structure):
    _fields_ = [("name", C.c_char * 24), ("kernels", C.c_char * 192), ("bound", C.c_int), ("launches", C.c_longlong),
                ("seconds", C.c_double), ("flops", C.c_double), ("bytes", C.c_double)]

    def as_dict(self):
        return {"name": self.name.decode(), "kernels": self.kernels.decode().split(","),
                "bound": "hbm" if self.bound == 0 else "mfma", "launches": int(self.launches),
                "seconds": self.seconds, "flops": self.flops, "bytes": self.bytes}


class FeatMeas(C.Structure):
    """uvio_hp_feat_meas_t: one Feature::uvs / uvs_norm / timestamps entry"""
    _fields_ = [("cam", C.c_int), ("t", C.c_double), ("u", C.c_float), ("v", C.c_float), ("un", C.c_float),
                ("vn", C.c_float)]


class FeatResult(C.Structure):
    """uvio_hp_feat_result_t: what an updater call left on a feature"""
    _fields_ = [("featid", C.c_uint64), ("status", C.c_int), ("to_delete", C.c_int), ("p_FinG", C.c_double * 3),
                ("chi2", C.c_double)]


_P = C.POINTER
_D = C.c_double
_I = C.c_int

# (name, restype, argtypes) for the product C ABI; the oracle exports the same entries with orc_
SIGNATURES = [
    ("options_default", _I, [_P(Options)]),
    ("options_load", _I, [C.c_char_p, _P(Options)]),
    ("create", _I, [_P(Options), _I, _P(C.c_void_p)]),
    ("destroy", _I, [C.c_void_p]),
    ("last_error", C.c_char_p, [C.c_void_p]),
    ("initialize_with_gt", _I, [C.c_void_p, _P(_D)]),
    ("feed_imu", _I, [C.c_void_p, _D, _P(_D), _P(_D)]),
    ("feed_imu_batch", _I, [C.c_void_p, C.c_int, _P(_D), _P(_D), _P(_D)]),
    ("feed_simulation", _I, [C.c_void_p, _D, _I, _P(_I), _P(_I), _P(C.c_uint64), _P(C.c_float)]),
    ("feed_camera", _I, [C.c_void_p, _D, _I, _P(_I), _P(_P(C.c_uint8)), _P(_I), _P(_P(C.c_uint8))]),
    ("feed_uwb", _I, [C.c_void_p, _D, _I, _P(C.c_uint64), _P(_D)]),
    ("init_anchors", _I, [C.c_void_p, _I, _P(Anchor)]),
    ("initialized", _I, [C.c_void_p, _P(_I)]),
    ("get_imu_state", _I, [C.c_void_p, _P(_D), _P(_D)]),
    ("get_cov_dim", _I, [C.c_void_p, _P(_I)]),
    ("get_cov", _I, [C.c_void_p, _P(_D), _I]),
    ("get_state_vector", _I, [C.c_void_p, _P(_D), _I, _P(_I), _P(_I), _I, _P(_I)]),
    ("get_fej_vector", _I, [C.c_void_p, _P(_D), _I, _P(_I)]),
    ("get_timing", _I, [C.c_void_p, _P(Timing)]),
    ("get_clone_times", _I, [C.c_void_p, _P(_D), _I, _P(_I)]),
    ("get_active_tracks", _I, [C.c_void_p, _P(_D), _P(C.c_uint64), _P(_D), _P(_D), _P(_I), _I, _P(_I)]),
    ("set_kernel_timing", _I, [C.c_void_p, _I]),
    ("get_kernel_stats", _I, [C.c_void_p, _I, _P(KStat), _I, _P(_I)]),
    ("feed_camera_device", _I, [C.c_void_p, _D, _I, _P(_I), _P(C.c_void_p), _P(_I), _P(_P(C.c_uint8))]),
    ("get_tracks", _I, [C.c_void_p, _I, _P(C.c_uint64), _P(C.c_float), _I, _P(_I)]),
    ("get_pyramid", _I, [C.c_void_p, _I, _I, _P(_I), _P(_I), _P(C.c_uint8), _P(C.c_int16), C.c_size_t]),
    ("debug_last_msckf", _I, [C.c_void_p, _P(C.c_uint64), _P(_D), _P(_I), _P(_D), _I, _P(_I)]),
    ("debug_frame_feats", _I, [C.c_void_p, _P(_I), _P(C.c_uint64), _P(_D), _P(_I), _P(_D), _I, _P(_I)]),
    ("ekf_update", _I, [_P(_D), _I, _P(_I), _I, _P(_D), _I, _P(_D), _D, _P(_D)]),
    ("msckf_compressed_update", _I, [_P(_D), _I, _P(_I), _I, _P(_D), _I, _P(_D), _D, _P(_D)]),
    ("compress", _I, [_P(_D), _I, _I, _P(_D)]),
    ("undistort", _I, [_I, _P(_D), _I, _P(C.c_float), _P(C.c_float), _P(C.c_uint8)]),
    ("set_state", _I, [C.c_void_p, _P(_D), _P(_D), _I, _P(_D), _I, _I]),
    ("propagate_and_clone", _I, [C.c_void_p, _D]),
    ("msckf_update", _I, [C.c_void_p, _I, _P(C.c_uint64), _P(_I), _P(FeatMeas), _P(FeatResult)]),
    ("slam_update", _I, [C.c_void_p, _I, _P(C.c_uint64), _P(_I), _P(FeatMeas), _P(FeatResult)]),
    ("slam_delayed_init", _I, [C.c_void_p, _I, _P(C.c_uint64), _P(_I), _P(FeatMeas), _P(FeatResult)]),
    ("slam_change_anchors", _I, [C.c_void_p]),
    ("marginalize_slam", _I, [C.c_void_p]),
    ("marginalize_old_clone", _I, [C.c_void_p]),
    ("uwb_update_single", _I, [C.c_void_p, _D, C.c_uint64, _D, _P(_I)]),
    ("shard_unique_id", _I, [_P(C.c_uint8)]),
    ("shard_init_rccl", _I, [C.c_void_p, _I, _I, _P(C.c_uint8), _I]),
    ("shard_init_host", _I, [C.c_void_p, _I, _I, C.c_void_p, C.c_void_p, _I]),
    ("shard_partition", _I, [_P(_I), _I, _I, _P(_I)]),
    ("debug_grid_order", _I, [_P(C.c_uint8), _P(_I), _I, _I, _I, _P(_I), _P(_I)]),
    ("debug_grid_stats", _I, [C.c_void_p, _P(C.c_uint64), _P(C.c_uint64)]),
]

# uvio_hp_allreduce_fn: int (*)(double *buf, size_t count, void *user)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, _P(_D), C.c_size_t, C.c_void_p)

# every symbol declared in include/uvio_hp.h
EXPORTED = ["uvio_hp_" + s[0] for s in SIGNATURES]


MISSING = set()  # entry points an older build under UVIO_HP_AB_OLD=1 (A/B runs, tools/gpu_ab.sh) does not export


def bind(lib, prefix, names=None):
    """Bind the declared signatures; a missing entry point raises, except in an explicit A/B run against an
    older build (UVIO_HP_AB_OLD=1 with UVIO_HP_LIB), where it is recorded in MISSING and reported."""
    ab_old = os.environ.get("UVIO_HP_AB_OLD") == "1" and "UVIO_HP_LIB" in os.environ
    for name, res, args in SIGNATURES:
        if names is not None and name not in names:
            continue
        if ab_old and prefix == "uvio_hp_" and not hasattr(lib, prefix + name):
            MISSING.add(name)
            continue
        f = getattr(lib, prefix + name)
        f.restype = res
        f.argtypes = args
    if MISSING:
        import sys
        sys.stderr.write("uvio_amd: A/B library %s lacks %s\n" % (os.environ["UVIO_HP_LIB"], ", ".join(sorted(MISSING))))
    return lib


_lib = None


def load():
    """Load libuvio_hp.so (built in-tree).  Raises if it is missing: there is no fallback path."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libuvio_hp.so not built: run `python -m uvio_amd.build` (hipcc, gfx950)")
        # In a process that also uses PyTorch-ROCm (the tests / bench harness), torch's bundled HIP
        # runtime must be loaded first so the library's HIP symbols bind to the same runtime; two HIP
        # runtimes in one process can leave the second without a device.  Without torch the system
        # ROCm runtime is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = bind(C.CDLL(LIB_PATH), "uvio_hp_")
    return _lib


def check(rc, lib=None, handle=None, what=""):
    if rc != 0:
        msg = ""
        if lib is not None and handle is not None:
            try:
                msg = (lib.uvio_hp_last_error(handle) or b"").decode()
            except Exception:  # noqa: BLE001
                msg = ""
        raise RuntimeError("%s failed: %s %s" % (what, ERRNAMES.get(rc, rc), msg))
    return rc
