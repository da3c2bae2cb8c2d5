"""ORACLE — test infrastructure only.

ctypes binding of ``oracle/build/liboracle.so``, the CPU restatement of the reference path (see
oracle/src/*.h headers for the reference file:line each function follows).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only as the
checker / CPU baseline.  The product (uvio_amd/) never imports or links it.

Parity status: the reference (OpenVINS/uvio, Eigen + OpenCV + Boost) cannot be built in this image
and its tests hold no golden vectors for this path.  The restatement is pinned by
independent numeric fixtures instead (tests/golden/: scipy chi2 quantiles, finite-difference
Jacobians, numpy QR / Kalman identities) — "parity unpinned" against the reference binary itself.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from uvio_amd import _native as N
from uvio_amd.manager import VioManager

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_ORC_NAMES = ["create", "destroy", "initialize_with_gt", "feed_imu", "feed_simulation", "feed_uwb", "init_anchors",
              "get_imu_state", "get_cov_dim", "get_cov", "get_state_vector", "get_timing", "get_clone_times",
              "ekf_update", "compress", "debug_last_msckf", "get_fej_vector",
              "msckf_compressed_update", "feed_camera", "get_tracks", "get_pyramid"]

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        N.bind(lib, "orc_", _ORC_NAMES)
        lib.orc_create.argtypes = [C.POINTER(N.Options), C.POINTER(C.c_void_p)]
        lib.orc_set_state.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int,
                                      C.POINTER(C.c_double), C.c_int]
        lib.orc_chi2_quantile95.restype = C.c_double
        lib.orc_chi2_quantile95.argtypes = [C.c_int]
        lib.orc_camera_distort.argtypes = [C.POINTER(N.Camera), C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                           C.POINTER(C.c_double), C.POINTER(C.c_double)]
        lib.orc_camera_undistort.argtypes = [C.POINTER(N.Camera), C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        _lib = lib
    return _lib


class OracleManager(VioManager):
    """The CPU restatement behind the same Python surface as the product."""

    _prefix = "orc_"

    @classmethod
    def _load(cls):
        return load()

    def set_state(self, val, fej, P):
        """Lock-step parity: adopt another implementation's mean / FEJ / covariance."""
        val = np.ascontiguousarray(val, dtype=np.float64)
        fej = np.ascontiguousarray(fej, dtype=np.float64)
        P = np.ascontiguousarray(P, dtype=np.float64)
        rc = self._lib.orc_set_state(self._h, _dp(val), _dp(fej), val.size, _dp(P), P.shape[0])
        if rc != 0:
            raise RuntimeError("orc_set_state: layout mismatch (%d)" % rc)


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def chi2_quantile95(dof):
    return load().orc_chi2_quantile95(int(dof))


def ekf_update(P, H_index, H, res, sigma2, compressed=False):
    lib = load()
    P = np.array(P, dtype=np.float64, order="C", copy=True)
    H = np.ascontiguousarray(H, dtype=np.float64)
    res = np.ascontiguousarray(res, dtype=np.float64)
    idx = np.ascontiguousarray(H_index, dtype=np.int32)
    n_ = P.shape[0]
    r, n = H.shape
    dx = np.zeros(n_)
    fn = lib.orc_msckf_compressed_update if compressed else lib.orc_ekf_update
    rc = fn(_dp(P), n_, idx.ctypes.data_as(C.POINTER(C.c_int)), n, _dp(H), r, _dp(res), float(sigma2), _dp(dx))
    if rc != 0:
        raise RuntimeError("orc_ekf_update failed %d" % rc)
    return P, dx


def compress(A):
    lib = load()
    A = np.ascontiguousarray(A, dtype=np.float64)
    m, nc = A.shape
    R = np.zeros((nc, nc))
    lib.orc_compress(_dp(A), m, nc - 1, _dp(R))
    return R


def camera_distort(cam, xy):
    lib = load()
    xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
    n = xy.shape[0]
    uv = np.zeros((n, 2))
    dzn = np.zeros((n, 2, 2))
    dzeta = np.zeros((n, 2, 8))
    lib.orc_camera_distort(C.byref(cam), n, _dp(xy), _dp(uv), _dp(dzn), _dp(dzeta))
    return uv, dzn, dzeta


def camera_undistort(cam, uv):
    lib = load()
    uv = np.ascontiguousarray(uv, dtype=np.float32).reshape(-1, 2)
    out = np.zeros_like(uv)
    lib.orc_camera_undistort(C.byref(cam), uv.shape[0], uv.ctypes.data_as(C.POINTER(C.c_float)),
                             out.ctypes.data_as(C.POINTER(C.c_float)))
    return out
