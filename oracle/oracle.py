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
              "ekf_update", "compress", "debug_last_msckf", "debug_frame_feats", "get_fej_vector",
              "msckf_compressed_update", "feed_camera", "get_tracks", "get_pyramid", "get_active_tracks", "initialized"]

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
        fm, i32p = C.POINTER(N.FeatMeas), C.POINTER(C.c_int)
        lib.orc_updater.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_uint64), i32p, fm, i32p, i32p]
        lib.orc_propagate_and_clone.argtypes = [C.c_void_p, C.c_double]
        lib.orc_slam_change_anchors.argtypes = [C.c_void_p]
        lib.orc_marginalize_slam.argtypes = [C.c_void_p]
        lib.orc_marginalize_old_clone.argtypes = [C.c_void_p]
        lib.orc_uwb_update_single.argtypes = [C.c_void_p, C.c_double, C.c_uint64, C.c_double, i32p]
        u64p, dp = C.POINTER(C.c_uint64), C.POINTER(C.c_double)
        lib.orc_set_steer.argtypes = [C.c_void_p, C.c_int, C.c_int, i32p, u64p, dp, i32p, dp]
        lib.orc_get_steer_log.argtypes = [C.c_void_p, i32p, u64p, i32p, C.POINTER(C.c_int64), dp, dp, dp, i32p, i32p,
                                          C.c_int, i32p]
        lib.orc_static_initialize.argtypes = [C.POINTER(N.Options), C.c_int, dp, dp, dp, C.c_int, dp, dp]
        lib.orc_chi2_quantile95.restype = C.c_double
        lib.orc_chi2_quantile95.argtypes = [C.c_int]
        lib.orc_camera_distort.argtypes = [C.POINTER(N.Camera), C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                           C.POINTER(C.c_double), C.POINTER(C.c_double)]
        lib.orc_camera_undistort.argtypes = [C.POINTER(N.Camera), C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        u8, i16, f32, f64, i32 = (C.POINTER(C.c_uint8), C.POINTER(C.c_int16), C.POINTER(C.c_float),
                                  C.POINTER(C.c_double), C.c_int)
        lib.orc_equalize_hist.argtypes = [u8, i32, i32, u8]
        lib.orc_pyr_down.argtypes = [u8, i32, i32, u8]
        lib.orc_scharr.argtypes = [u8, i32, i32, i16]
        lib.orc_pyramid_levels.argtypes = [i32, i32, i32, i32]
        lib.orc_fast.argtypes = [u8, i32, i32, i32, i32, i32, i32, i32, f32, i32, C.POINTER(C.c_int)]
        lib.orc_grid_order.argtypes = [f32, i32, i32, C.POINTER(C.c_int)]
        lib.orc_corner_subpix.argtypes = [u8, i32, i32, f32, i32, i32, i32, C.c_double]
        lib.orc_lk.argtypes = [u8, u8, i32, i32, i32, i32, i32, C.c_float, f32, f32, u8, i32]
        lib.orc_ransac_mask.argtypes = [f32, f32, f32, f32, i32, C.c_double, C.c_double, i32, u8]
        lib.orc_fundamental_7pt.argtypes = [f64, f64, f64, f64, f64]
        ip = C.POINTER(C.c_int)
        lib.orc_probe_boxplus.argtypes = [C.c_void_p, f64, i32]
        lib.orc_probe_predict.argtypes = [C.c_void_p, f64, f64, f64, f64, i32, ip, ip, ip, i32, ip]
        lib.orc_probe_uwb.argtypes = [C.c_void_p, C.c_uint64, f64, f64, i32, ip, ip, ip, i32, ip]
        lib.orc_probe_feature_jacobian.argtypes = [C.c_void_p, i32, i32, ip, f64, f32, f32, f64, f64, i32, C.c_double,
                                                   f64, f64, f64, i32, ip, ip, ip, i32, ip]
        lib.orc_probe_triangulate.argtypes = [C.c_void_p, i32, ip, f64, f32, f32, i32, f64, ip, f64]
        _lib = lib
    return _lib


class OracleManager(VioManager):
    """The CPU restatement behind the same Python surface as the product."""

    _prefix = "orc_"

    @classmethod
    def _load(cls):
        return load()

    def _updater(self, name, features):
        """The reference updaters on the oracle's state; per feature: still in feature_vec (used) and to_delete"""
        which = {"msckf_update": 0, "slam_update": 1, "slam_delayed_init": 2}[name]
        ids, off, arr = self.pack_features(features)
        n = max(len(features), 1)
        kept, dele = (C.c_int * n)(), (C.c_int * n)()
        rc = self._lib.orc_updater(self._h, which, len(features), ids, off, arr, kept, dele)
        if rc != 0:
            raise RuntimeError("orc_%s failed (%d)" % (name, rc))
        return [{"featid": int(f[0]), "used": bool(kept[i]), "to_delete": bool(dele[i])} for i, f in enumerate(features)]

    # ---- probes of single restated routines (oracle/src/probe.cpp; tests/test_fd_goldens.py) ----
    @staticmethod
    def _dp(a):
        return a.ctypes.data_as(C.POINTER(C.c_double))

    @staticmethod
    def _ip(a):
        return a.ctypes.data_as(C.POINTER(C.c_int))

    def _check_probe(self, rc, what):
        if rc != 0:
            raise RuntimeError("orc_probe_%s failed (%d)" % (what, rc))

    def probe_boxplus(self, dx):
        """x <- x boxplus dx on every variable (Type::update), dx indexed by covariance id"""
        dx = np.ascontiguousarray(dx, dtype=np.float64)
        self._check_probe(self._lib.orc_probe_boxplus(self._h, self._dp(dx), dx.size), "boxplus")

    def probe_predict(self, dm, dp):
        """Propagator::predict_and_compute on one IMU interval: (F, Qd, [(cov id, size)] of the phi order); the
        IMU mean is replaced by the prediction.  dm / dp: (t, wm[3], am[3])"""
        dm = np.ascontiguousarray(dm, dtype=np.float64)
        dp = np.ascontiguousarray(dp, dtype=np.float64)
        cap = 64 * 64
        F, Q = np.zeros(cap), np.zeros(cap)
        ids, sz = np.zeros(16, np.int32), np.zeros(16, np.int32)
        n, nv = C.c_int(), C.c_int()
        self._check_probe(self._lib.orc_probe_predict(self._h, self._dp(dm), self._dp(dp), self._dp(F), self._dp(Q), cap,
                                                      C.byref(n), self._ip(ids), self._ip(sz), 16, C.byref(nv)), "predict")
        k = n.value
        return F[:k * k].reshape(k, k), Q[:k * k].reshape(k, k), list(zip(ids[:nv.value], sz[:nv.value]))

    def probe_uwb(self, anchor_id):
        """(predicted range, H_x, [(cov id, size)]) of UVioUpdaterHelper::get_uwb_jacobian_single"""
        H = np.zeros(64)
        ids, sz = np.zeros(8, np.int32), np.zeros(8, np.int32)
        pred, nc, nv = C.c_double(), C.c_int(), C.c_int()
        self._check_probe(self._lib.orc_probe_uwb(self._h, C.c_uint64(int(anchor_id)), C.byref(pred), self._dp(H), 64,
                                                  C.byref(nc), self._ip(ids), self._ip(sz), 8, C.byref(nv)), "uwb")
        return pred.value, H[:nc.value].copy(), list(zip(ids[:nv.value], sz[:nv.value]))

    def probe_feature_jacobian(self, rep, cams, times, uv, uvn, lam, uvn0=(0.0, 0.0), anchor_cam=-1, anchor_time=-1.0):
        """(res, H_f, H_x, [(cov id, size)]) of UpdaterHelper::get_feature_jacobian_full for a landmark with value
        lam in representation rep"""
        m = len(cams)
        cams = np.ascontiguousarray(cams, dtype=np.int32)
        times = np.ascontiguousarray(times, dtype=np.float64)
        uv = np.ascontiguousarray(uv, dtype=np.float32).reshape(-1)
        uvn = np.ascontiguousarray(uvn, dtype=np.float32).reshape(-1)
        lam = np.ascontiguousarray(lam, dtype=np.float64)
        u0 = np.ascontiguousarray(uvn0, dtype=np.float64)
        cap = 512
        res, Hf, Hx = np.zeros(2 * m), np.zeros(2 * m * 3), np.zeros(2 * m * cap)
        ids, sz = np.zeros(128, np.int32), np.zeros(128, np.int32)
        nc, nv = C.c_int(), C.c_int()
        fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
        self._check_probe(self._lib.orc_probe_feature_jacobian(
            self._h, rep, m, self._ip(cams), self._dp(times), fp(uv), fp(uvn), self._dp(lam), self._dp(u0), anchor_cam,
            C.c_double(anchor_time), self._dp(res), self._dp(Hf), self._dp(Hx), cap, C.byref(nc), self._ip(ids),
            self._ip(sz), 128, C.byref(nv)), "feature_jacobian")
        dim = 1 if rep == 5 else 3
        return (res, Hf[:2 * m * dim].reshape(2 * m, dim), Hx[:2 * m * nc.value].reshape(2 * m, nc.value),
                list(zip(ids[:nv.value], sz[:nv.value])))

    def probe_triangulate(self, cams, times, uv, uvn, refine=True):
        """FeatureInitializer::single_triangulation (+ single_gaussnewton): (ok, p_FinG, p_FinA, anchor cam, time)"""
        m = len(cams)
        cams = np.ascontiguousarray(cams, dtype=np.int32)
        times = np.ascontiguousarray(times, dtype=np.float64)
        uv = np.ascontiguousarray(uv, dtype=np.float32).reshape(-1)
        uvn = np.ascontiguousarray(uvn, dtype=np.float32).reshape(-1)
        out = np.zeros(6)
        ac, at = C.c_int(), C.c_double()
        fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
        ok = self._lib.orc_probe_triangulate(self._h, m, self._ip(cams), self._dp(times), fp(uv), fp(uvn),
                                             1 if refine else 0, self._dp(out), C.byref(ac), C.byref(at))
        return bool(ok), out[:3].copy(), out[3:].copy(), ac.value, at.value

    def feed_measurement_imu_batch(self, t, wm, am):
        for i in range(len(t)):
            self.feed_measurement_imu(float(t[i]), wm[i], am[i])

    def uwb_update_single(self, t, anchor_id, rng):
        a = C.c_int(0)
        rc = self._lib.orc_uwb_update_single(self._h, C.c_double(t), C.c_uint64(int(anchor_id)), C.c_double(rng),
                                             C.byref(a))
        if rc != 0:
            raise RuntimeError("orc_uwb_update_single failed (%d)" % rc)
        return bool(a.value)

    def set_steer(self, frame_feats):
        """Lock-step steering (oracle/src/flip.h, updater.h FrameDebug): the device's per-feature results of the
        frame this oracle processes next (VioManager.debug_frame_feats()); None turns steering off."""
        if frame_feats is None:
            self._lib.orc_set_steer(self._h, 0, 0, None, None, None, None, None)
            return
        kind, ids, pG, st, c2 = [np.ascontiguousarray(a) for a in frame_feats]
        kind, st = kind.astype(np.int32), st.astype(np.int32)
        pG = np.ascontiguousarray(pG, dtype=np.float64)
        ids = ids.astype(np.uint64)
        c2 = c2.astype(np.float64)
        self._lib.orc_set_steer(self._h, 1, len(ids), kind.ctypes.data_as(C.POINTER(C.c_int)),
                                ids.ctypes.data_as(C.POINTER(C.c_uint64)), _dp(pG), st.ctypes.data_as(C.POINTER(C.c_int)),
                                _dp(c2))
        self._steer_keep = (kind, ids, pG, st, c2)

    def steer_log(self):
        """Steering events since creation: list of dicts (kind, featid, stage, index, margin, before, after,
        found, candidates)."""
        cap = 4096
        i32 = lambda: np.zeros(cap, dtype=np.int32)
        kind, stage, found, cands = i32(), i32(), i32(), i32()
        ids = np.zeros(cap, dtype=np.uint64)
        index = np.zeros(cap, dtype=np.int64)
        margin, before, after = np.zeros(cap), np.zeros(cap), np.zeros(cap)
        n = C.c_int()
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
        self._lib.orc_get_steer_log(self._h, ip(kind), ids.ctypes.data_as(C.POINTER(C.c_uint64)), ip(stage),
                                    index.ctypes.data_as(C.POINTER(C.c_int64)), _dp(margin), _dp(before), _dp(after),
                                    ip(found), ip(cands), cap, C.byref(n))
        keys = ("kind", "featid", "stage", "index", "margin", "before", "after", "found", "candidates")
        cols = (kind, ids, stage, index, margin, before, after, found, cands)
        return [{k: c[i].item() for k, c in zip(keys, cols)} for i in range(min(n.value, cap))]

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


def set_threads(n):
    """threads of the restated OpenCV calls (num_opencv_threads: LK per point, pyrDown / Scharr per row)"""
    lib = load()
    lib.orc_set_threads.argtypes = [C.c_int]
    return lib.orc_set_threads(int(n))


def static_initialize(opts, t, wm, am, wait_for_jerk):
    """StaticInitializer::initialize (StaticInitializer.cpp:37-165) on one IMU buffer: (t_init, state16) or None."""
    lib = load()
    t = np.ascontiguousarray(t, dtype=np.float64)
    wm = np.ascontiguousarray(wm, dtype=np.float64)
    am = np.ascontiguousarray(am, dtype=np.float64)
    ti = C.c_double()
    x = np.zeros(16)
    ok = lib.orc_static_initialize(C.byref(opts), len(t), _dp(t), _dp(wm), _dp(am), int(bool(wait_for_jerk)), C.byref(ti),
                                   _dp(x))
    return (ti.value, x) if ok else None


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


def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _f32(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _img(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    assert img.ndim == 2
    return img, img.shape[1], img.shape[0]


def equalize_hist(img):
    """cv::equalizeHist restatement (oracle/src/tracker.cpp)."""
    img, w, h = _img(img)
    out = np.empty_like(img)
    load().orc_equalize_hist(_u8(img), w, h, _u8(out))
    return out


def pyr_down(img):
    """cv::pyrDown restatement: ((w+1)/2, (h+1)/2), 5x5 binomial, BORDER_REFLECT_101."""
    img, w, h = _img(img)
    out = np.empty(((h + 1) // 2, (w + 1) // 2), dtype=np.uint8)
    load().orc_pyr_down(_u8(img), w, h, _u8(out))
    return out


def scharr(img):
    """calcSharrDeriv restatement: (h, w, 2) int16 (dx, dy)."""
    img, w, h = _img(img)
    out = np.empty((h, w, 2), dtype=np.int16)
    load().orc_scharr(_u8(img), w, h, out.ctypes.data_as(C.POINTER(C.c_int16)))
    return out


def pyramid_levels(w, h, win=15, max_level=5):
    return load().orc_pyramid_levels(w, h, win, max_level)


def fast(img, thr, roi=None):
    """cv::FAST(img(roi), thr, nonmax=true) restatement: (k, 3) float32 of (x, y, response), ROI coords."""
    img, w, h = _img(img)
    x0, y0, rw, rh = roi if roi is not None else (0, 0, w, h)
    cap = rw * rh
    out = np.zeros((cap, 3), dtype=np.float32)
    n = C.c_int(0)
    rc = load().orc_fast(_u8(img), w, h, x0, y0, rw, rh, thr, _f32(out), cap, C.byref(n))
    assert rc == 0
    return out[:n.value]


def grid_order(resp, mode=0):
    """Grider_GRID.h:128 on one cell's cv::FAST responses (raster order): the raster indices in the order
    std::sort(compare_response) leaves them (mode 0), std::stable_sort (1) or std::partial_sort over the
    whole range (2, introsort's heap-sort fallback)."""
    r = np.ascontiguousarray(resp, dtype=np.float32).ravel()
    out = np.zeros(r.size, dtype=np.int32)
    rc = load().orc_grid_order(_f32(r), r.size, mode, out.ctypes.data_as(C.POINTER(C.c_int)))
    assert rc == 0
    return out


def corner_subpix(img, pts, win=5, max_iters=20, eps=1e-3):
    img, w, h = _img(img)
    p = np.array(pts, dtype=np.float32, order="C").reshape(-1, 2)
    load().orc_corner_subpix(_u8(img), w, h, _f32(p), p.shape[0], win, max_iters, eps)
    return p


def lk(prev, nxt, p0, p1=None, win=15, max_level=5, max_iters=30, eps=0.01):
    """calcOpticalFlowPyrLK(OPTFLOW_USE_INITIAL_FLOW) restatement: (p1, status)."""
    prev, w, h = _img(prev)
    nxt, w2, h2 = _img(nxt)
    assert (w, h) == (w2, h2)
    a = np.array(p0, dtype=np.float32, order="C").reshape(-1, 2)
    b = np.array(a if p1 is None else p1, dtype=np.float32, order="C").reshape(-1, 2)
    st = np.zeros(a.shape[0], dtype=np.uint8)
    load().orc_lk(_u8(prev), _u8(nxt), w, h, win, max_level, max_iters, eps, _f32(a), _f32(b), _u8(st), a.shape[0])
    return b, st


def ransac_mask(p0, p1, thr, conf=0.999, max_iters=1000):
    """findFundamentalMat(FM_RANSAC) restatement: inlier mask (uint8) of the n correspondences."""
    p0 = np.asarray(p0, dtype=np.float32)
    p1 = np.asarray(p1, dtype=np.float32)
    cols = [np.ascontiguousarray(c) for c in (p0[:, 0], p0[:, 1], p1[:, 0], p1[:, 1])]
    m = np.zeros(p0.shape[0], dtype=np.uint8)
    load().orc_ransac_mask(*[_f32(c) for c in cols], p0.shape[0], thr, conf, max_iters, _u8(m))
    return m


def fundamental_7pt(p0, p1):
    """7-point solver restatement: list of the (<= 3) 3x3 fundamental matrices."""
    p0 = np.asarray(p0, dtype=np.float64)
    p1 = np.asarray(p1, dtype=np.float64)
    cols = [np.ascontiguousarray(c) for c in (p0[:, 0], p0[:, 1], p1[:, 0], p1[:, 1])]
    F = np.zeros(27)
    n = load().orc_fundamental_7pt(*[_dp(c) for c in cols], _dp(F))
    return [F[9 * k:9 * k + 9].reshape(3, 3) for k in range(n)]


def camera_undistort(cam, uv):
    lib = load()
    uv = np.ascontiguousarray(uv, dtype=np.float32).reshape(-1, 2)
    out = np.zeros_like(uv)
    lib.orc_camera_undistort(C.byref(cam), uv.shape[0], uv.ctypes.data_as(C.POINTER(C.c_float)),
                             out.ctypes.data_as(C.POINTER(C.c_float)))
    return out
