"""Python mirror of the reference manager surface (ov_msckf::VioManager / uvio::UVioManager).

Method names follow the reference C++ API (VioManager.h:75-111, UVioManager.h:48-73):
``feed_measurement_imu``, ``feed_measurement_simulation``, ``feed_measurement_uwb``,
``try_to_initialize_uwb_anchors``, ``initialize_with_gt``, ``initialized``, ``get_state`` ...
Every call goes through the C ABI of libuvio_hp.so (include/uvio_hp.h); the estimator state and the
covariance live on the MI355X.  Errors the reference would turn into ``std::exit`` raise here.
"""
import ctypes as C

import numpy as np

from . import _native as N


def load_options(yaml_path=None, **overrides):
    """VioManagerOptions::print_and_load equivalent: defaults, then the YAML keys, then overrides."""
    lib = N.load()
    opts = N.Options()
    N.check(lib.uvio_hp_options_default(C.byref(opts)), what="options_default")
    if yaml_path is not None:
        N.check(lib.uvio_hp_options_load(yaml_path.encode(), C.byref(opts)), what="options_load(%s)" % yaml_path)
    apply_overrides(opts, overrides)
    return opts


def _mask_ptrs(masks, ncam):
    """per-camera u8 masks (None: no mask for that camera) -> (kept arrays, uint8_t*[ncam])"""
    mk = [None if m is None else np.ascontiguousarray(m, dtype=np.uint8) for m in masks]
    ptrs = [C.POINTER(C.c_uint8)() if m is None else m.ctypes.data_as(C.POINTER(C.c_uint8)) for m in mk]
    return mk, (C.POINTER(C.c_uint8) * ncam)(*ptrs)


def apply_overrides(opts, overrides):
    for k, v in overrides.items():
        if not hasattr(opts, k):
            raise KeyError(k)
        setattr(opts, k, v)
    return opts


def shard_unique_id():
    """ncclGetUniqueId (rank 0): 128 bytes to distribute to every rank for enable_feature_sharding."""
    lib = N.load()
    uid = (C.c_uint8 * 128)()
    rc = lib.uvio_hp_shard_unique_id(uid)
    if rc != 0:
        msg = (lib.uvio_hp_last_error(None) or b"").decode()
        raise RuntimeError("shard_unique_id failed: %s %s" % (N.ERRNAMES.get(rc, rc), msg))
    return bytes(uid)


def host_allreduce_callback(group=None):
    """uvio_hp_allreduce_fn over torch.distributed: the library hands a host buffer of doubles, the
    callback sums it in place across the ranks of `group` (default group when None)."""
    import torch
    import torch.distributed as dist

    def _allreduce(buf, count, user):
        try:
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,)))
            dist.all_reduce(t, group=group)
            return 0
        except Exception:  # noqa: BLE001
            return 1

    return N.ALLREDUCE_FN(_allreduce)


def shard_partition(rows, world):
    """The feature split the sharded update uses: bounds (world + 1) of contiguous row-balanced chunks."""
    lib = N.load()
    r = np.ascontiguousarray(rows, dtype=np.int32)
    b = np.zeros(world + 1, dtype=np.int32)
    rc = lib.uvio_hp_shard_partition(r.ctypes.data_as(C.POINTER(C.c_int)), len(r), world,
                                     b.ctypes.data_as(C.POINTER(C.c_int)))
    if rc != 0:
        raise RuntimeError("shard_partition failed: %s" % N.ERRNAMES.get(rc, rc))
    return b


def pack_sim_frame(feats):
    """(counts, ids uint64[n], uv float32[n, 2]) of one TrackSIM frame, cameras concatenated."""
    counts = [len(f[0]) for f in feats]
    ids = np.ascontiguousarray(np.concatenate([np.asarray(f[0], dtype=np.uint64) for f in feats]))
    uv = np.ascontiguousarray(np.concatenate([np.asarray(f[1], dtype=np.float32).reshape(-1, 2) for f in feats]))
    return counts, ids, uv


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class VioManager:
    """Handle on one estimator instance (one MI355X device)."""

    _prefix = "uvio_hp_"

    def __init__(self, options, device=0):
        self._lib = self._load()
        self._h = C.c_void_p()
        rc = self._call("create", C.byref(options), device, C.byref(self._h)) if self._prefix == "uvio_hp_" else \
            self._call("create", C.byref(options), C.byref(self._h))
        if rc != 0:
            why = ""
            if self._prefix == "uvio_hp_":
                msg = self._call("last_error", None)
                why = ": " + msg.decode() if msg else ""
            raise RuntimeError("%screate failed: %s%s" % (self._prefix, N.ERRNAMES.get(rc, rc), why))
        self.options = options

    @classmethod
    def _load(cls):
        return N.load()

    def _call(self, name, *args):
        return getattr(self._lib, self._prefix + name)(*args)

    def _check(self, rc, what):
        if rc != 0:
            msg = ""
            if self._prefix == "uvio_hp_":
                msg = (self._lib.uvio_hp_last_error(self._h) or b"").decode()
            raise RuntimeError("%s failed: %s %s" % (what, N.ERRNAMES.get(rc, rc), msg))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._call("destroy", self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ---- feature sharding across ranks (include/uvio_hp.h) ----
    def enable_feature_sharding(self, rank, world, backend="rccl", unique_id=None, group=None, min_features=1):
        """Split every MSCKF update with >= min_features features across `world` replicas of this filter
        (one per rank, all fed the same stream).  backend "rccl": the library all-reduces on its own
        stream over an RCCL communicator (unique_id: the 128 bytes of shard_unique_id() made on rank 0 and
        shared with every rank).  backend "host": the blocks go through torch.distributed.all_reduce on
        `group` (e.g. gloo; ranks may then share one GPU)."""
        if backend == "rccl":
            if unique_id is None or len(unique_id) != 128:
                raise ValueError("rccl backend needs the 128-byte unique id of shard_unique_id()")
            uid = (C.c_uint8 * 128)(*bytearray(unique_id))
            self._check(self._call("shard_init_rccl", self._h, rank, world, uid, min_features), "shard_init_rccl")
        elif backend == "host":
            self._allreduce_cb = host_allreduce_callback(group)  # kept alive with the handle
            fn = C.cast(self._allreduce_cb, C.c_void_p)
            self._check(self._call("shard_init_host", self._h, rank, world, fn, None, min_features),
                        "shard_init_host")
        else:
            raise ValueError("backend must be 'rccl' or 'host'")

    # ---- feeds ----
    def initialize_with_gt(self, imustate17):
        x = np.ascontiguousarray(imustate17, dtype=np.float64)
        assert x.shape == (17,)
        self._check(self._call("initialize_with_gt", self._h, _dp(x)), "initialize_with_gt")

    def feed_measurement_imu(self, t, wm, am):
        w = (C.c_double * 3)(*wm)
        a = (C.c_double * 3)(*am)
        self._check(self._call("feed_imu", self._h, C.c_double(t), w, a), "feed_measurement_imu")

    def feed_measurement_imu_batch(self, t, wm, am):
        """n consecutive feed_measurement_imu calls: t (n,), wm (n,3), am (n,3)."""
        t = np.ascontiguousarray(t, dtype=np.float64)
        wm = np.ascontiguousarray(wm, dtype=np.float64)
        am = np.ascontiguousarray(am, dtype=np.float64)
        n = t.shape[0]
        assert wm.shape == (n, 3) and am.shape == (n, 3)
        if "feed_imu_batch" in N.MISSING:  # an older library under A/B
            for i in range(n):
                self.feed_measurement_imu(float(t[i]), wm[i], am[i])
            return
        self._check(self._call("feed_imu_batch", self._h, n, _dp(t), _dp(wm), _dp(am)), "feed_measurement_imu_batch")

    def feed_measurement_simulation(self, t, camids, feats, allow_uninit=False):
        """feats[i] = (ids uint64[n], uv float32[n,2]) for camera camids[i] (TrackSIM input)."""
        return self.feed_measurement_simulation_packed(t, camids, *pack_sim_frame(feats), allow_uninit=allow_uninit)

    def feed_measurement_simulation_packed(self, t, camids, counts, ids, uv, allow_uninit=False):
        """feed_measurement_simulation with the cameras' tracks already concatenated (pack_sim_frame)."""
        ncam = len(camids)
        cam = (C.c_int * ncam)(*camids)
        cnt = (C.c_int * ncam)(*[int(c) for c in counts])
        rc = self._call("feed_simulation", self._h, C.c_double(t), ncam, cam, cnt,
                        ids.ctypes.data_as(C.POINTER(C.c_uint64)), uv.ctypes.data_as(C.POINTER(C.c_float)))
        if rc == N.E_STATE and allow_uninit:
            return rc
        self._check(rc, "feed_measurement_simulation")
        return rc

    def feed_measurement_camera(self, t, camids, images, masks=None, allow_uninit=False):
        """VioManager::feed_measurement_camera: images[i] is a u8 (H, W) array for camera camids[i]."""
        ncam = len(camids)
        imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        cam = (C.c_int * ncam)(*camids)
        ptrs = (C.POINTER(C.c_uint8) * ncam)(*[im.ctypes.data_as(C.POINTER(C.c_uint8)) for im in imgs])
        strides = (C.c_int * ncam)(*[im.strides[0] for im in imgs])
        mptr = None
        if masks is not None:
            mk, mptr = _mask_ptrs(masks, ncam)
        rc = self._call("feed_camera", self._h, C.c_double(t), ncam, cam, ptrs, strides, mptr)
        if rc == N.E_STATE and allow_uninit:
            return rc
        self._check(rc, "feed_measurement_camera")
        return rc

    def feed_measurement_camera_device(self, t, camids, images, masks=None, allow_uninit=False):
        """feed_measurement_camera with images already in HBM: images[i] is a uint8 (H, W) CUDA tensor
        (row stride = tensor stride).  The producer stream is synchronized before the call."""
        import torch
        ncam = len(camids)
        for im in images:
            if not (im.is_cuda and im.dtype == torch.uint8 and im.dim() == 2 and im.stride(1) == 1):
                raise ValueError("images must be 2-D uint8 CUDA tensors with unit column stride")
        torch.cuda.current_stream(images[0].device).synchronize()
        cam = (C.c_int * ncam)(*camids)
        ptrs = (C.c_void_p * ncam)(*[im.data_ptr() for im in images])
        strides = (C.c_int * ncam)(*[im.stride(0) for im in images])
        mptr = None
        if masks is not None:
            mk, mptr = _mask_ptrs(masks, ncam)
        rc = self._call("feed_camera_device", self._h, C.c_double(t), ncam, cam, ptrs, strides, mptr)
        if rc == N.E_STATE and allow_uninit:
            return rc
        self._check(rc, "feed_measurement_camera_device")
        return rc

    def get_tracks(self, cam):
        """(ids uint64[n], uv float32[n, 2]) of the KLT tracks of camera `cam` after the last feed."""
        n = C.c_int()
        cap = 4096
        ids = np.zeros(cap, dtype=np.uint64)
        uv = np.zeros((cap, 2), dtype=np.float32)
        self._check(self._call("get_tracks", self._h, cam, ids.ctypes.data_as(C.POINTER(C.c_uint64)),
                               uv.ctypes.data_as(C.POINTER(C.c_float)), cap, C.byref(n)), "get_tracks")
        return ids[:n.value].copy(), uv[:n.value].copy()

    def grid_stats(self):
        """(cells, introsort_cells): the tracker's FAST cells so far and how many had > 16 candidates (the
        cells whose selection std::sort's introsort tie order decides, Grider_GRID.h:128)."""
        c, i = C.c_uint64(), C.c_uint64()
        self._check(self._call("debug_grid_stats", self._h, C.byref(c), C.byref(i)), "debug_grid_stats")
        return int(c.value), int(i.value)

    def get_pyramid(self, cam, level):
        """(img u8 (h, w), der int16 (h, w, 2)) of the last pyramid level of camera `cam`."""
        w, h = C.c_int(), C.c_int()
        self._check(self._call("get_pyramid", self._h, cam, level, C.byref(w), C.byref(h), None, None, 0),
                    "get_pyramid")
        img = np.zeros((h.value, w.value), dtype=np.uint8)
        der = np.zeros((h.value, w.value, 2), dtype=np.int16)
        self._check(self._call("get_pyramid", self._h, cam, level, C.byref(w), C.byref(h),
                               img.ctypes.data_as(C.POINTER(C.c_uint8)), der.ctypes.data_as(C.POINTER(C.c_int16)),
                               img.size), "get_pyramid")
        return img, der

    def feed_measurement_uwb(self, t, anchor_ids, ranges):
        n = len(anchor_ids)
        ids = (C.c_uint64 * n)(*anchor_ids)
        r = (C.c_double * n)(*ranges)
        self._check(self._call("feed_uwb", self._h, C.c_double(t), n, ids, r), "feed_measurement_uwb")

    def try_to_initialize_uwb_anchors(self, anchors):
        n = len(anchors)
        arr = (N.Anchor * max(n, 1))(*anchors)
        self._check(self._call("init_anchors", self._h, n, arr), "try_to_initialize_uwb_anchors")

    # ---- updater-level boundary (include/uvio_hp.h; UpdaterMSCKF.h:68, UpdaterSLAM.h:70-87, UpdaterUWB.h:55) ----
    @staticmethod
    def pack_features(features):
        """features: [(featid, [(cam, t, u, v, un, vn), ...]), ...] in observation order -> flat C arrays"""
        ids = (C.c_uint64 * max(len(features), 1))(*[int(f[0]) for f in features])
        offs, meas = [0], []
        for _, ms in features:
            for (cam, t, u, v, un, vn) in ms:
                meas.append(N.FeatMeas(int(cam), float(t), float(u), float(v), float(un), float(vn)))
            offs.append(len(meas))
        off = (C.c_int * len(offs))(*offs)
        arr = (N.FeatMeas * max(len(meas), 1))(*meas)
        return ids, off, arr

    def set_state(self, val, fej, P):
        """Adopt a state snapshot (mean, first estimates, covariance) in this state's layout."""
        val = np.ascontiguousarray(val, dtype=np.float64)
        fej = np.ascontiguousarray(fej, dtype=np.float64)
        P = np.ascontiguousarray(P, dtype=np.float64)
        self._check(self._call("set_state", self._h, _dp(val), _dp(fej), val.size, _dp(P), P.shape[0], P.shape[0]),
                    "set_state")

    def propagate_and_clone(self, t):
        self._check(self._call("propagate_and_clone", self._h, C.c_double(t)), "propagate_and_clone")

    def _updater(self, name, features):
        ids, off, arr = self.pack_features(features)
        out = (N.FeatResult * max(len(features), 1))()
        self._check(self._call(name, self._h, len(features), ids, off, arr, out), name)
        return [{"featid": int(o.featid), "status": o.status, "used": o.status == 0, "to_delete": bool(o.to_delete),
                 "p_FinG": np.array(o.p_FinG[:]), "chi2": o.chi2} for o in out[:len(features)]]

    def msckf_update(self, features):
        """UpdaterMSCKF::update on the current state; one result dict per feature"""
        return self._updater("msckf_update", features)

    def slam_update(self, features):
        """UpdaterSLAM::update (the features must be SLAM landmarks of the state)"""
        return self._updater("slam_update", features)

    def slam_delayed_init(self, features):
        """UpdaterSLAM::delayed_init: accepted features become SLAM landmarks"""
        return self._updater("slam_delayed_init", features)

    def slam_change_anchors(self):
        self._check(self._call("slam_change_anchors", self._h), "slam_change_anchors")

    def marginalize_slam(self):
        self._check(self._call("marginalize_slam", self._h), "marginalize_slam")

    def marginalize_old_clone(self):
        self._check(self._call("marginalize_old_clone", self._h), "marginalize_old_clone")

    def uwb_update_single(self, t, anchor_id, rng):
        """UpdaterUWB::update_single; True when the range passed the chi2 test and updated the state"""
        a = C.c_int(0)
        self._check(self._call("uwb_update_single", self._h, C.c_double(t), C.c_uint64(int(anchor_id)),
                               C.c_double(rng), C.byref(a)), "uwb_update_single")
        return bool(a.value)

    # ---- getters ----
    def initialized(self):
        """VioManager::initialized (VioManager.h:99): initialize_with_gt ran or an initializer succeeded."""
        out = C.c_int()
        self._check(self._call("initialized", self._h, C.byref(out)), "initialized")
        return bool(out.value)

    def get_imu_state(self):
        t = C.c_double()
        out = np.zeros(16)
        self._check(self._call("get_imu_state", self._h, C.byref(t), _dp(out)), "get_imu_state")
        return t.value, out

    def cov_dim(self):
        n = C.c_int()
        self._check(self._call("get_cov_dim", self._h, C.byref(n)), "get_cov_dim")
        return n.value

    def get_cov(self):
        n = self.cov_dim()
        P = np.zeros((n, n))
        self._check(self._call("get_cov", self._h, _dp(P), n), "get_cov")
        return P

    def get_state_vector(self):
        cap = 4096
        out = np.zeros(cap)
        meta = np.zeros(3 * 1024, dtype=np.int32)
        ln, nv = C.c_int(), C.c_int()
        self._check(self._call("get_state_vector", self._h, _dp(out), cap, C.byref(ln),
                               meta.ctypes.data_as(C.POINTER(C.c_int)), meta.size, C.byref(nv)), "get_state_vector")
        return out[:ln.value].copy(), meta[:3 * nv.value].reshape(-1, 3).copy()

    def get_fej_vector(self):
        out = np.zeros(4096)
        ln = C.c_int()
        self._check(self._call("get_fej_vector", self._h, _dp(out), out.size, C.byref(ln)), "get_fej_vector")
        return out[:ln.value].copy()

    def get_timing(self):
        return self.get_timing_raw().as_dict()

    def get_timing_raw(self):
        """the timing struct itself (uvio_hp_timing_t); .as_dict() gives get_timing()'s dict"""
        t = N.Timing()
        self._check(self._call("get_timing", self._h, C.byref(t)), "get_timing")
        return t

    def set_kernel_timing(self, period=1):
        """Live per-class device timing of the roofline kernels (HIP events, include/uvio_hp.h): the launches
        of every `period`-th frame are timed (0 = off)."""
        self._check(self._call("set_kernel_timing", self._h, int(period)), "set_kernel_timing")

    def kernel_stats(self, flush=True):
        """{class name: {kernels, bound, launches, seconds, flops, bytes}} cumulative since switched on."""
        cap = 16
        arr = (N.KStat * cap)()
        n = C.c_int()
        self._check(self._call("get_kernel_stats", self._h, 1 if flush else 0, arr, cap, C.byref(n)),
                    "get_kernel_stats")
        return {d["name"]: d for d in (arr[i].as_dict() for i in range(min(n.value, cap)))}

    def debug_last_msckf(self):
        cap = 8192
        ids = np.zeros(cap, dtype=np.uint64)
        pG = np.zeros((cap, 3))
        st = np.zeros(cap, dtype=np.int32)
        c2 = np.zeros(cap)
        n = C.c_int()
        self._check(self._call("debug_last_msckf", self._h, ids.ctypes.data_as(C.POINTER(C.c_uint64)), _dp(pG),
                               st.ctypes.data_as(C.POINTER(C.c_int)), _dp(c2), cap, C.byref(n)), "debug_last_msckf")
        k = n.value
        return ids[:k].copy(), pG[:k].copy(), st[:k].copy(), c2[:k].copy()

    def debug_frame_feats(self):
        """Per-feature results of every updater call of the last frame: (kind, ids, p_FinG, status, chi2);
        kind 0 MSCKF update, 1 SLAM update, 2 delayed initialization."""
        cap = 16384
        kind = np.zeros(cap, dtype=np.int32)
        ids = np.zeros(cap, dtype=np.uint64)
        pG = np.zeros((cap, 3))
        st = np.zeros(cap, dtype=np.int32)
        c2 = np.zeros(cap)
        n = C.c_int()
        self._check(self._call("debug_frame_feats", self._h, kind.ctypes.data_as(C.POINTER(C.c_int)),
                               ids.ctypes.data_as(C.POINTER(C.c_uint64)), _dp(pG), st.ctypes.data_as(C.POINTER(C.c_int)),
                               _dp(c2), cap, C.byref(n)), "debug_frame_feats")
        k = min(n.value, cap)
        return kind[:k].copy(), ids[:k].copy(), pG[:k].copy(), st[:k].copy(), c2[:k].copy()

    def get_active_tracks(self):
        """VioManager::get_active_tracks: (time, {featid: p_FinG}, {featid: (u, v, depth)})."""
        cap = 16384
        t = C.c_double()
        ids = np.zeros(cap, dtype=np.uint64)
        pos = np.zeros((cap, 3))
        uvd = np.zeros((cap, 3))
        ok = np.zeros(cap, dtype=np.int32)
        n = C.c_int()
        self._check(self._call("get_active_tracks", self._h, C.byref(t), ids.ctypes.data_as(C.POINTER(C.c_uint64)),
                               _dp(pos), _dp(uvd), ok.ctypes.data_as(C.POINTER(C.c_int)), cap, C.byref(n)),
                    "get_active_tracks")
        k = n.value
        P = {int(ids[i]): pos[i].copy() for i in range(k)}
        D = {int(ids[i]): uvd[i].copy() for i in range(k) if ok[i]}
        return t.value, P, D

    def get_clone_times(self):
        out = np.zeros(256)
        n = C.c_int()
        self._check(self._call("get_clone_times", self._h, _dp(out), 256, C.byref(n)), "get_clone_times")
        return out[:n.value].copy()


def ekf_update(P, H_index, H, res, sigma2, compressed=False):
    """StateHelper::EKFUpdate on a standalone covariance, on the device (returns P_new, dx).
    compressed=True: measurement compression + EKFUpdate as UpdaterMSCKF.cpp:274-286 does it."""
    lib = N.load()
    P = np.array(P, dtype=np.float64, order="C", copy=True)
    H = np.ascontiguousarray(H, dtype=np.float64)
    res = np.ascontiguousarray(res, dtype=np.float64)
    idx = np.ascontiguousarray(H_index, dtype=np.int32)
    Nn = P.shape[0]
    r, n = H.shape
    dx = np.zeros(Nn)
    fn = lib.uvio_hp_msckf_compressed_update if compressed else lib.uvio_hp_ekf_update
    rc = fn(_dp(P), Nn, idx.ctypes.data_as(C.POINTER(C.c_int)), n, _dp(H), r, _dp(res), float(sigma2), _dp(dx))
    N.check(rc, what="uvio_hp_ekf_update")
    return P, dx


def compress(A):
    """R factor of [H | res] (measurement_compress_inplace semantics), on the device."""
    lib = N.load()
    A = np.ascontiguousarray(A, dtype=np.float64)
    m, nc = A.shape
    R = np.zeros((nc, nc))
    N.check(lib.uvio_hp_compress(_dp(A), m, nc - 1, _dp(R)), what="uvio_hp_compress")
    return R


def grid_order(cells, kmax=0, depth=-1):
    """Grider_GRID.h:128's std::sort as the device's FAST selection runs it (uvio_hp_debug_grid_order).
    cells: per cell the cv::FAST responses in raster order.  Returns (arrangements, tops): per cell the raster
    indices as libstdc++'s introsort loop leaves them and, for kmax > 0, the first min(n, kmax) raster indices
    of the sorted cell.  depth 0 forces the heap-sort fallback."""
    lib = N.load()
    off = np.zeros(len(cells) + 1, dtype=np.int32)
    for i, c in enumerate(cells):
        off[i + 1] = off[i] + len(c)
    resp = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
    for i, c in enumerate(cells):
        resp[off[i]:off[i + 1]] = np.asarray(c, dtype=np.int64)
    arr = np.zeros(max(int(off[-1]), 1), dtype=np.int32)
    top = np.full(max(len(cells) * kmax, 1), -1, dtype=np.int32)
    ip = C.POINTER(C.c_int)
    rc = lib.uvio_hp_debug_grid_order(resp.ctypes.data_as(C.POINTER(C.c_uint8)), off.ctypes.data_as(ip), len(cells),
                                      kmax, depth, arr.ctypes.data_as(ip), top.ctypes.data_as(ip))
    N.check(rc, what="uvio_hp_debug_grid_order")
    arrs = [arr[off[i]:off[i + 1]].copy() for i in range(len(cells))]
    tops = [top[i * kmax:i * kmax + min(kmax, len(c))].copy() for i, c in enumerate(cells)] if kmax > 0 else None
    return arrs, tops


def undistort(cam, uv, return_ambiguous=False):
    """CamBase::undistort_f (CamBase.h:89) of n pixel points on the device (uvio_hp_undistort); cam is a
    Camera of the options.  With return_ambiguous, also the per-point flags of the points the library
    recomputed with the host's libm tan (equidistant points next to a float rounding boundary)."""
    lib = N.load()
    uv = np.ascontiguousarray(uv, dtype=np.float32).reshape(-1, 2)
    out = np.zeros_like(uv)
    amb = np.zeros(uv.shape[0], dtype=np.uint8)
    intr = np.array(cam.intrinsics[:], dtype=np.float64)
    fp = C.POINTER(C.c_float)
    rc = lib.uvio_hp_undistort(int(cam.model), _dp(intr), uv.shape[0], uv.ctypes.data_as(fp), out.ctypes.data_as(fp),
                               amb.ctypes.data_as(C.POINTER(C.c_uint8)))
    N.check(rc, what="uvio_hp_undistort")
    return (out, amb) if return_ambiguous else out
