"""Independent goldens for the oracle's estimator Jacobians, on the CPU.

The reference cannot be built here, so these are what can catch an error the oracle and the device share:
each analytic Jacobian the restatement computes is compared with central finite differences of the SAME
restated model, perturbed through the reference's own error-state parametrization (Type::update: JPL
quaternions left-multiplied by [dtheta/2, 1], everything else additive; oracle/src/probe.cpp), on a live state
of the cfg 5 composite (rpng_sim 4 cameras, IMU intrinsics + g-sensitivity, UWB anchors, camera calibration).

  * UWB range (UVioUpdaterHelper.cpp:147-241): every block matches, except the anchor-position block, which
    the reference writes as (1 + dist_bias) H_n R_GtoI^T (:236) where the model's derivative is (1 + dist_bias)
    H_n: the test pins that the block equals the finite difference times R_GtoI^T, i.e. the reference's quirk,
    kept for parity and documented.
  * feature measurement (UpdaterHelper.cpp:32-424), all six LandmarkRepresentations: H_f against the
    landmark parameters, H_x against clones, camera extrinsics and intrinsics, anchor clone.
  * IMU propagation (Propagator.cpp:395-828, 964-1015): F of one IMU interval, including the Dw / Da / Tg /
    R_GYROtoIMU columns, against the finite-difference Jacobian of the predicted mean (analytical and rk4
    integration).
  * triangulation + Gauss-Newton (FeatureInitializer.cpp:30-375): noiseless views of a known point give it
    back; views from one position are rejected by the condition-number test.

Finite-difference accuracy: the reference rounds every predicted pixel to float (CamBase.h:130), ~3e-5 px at
these magnitudes, so the feature steps are 1e-3 (poses, landmark parameters) or sized per intrinsic, and the
tolerances below are relative to each column's norm.
"""
import os

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG5 = os.path.join(ROOT, "configs", "rpng_sim_uwb", "estimator_config.yaml")
K_IMU, K_VEC, K_QUAT, K_POSE, K_LANDMARK, K_ANCHOR = range(6)


def _vlen(kind, size):
    return size + (1 if kind in (K_IMU, K_QUAT, K_POSE) else 0)


def _rot(q):
    from uvio_amd.sim import quat_2_rot
    return quat_2_rot(np.asarray(q))


def boxminus(xa, xb, meta, N):
    """xa - xb in the error state (covariance ids): JPL R(dq (x) q) = R(dq) R(q), R(dq) = exp(-[axis]x angle)"""
    out = np.zeros(N)
    off = 0
    for kind, cid, size in meta:
        n = _vlen(kind, size)
        va, vb = xa[off:off + n], xb[off:off + n]
        if kind in (K_IMU, K_QUAT, K_POSE):
            # Type::update's dq = normalize([dtheta / 2, 1]) turns by 2 atan(|dtheta| / 2): invert that exactly
            r = -Rotation.from_matrix(_rot(va[:4]) @ _rot(vb[:4]).T).as_rotvec()
            phi = np.linalg.norm(r)
            out[cid:cid + 3] = r * (2 * np.tan(phi / 2) / phi) if phi > 0 else r
            out[cid + 3:cid + size] = va[4:] - vb[4:]
        else:
            out[cid:cid + size] = va - vb
        off += n
    return out


class Probe:
    """An oracle estimator run into a live cfg-5 state; evaluations at base boxplus dx (first estimates = base)."""

    def __init__(self, n_frames=22, **ov):
        import uvio_amd as U
        from oracle import oracle as O
        from uvio_amd.sim import SimStream
        kw = dict(max_clone_size=8, max_msckf_in_update=40, max_slam_features=6, max_slam_in_update=6,
                  dt_slam_delay=0.2)
        kw.update(ov)
        self.opts = U.load_options(CFG5, **kw)
        self.sim = SimStream(self.opts, duration=n_frames / self.opts.track_frequency + 1.2, seed=11, spawn=120,
                             frac_long=0.3, anchors=[self.opts.anchors[i] for i in range(self.opts.n_anchors)])
        self.o = O.OracleManager(self.opts)
        self.sim.run(self.o, n_frames=n_frames)
        self.x, self.meta = self.o.get_state_vector()
        self.P = self.o.get_cov()
        self.N = self.P.shape[0]
        self.reset()

    def reset(self):
        self.o.set_state(self.x, self.x, self.P)

    def at(self, dx, fn):
        self.reset()
        self.o.probe_boxplus(dx)
        return fn()

    def var(self, cid):
        off = 0
        for kind, c, size in self.meta:
            if c == cid:
                return kind, size, off
            off += _vlen(kind, size)
        raise KeyError(cid)

    def central(self, fn, cid, j, eps):
        dx = np.zeros(self.N)
        dx[cid + j] = eps
        fp = np.asarray(self.at(dx, fn), dtype=np.float64)
        dx[cid + j] = -eps
        fm = np.asarray(self.at(dx, fn), dtype=np.float64)
        self.reset()
        return (fp - fm) / (2 * eps)


@pytest.fixture(scope="module")
def probe():
    return Probe()


def test_boxminus_inverts_the_reference_update(probe):
    """the test's own error-state difference undoes Type::update (checks the JPL sign convention used below)"""
    rng = np.random.default_rng(2)
    dx = 1e-3 * rng.standard_normal(probe.N)
    probe.reset()
    probe.o.probe_boxplus(dx)
    x1 = probe.o.get_state_vector()[0]
    probe.reset()
    assert np.max(np.abs(boxminus(x1, probe.x, probe.meta, probe.N) - dx)) < 1e-9


def test_uwb_range_jacobian_finite_difference(probe):
    """get_uwb_jacobian_single (UVioUpdaterHelper.cpp:147-241) against central differences of the range model"""
    o = probe.o
    opts = probe.opts
    anchors = [opts.anchors[i] for i in range(opts.n_anchors)]
    R_GtoI = _rot(probe.x[:4])
    assert np.linalg.norm(R_GtoI - np.eye(3)) > 0.1  # a rotated platform: the anchor quirk is visible
    n_unfixed = 0
    for a in anchors:
        _, H, blocks = o.probe_uwb(a.id)
        col = 0
        for cid, size in blocks:
            kind, _, _ = probe.var(cid)
            fd = np.array([probe.central(lambda: o.probe_uwb(a.id)[0], cid, j, 1e-5) for j in range(size)])
            h = H[col:col + size]
            if kind == K_ANCHOR:
                n_unfixed += 1
                # const_bias / dist_bias columns match the model
                assert np.allclose(h[3:], fd[3:], rtol=1e-7, atol=1e-9), (h, fd)
                # the position columns: the reference's (1 + dist_bias) H_n R_GtoI^T (UVioUpdaterHelper.cpp:236)
                # = the model's derivative (1 + dist_bias) H_n, times R_GtoI^T
                assert np.allclose(h[:3], fd[:3] @ R_GtoI.T, rtol=1e-7, atol=1e-9), (h[:3], fd[:3])
                assert np.linalg.norm(h[:3] - fd[:3]) > 1e-3  # ... and not the model's derivative
            else:
                assert np.allclose(h, fd, rtol=1e-7, atol=1e-9), (kind, cid, h, fd)
            col += size
        assert col == H.size
    assert n_unfixed == sum(1 for a in anchors if not a.fix) > 0


def _landmark_views(probe, depth=4.0):
    """a point seen by one camera from every clone (cams 0..K-1 tried in order): (cams, times, uv, uvn, p_FinG,
    anchor cam, anchor time)"""
    from oracle import oracle as O
    opts = probe.opts
    x, meta = probe.x, probe.meta
    clones = []  # (time, R_GtoI, p_IinG)
    times = probe.o.get_clone_times()
    off = 0
    poses = []
    for kind, cid, size in meta:
        n = _vlen(kind, size)
        if kind == K_POSE:
            poses.append((cid, x[off:off + 7]))
        off += n
    # camera extrinsics come first (2 * K PoseJPL?) : the last len(times) poses are the clones, in time order
    cl = poses[-len(times):]
    ext = poses[:opts.num_cameras]
    for t, (_, v) in zip(times, cl):
        clones.append((t, _rot(v[:4]), v[4:7]))
    for c in range(opts.num_cameras):
        R_ItoC, p_IinC = _rot(ext[c][1][:4]), ext[c][1][4:7]
        t_a, R_a, p_a = clones[-1]
        R_GtoC = R_ItoC @ R_a
        p_CinG = p_a - R_GtoC.T @ p_IinC
        p_FinG = p_CinG + R_GtoC.T @ np.array([0.15, -0.1, 1.0]) * depth
        cams, ts, uv, uvn = [], [], [], []
        for t, R, p in clones:
            p_C = R_ItoC @ (R @ (p_FinG - p)) + p_IinC
            if p_C[2] < 0.5:
                continue
            cam = opts.cams[c]
            u, _, _ = O.camera_distort(cam, (p_C[:2] / p_C[2])[None, :])
            if not (0 < u[0, 0] < cam.width and 0 < u[0, 1] < cam.height):
                continue
            cams.append(c)
            ts.append(t)
            uv.append(u[0])
        if len(cams) >= 4:
            uv = np.array(uv, dtype=np.float32)
            uv_noisy = uv + np.float32(0.7) * np.float32(np.sin(np.arange(uv.size))).reshape(uv.shape)
            uvn = O.camera_undistort(opts.cams[c], uv_noisy)
            return np.array(cams), np.array(ts), uv_noisy, uvn, p_FinG, c, clones[-1][0], (R_ItoC, p_IinC, R_a, p_a)
    raise AssertionError("no camera sees the synthetic landmark")


def _lambda(rep, p):
    """LandmarkRepresentation parameters of the xyz point p (Landmark.cpp:65-144 set_from_xyz)"""
    if rep in (0, 2):
        return np.array(p)
    if rep in (1, 3):
        rho = 1 / np.linalg.norm(p)
        return np.array([np.arctan2(p[1], p[0]), np.arccos(rho * p[2]), rho])
    if rep == 4:
        return np.array([p[0] / p[2], p[1] / p[2], 1 / p[2]])
    return np.array([1 / p[2]])


@pytest.mark.parametrize("rep", [0, 1, 2, 3, 4, 5],
                         ids=["GLOBAL_3D", "GLOBAL_FULL_INVERSE_DEPTH", "ANCHORED_3D", "ANCHORED_FULL_INVERSE_DEPTH",
                              "ANCHORED_MSCKF_INVERSE_DEPTH", "ANCHORED_INVERSE_DEPTH_SINGLE"])
def test_feature_jacobian_finite_difference(probe, rep):
    """get_feature_jacobian_full (UpdaterHelper.cpp:192-424) + _representation (:32-190): H_f and H_x against
    central differences of the residual (res = z - h, so dres = -H dx)"""
    o = probe.o
    cams, ts, uv, uvn, p_FinG, ac, at, (R_ItoC, p_IinC, R_a, p_a) = _landmark_views(probe)
    p_FinA = R_ItoC @ (R_a @ (p_FinG - p_a)) + p_IinC
    rel = rep >= 2
    lam = _lambda(rep, p_FinA if rel else p_FinG)
    uvn0 = (p_FinA[0] / p_FinA[2], p_FinA[1] / p_FinA[2])

    def res_of(l=lam):
        return o.probe_feature_jacobian(rep, cams, ts, uv, uvn, l, uvn0, ac if rel else -1, at if rel else -1.0)[0]

    res, Hf, Hx, blocks = o.probe_feature_jacobian(rep, cams, ts, uv, uvn, lam, uvn0, ac if rel else -1,
                                                   at if rel else -1.0)
    assert 0.05 < np.abs(res).max() < 5  # the perturbed measurements: a residual of a pixel or so
    # landmark parameters
    for j in range(lam.size):
        e = 1e-3 * max(abs(lam[j]), 0.1)
        lp, lm = lam.copy(), lam.copy()
        lp[j] += e
        lm[j] -= e
        fd = -(res_of(lp) - res_of(lm)) / (2 * e)
        assert np.linalg.norm(fd - Hf[:, j]) <= 2e-3 * np.linalg.norm(Hf[:, j]), (j, fd, Hf[:, j])
    # state blocks
    col = 0
    kinds = set()
    for cid, size in blocks:
        kind, _, _ = probe.var(cid)
        kinds.add((kind, size))
        for j in range(size):
            if size == 8:  # camera intrinsics: fx fy cx cy in pixels, distortion coefficients
                e = 1.0 if j < 4 else 0.1  # the pixel is linear in each: no truncation error
            else:
                e = 1e-2  # poses: truncation ~(e / depth)^2, float-pixel noise ~3e-5 px / e
            fd = -probe.central(res_of, cid, j, e)
            h = Hx[:, col + j]
            assert np.linalg.norm(fd - h) <= 2e-3 * max(np.linalg.norm(h), 1.0), (kind, cid, j, fd, h)
        col += size
    assert col == Hx.shape[1]
    assert (K_POSE, 6) in kinds and (K_VEC, 8) in kinds  # clones / extrinsics and intrinsics were covered


@pytest.mark.parametrize("integration", [2, 1], ids=["analytical", "rk4"])
def test_propagation_F_finite_difference(integration):
    """compute_F_and_G_analytic (Propagator.cpp:683-828) with IMU intrinsics + g-sensitivity (compute_H_Dw / Da /
    Tg, :964-1015): F of one 5 ms IMU interval against the finite-difference Jacobian of the predicted mean over
    the same interval, at non-trivial intrinsics (Dw, Da off identity, Tg and R_GYROtoIMU non-zero)"""
    p = Probe(n_frames=8, integration=integration)
    o = p.o
    assert p.opts.do_calib_imu_intrinsics and p.opts.do_calib_imu_g_sensitivity
    rng = np.random.default_rng(4)
    # move the IMU intrinsics (Dw, Da, Tg: Vec; R_GYROtoIMU: JPLQuat) and the biases off their nominal values
    order_probe = o.probe_predict(np.zeros(7), np.r_[0.005, np.zeros(6)])[2]
    p.reset()
    dx = np.zeros(p.N)
    for cid, size in order_probe[1:]:
        dx[cid:cid + size] = 0.02 * rng.standard_normal(size)
    dx[9:15] = 0.01 * rng.standard_normal(6)
    p.reset()
    o.probe_boxplus(dx)
    p.x = o.get_state_vector()[0]
    p.reset()
    t0 = 10.0
    dm = np.r_[t0, 0.3, -0.2, 0.5, 0.4, -0.3, 9.6]
    dp = np.r_[t0 + 0.005, 0.35, -0.1, 0.45, 0.6, -0.2, 9.9]
    F, Qd, order = o.probe_predict(dm, dp)
    x1 = o.get_state_vector()[0]
    assert len(order) == 5 and F.shape[0] == 15 + 6 + 6 + 9 + 3  # IMU, Dw, Da, Tg, R_GYROtoIMU (kalibr model)

    def mean_after():
        o.probe_predict(dm, dp)
        return o.get_state_vector()[0]

    imu_id = order[0][0]
    col = 0
    worst = {}
    for cid, size in order:
        kind, _, _ = p.var(cid)
        for j in range(size):
            e = 1e-6
            dxp = np.zeros(p.N)
            dxp[cid + j] = e
            xp = p.at(dxp, mean_after)
            dxp[cid + j] = -e
            xm = p.at(dxp, mean_after)
            fd = (boxminus(xp, x1, p.meta, p.N) - boxminus(xm, x1, p.meta, p.N))[imu_id:imu_id + 15] / (2 * e)
            f = F[:15, col + j]
            worst[(int(cid), j)] = np.abs(fd - f).max()
        col += size
    p.reset()
    # analytical integration: the mean is the closed form F linearizes, so they agree to the differences' own
    # rounding (1e-16 / e); rk4: the mean integrates the two end samples while F uses their average, an O(dt^2)
    # model gap (measured 2.6e-6 at 5 ms, 6.5e-7 at 2.5 ms) against entries up to 1
    tol = 2e-9 if integration == 2 else 1e-5
    bad = {k: v for k, v in worst.items() if v > tol}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:12]
    assert max(worst.values()) > (0 if integration == 2 else 1e-7)
    # the intrinsic blocks are the identity on themselves
    assert np.allclose(F[15:, 15:], np.eye(F.shape[0] - 15))


def test_triangulation_exact_answer(probe):
    """single_triangulation + single_gaussnewton (FeatureInitializer.cpp:30-375) on noiseless views of a known
    point return it (to the float rounding of the stored pixels), and views from a single position are rejected
    by the condition-number test (:96-106)"""
    from oracle import oracle as O
    o = probe.o
    cams, ts, uv, uvn, p_FinG, ac, at, _ = _landmark_views(probe)
    opts = probe.opts
    # noiseless pixels of the same point
    _, _, _, _, _, _, _, (R_ItoC, p_IinC, _, _) = _landmark_views(probe)
    clone_R, clone_p = {}, {}
    x = probe.x
    times = list(o.get_clone_times())
    poses = []
    off = 0
    for kind, cid, size in probe.meta:
        n = _vlen(kind, size)
        if kind == K_POSE:
            poses.append(x[off:off + 7])
        off += n
    for t, v in zip(times, poses[-len(times):]):
        clone_R[t], clone_p[t] = _rot(v[:4]), v[4:7]
    uv0 = []
    for t in ts:
        p_C = R_ItoC @ (clone_R[t] @ (p_FinG - clone_p[t])) + p_IinC
        u, _, _ = O.camera_distort(opts.cams[int(cams[0])], (p_C[:2] / p_C[2])[None, :])
        uv0.append(u[0])
    uv0 = np.array(uv0, dtype=np.float32)
    uvn0 = O.camera_undistort(opts.cams[int(cams[0])], uv0)
    ok, pG, pA, acam, atime = o.probe_triangulate(cams, ts, uv0, uvn0, refine=False)
    assert ok and np.linalg.norm(pG - p_FinG) < 2e-4 * np.linalg.norm(p_FinG), (pG, p_FinG)
    ok, pG2, _, _, _ = o.probe_triangulate(cams, ts, uv0, uvn0, refine=True)
    assert ok and np.linalg.norm(pG2 - p_FinG) < 2e-4 * np.linalg.norm(p_FinG), (pG2, p_FinG)
    # with a pixel of noise the refinement lowers the reprojection error and stays within centimetres
    ok, pG3, _, _, _ = o.probe_triangulate(cams, ts, uv, uvn, refine=True)
    assert ok and np.linalg.norm(pG3 - p_FinG) < 0.1
    # all views from ONE clone time (zero baseline): A is rank deficient, cond > max_cond_number -> rejected
    same_t = np.full_like(ts, ts[-1])
    ok, _, _, _, _ = o.probe_triangulate(cams, same_t, uv0, uvn0, refine=False)
    assert not ok
