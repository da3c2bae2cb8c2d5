"""GPU parity: the HIP path (libuvio_hp.so) against the CPU restatement (oracle/) on identical inputs.

Tolerances (FP64 everywhere):
  * standalone EKF update: P and dx within 1e-10 relative (max abs diff / max abs value)
  * compression R factor: rows equal up to sign within 1e-9 relative, R^T R == A^T A to 1e-12
  * compressed MSCKF update (Givens compression + EKFUpdate vs the device's information form), including
    exactly rank-deficient H: P and dx within 1e-9 relative
  * lock-step frames: before every camera frame the oracle adopts the device's mean / FEJ / covariance,
    then both process the same frame; the per-feature triangulations agree to 1e-9 m, chi2 to 1e-11
    relative, no feature changes its accept/reject decision, and the resulting state / P agree to 1e-10
    relative (measured on MI355X: 2e-11 m, 5e-14, 3e-13, 1.4e-11).
  * free-running estimator: both run the whole stream on their own; after 30 frames the state agrees
    to 1e-5 relative and the poses to 1e-5 m / rad (measured: 2e-7, 9e-7).

A frame in which such a flip happens (see below) is allowed looser bounds (p < 1e-6 m, chi2 < 1e-5,
x < 1e-8, P < 1e-9 relative) and at most two of them per 30-frame run (measured: one frame, p 4.8e-8,
chi2 2.2e-7, x 2.0e-10, P 2.2e-11; every other frame at the strict bounds).

Why lock-step and not bitwise: the reference quantizes every predicted pixel to float
(CamBase::distort_d -> distort_f, CamBase.h:130) and stores measured uv as float, and its feature
refinement runs on float residuals (FeatureInitializer.cpp:241-271).  A 1e-16 difference in a
triangulated point (the device sums in a different order than the CPU) can, rarely, flip one float
rounding of a predicted pixel, i.e. move a residual by one float ulp (~3e-5 px at u~400).  The filter
carries such a flip forward, so free runs drift apart slowly while every single step matches to
rounding (DESIGN.md "Parity").
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


def _spd(n, rng):
    A = rng.standard_normal((n, n))
    return A @ A.T / n + 1e-3 * np.eye(n)


@pytest.mark.parametrize("N,n,r", [(30, 12, 5), (120, 40, 60), (266, 100, 100), (266, 100, 37)])
def test_ekf_update_matches_oracle(N, n, r):
    import uvio_amd as U
    from oracle import oracle as O
    rng = np.random.default_rng(N * 7 + r)
    P = _spd(N, rng)
    idx = rng.choice(N, n, replace=False).astype(np.int32)
    H = rng.standard_normal((r, n))
    res = rng.standard_normal(r)
    Pg, dxg = U.ekf_update(P, idx, H, res, 1.0)
    Po, dxo = O.ekf_update(P, idx, H, res, 1.0)
    assert _rel(Pg, Po) < 1e-10
    assert _rel(dxg, dxo) < 1e-10
    assert np.array_equal(Pg, Pg.T)


@pytest.mark.parametrize("N,n,m,null", [(60, 30, 200, 0), (150, 94, 3000, 0), (150, 94, 5738, 6), (266, 100, 9000, 4)])
def test_compressed_update_matches_oracle(N, n, m, null):
    """UpdaterMSCKF.cpp:274-286 (Givens compression + EKFUpdate) vs the device's information-form
    update; `null` > 0 makes H exactly rank deficient, as real MSCKF batches are (gauge directions)."""
    import uvio_amd as U
    from oracle import oracle as O
    rng = np.random.default_rng(N + n + m)
    P = _spd(N, rng) * 1e-2
    idx = rng.choice(N, n, replace=False).astype(np.int32)
    H = rng.standard_normal((m, n)) * np.logspace(0, 3, n)[None, :]
    if null:
        Qn, _ = np.linalg.qr(rng.standard_normal((n, null)))
        H = H - (H @ Qn) @ Qn.T
    res = rng.standard_normal(m)
    Pg, dxg = U.ekf_update(P, idx, H, res, 1.0, compressed=True)
    Po, dxo = O.ekf_update(P, idx, H, res, 1.0, compressed=True)
    assert _rel(Pg, Po) < 1e-9
    assert _rel(dxg, dxo) < 1e-9
    assert np.array_equal(Pg, Pg.T)


@pytest.mark.parametrize("m,n", [(50, 10), (600, 40), (9000, 100)])
def test_compress_matches_givens(m, n):
    import uvio_amd as U
    from oracle import oracle as O
    rng = np.random.default_rng(m + n)
    A = rng.standard_normal((m, n + 1)) * np.logspace(0, 2, n + 1)[None, :]
    Rg = U.compress(A)
    Ro = O.compress(A)
    # rows equal up to a sign
    s = np.sign(np.diag(Rg)) * np.sign(np.diag(Ro))
    s[s == 0] = 1
    assert _rel(Rg * s[:, None], Ro) < 1e-9
    # invariant: R^T R == A^T A
    G = A.T @ A
    assert _rel(Rg.T @ Rg, G) < 1e-12


def _sim(opts, n_frames, seed=5, **simkw):
    from uvio_amd.sim import SimStream
    return SimStream(opts, duration=n_frames / opts.track_frequency + 1.2, seed=seed, **simkw)


def _free_run(opts, n_frames, **simkw):
    import uvio_amd as U
    from oracle import oracle as O
    s = _sim(opts, n_frames, **simkw)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    out = {"g": [], "o": []}
    s.run(g, n_frames=n_frames, on_frame=lambda nf, t: out["g"].append(_snap(g)))
    s.run(o, n_frames=n_frames, on_frame=lambda nf, t: out["o"].append(_snap(o)))
    return out["g"], out["o"]


def _snap(m):
    x, meta = m.get_state_vector()
    return {"x": x, "meta": meta, "P": m.get_cov(), "timing": m.get_timing(), "imu": m.get_imu_state()[1],
            "feats": m.debug_last_msckf()}


def _lockstep(opts, n_frames, **simkw):
    import uvio_amd as U
    from oracle import oracle as O
    s = _sim(opts, n_frames, **simkw)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    steps = []

    def before(nf, t):
        o.set_state(g.get_state_vector()[0], g.get_fej_vector(), g.get_cov())

    def after(nf, t):
        steps.append((_snap(g), _snap(o)))

    s.run([g, o], n_frames=n_frames, before_frame=before, on_frame=after)
    return steps


def _compare_feats(fg, fo):
    ig, pg, sg, cg = fg
    io, po, so, co = fo
    assert np.array_equal(np.sort(ig), np.sort(io))
    mo = {int(i): k for k, i in enumerate(io)}
    worst_p, worst_c = 0.0, 0.0
    for k, i in enumerate(ig):
        j = mo[int(i)]
        assert sg[k] == so[j], ("accept/reject differs", int(i), sg[k], so[j], cg[k], co[j])
        if sg[k] != 1:
            worst_p = max(worst_p, np.abs(pg[k] - po[j]).max())
            worst_c = max(worst_c, abs(cg[k] - co[j]) / max(abs(co[j]), 1.0))
    return worst_p, worst_c


def _check_lockstep(steps, max_flips=2):
    """Strict per-frame bounds, except on frames with a float-rounding flip of a predicted pixel (see the
    module docstring): those are detected by their triangulation / chi2 jump, must stay rare and within
    the looser bounds such a one-ulp residual change produces."""
    worst = {"p": 0.0, "c": 0.0, "x": 0.0, "P": 0.0}
    flips = []
    for k, (a, b) in enumerate(steps):
        assert a["x"].shape == b["x"].shape
        assert a["P"].shape == b["P"].shape
        assert a["timing"]["n_msckf"] == b["timing"]["n_msckf"]
        assert a["timing"]["n_slam"] == b["timing"]["n_slam"]
        assert a["timing"]["n_slam_delayed"] == b["timing"]["n_slam_delayed"]
        p, c = _compare_feats(a["feats"], b["feats"])
        x, P = _rel(a["x"], b["x"]), _rel(a["P"], b["P"])
        if p > 1e-9 or c > 1e-11:
            flips.append((k, p, c, x, P))
            assert p < 1e-6 and c < 1e-5 and x < 1e-8 and P < 1e-9, flips[-1]
            continue
        worst["p"], worst["c"] = max(worst["p"], p), max(worst["c"], c)
        worst["x"] = max(worst["x"], x)
        worst["P"] = max(worst["P"], P)
    assert len(flips) <= max_flips, flips
    assert worst["p"] < 1e-9, worst
    assert worst["c"] < 1e-11, worst
    assert worst["x"] < 1e-10, worst
    assert worst["P"] < 1e-10, worst
    return worst


def _pose_err(a, b):
    from uvio_amd.sim import quat_2_rot
    Ra, Rb = quat_2_rot(a["imu"][:4]), quat_2_rot(b["imu"][:4])
    dth = np.arccos(np.clip((np.trace(Ra @ Rb.T) - 1) / 2, -1, 1))
    return dth, np.abs(a["imu"][4:7] - b["imu"][4:7]).max()


def test_lockstep_msckf_parity(euroc_yaml):
    import uvio_amd as U
    opts = U.load_options(euroc_yaml, max_msckf_in_update=200, max_slam_features=0)
    steps = _lockstep(opts, 30, spawn=120)
    assert len(steps) == 30
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 300
    _check_lockstep(steps)


def test_lockstep_slam_parity(euroc_yaml):
    import uvio_amd as U
    opts = U.load_options(euroc_yaml, max_msckf_in_update=100, max_slam_features=20, max_slam_in_update=10,
                          dt_slam_delay=0.3)
    steps = _lockstep(opts, 30, spawn=80, frac_long=0.3)
    assert sum(a["timing"]["n_slam"] for a, _ in steps) > 0
    assert sum(a["timing"]["n_slam_delayed"] for a, _ in steps) > 0
    _check_lockstep(steps)


def test_free_run_msckf_parity(euroc_yaml):
    import uvio_amd as U
    opts = U.load_options(euroc_yaml, max_msckf_in_update=200, max_slam_features=0)
    G, Ov = _free_run(opts, 30, spawn=120)
    assert len(G) == len(Ov) == 30
    for a, b in zip(G, Ov):
        assert a["x"].shape == b["x"].shape
        assert a["timing"]["n_msckf"] == b["timing"]["n_msckf"]
    assert _rel(G[-1]["x"], Ov[-1]["x"]) < 1e-5
    dth, dp = _pose_err(G[-1], Ov[-1])
    assert dth < 1e-5 and dp < 1e-5, (dth, dp)


def test_free_run_slam_parity(euroc_yaml):
    import uvio_amd as U
    opts = U.load_options(euroc_yaml, max_msckf_in_update=100, max_slam_features=20, max_slam_in_update=10,
                          dt_slam_delay=0.3)
    G, Ov = _free_run(opts, 30, spawn=80, frac_long=0.3)
    assert len(G) == len(Ov) == 30
    assert _rel(G[-1]["x"], Ov[-1]["x"]) < 1e-5
    dth, dp = _pose_err(G[-1], Ov[-1])
    assert dth < 1e-5 and dp < 1e-5, (dth, dp)


def make_anchors(N):
    """6 anchors at room corners / mid-walls, 2 fixed (uwb_config.yaml:6 n_anchors_to_fix 2)."""
    pos = [(6, 6, 0.5), (-6, 6, 2.5), (-6, -6, 0.5), (6, -6, 2.5), (0, 7, 1.5), (7, 0, 1.0)]
    out = []
    for i, p in enumerate(pos):
        a = N.Anchor()
        a.id = 100 + i
        a.fix = 1 if i < 2 else 0
        for k in range(3):
            a.p_AinG[k] = p[k]
        a.const_bias, a.dist_bias = 0.0, 0.0
        for k, v in enumerate([0.1, 0.1, 0.1, 0.01, 0.001]):
            a.cov_diag[k] = v
        out.append(a)
    return out


def test_lockstep_uwb_parity(euroc_yaml):
    """UpdaterUWB::update_single (UpdaterUWB.cpp:53-90) + UVioPropagator + anchor init, lock-step."""
    import uvio_amd as U
    from uvio_amd import _native as N
    from uvio_amd.sim import SimStream
    from oracle import oracle as O
    opts = U.load_options(euroc_yaml, max_msckf_in_update=60, max_slam_features=0, use_uwb=1,
                          do_calib_uwb_extrinsics=1, min_dist_to_use_uwb=0.05)
    for k, v in enumerate([0.05, -0.02, 0.03]):
        opts.p_IinU[k] = v
    anchors = make_anchors(N)
    n = 30
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=60, anchors=anchors, uwb_rate=10.0,
                    uwb_sigma=0.1)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    steps = []

    def init(m):
        m.try_to_initialize_uwb_anchors(anchors)

    def before(nf, t):
        o.set_state(g.get_state_vector()[0], g.get_fej_vector(), g.get_cov())

    def after(nf, t):
        steps.append((_snap(g), _snap(o)))

    sim.run([g, o], n_frames=n, before_frame=before, on_frame=after, after_init=init)
    # 4 non-fixed anchors x 5 + p_IinU 3 extra state dims
    assert steps[-1][0]["P"].shape[0] >= 15 + 1 + 28 + 6 * 12 + 20 + 3 - 6
    worst_x = max(_rel(a["x"], b["x"]) for a, b in steps)
    worst_P = max(_rel(a["P"], b["P"]) for a, b in steps)
    assert worst_x < 1e-10 and worst_P < 1e-10, (worst_x, worst_P)
