"""GPU parity of the Updater-level C ABI (include/uvio_hp.h "Updater-level boundary"):
uvio_hp_msckf_update / slam_delayed_init / slam_update / slam_change_anchors / marginalize_* /
propagate_and_clone / uwb_update_single called with caller-built features on a state snapshot, against
the oracle's restatement of the reference's own calls (UpdaterMSCKF::update, UpdaterSLAM::delayed_init /
update / change_anchors, StateHelper::marginalize_*, Propagator::propagate_and_clone,
UpdaterUWB::update_single) on the same snapshot and features.

The snapshot comes from a lock-step run of both managers over the simulated stream (so both hold the same
variables); features are the stream's TrackSIM measurements over the clone times, normalized with the
oracle's camera model.  Before each call the oracle adopts the device's state, so every call is compared
on identical inputs.  Tolerances as in test_gpu_parity.py's lock-step frames: the same features used /
erased / flagged to_delete, the same state layout, state and covariance within 1e-10 relative.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


def _sync(g, o):
    o.set_state(g.get_state_vector()[0], g.get_fej_vector(), g.get_cov())


def _same_state(g, o, tol=1e-10):
    xg, mg = g.get_state_vector()
    xo, mo = o.get_state_vector()
    assert np.array_equal(mg, mo), "state layouts differ"
    Pg, Po = g.get_cov(), o.get_cov()
    assert _rel(xg, xo) < tol, _rel(xg, xo)
    assert _rel(Pg, Po) < tol, _rel(Pg, Po)
    return _rel(xg, xo), _rel(Pg, Po)


def _tracks(sim, opts, frames):
    """featid -> [(cam, t, u, v, un, vn)] over the given sim frame indices, in observation order"""
    from oracle import oracle as O
    tr = {}
    for i in frames:
        t = float(sim.cam_t[i])
        for k, (ids, uv) in enumerate(sim.frames[i]):
            if len(ids) == 0:
                continue
            xy = O.camera_undistort(opts.cams[k], uv)
            for j, fid in enumerate(ids):
                tr.setdefault(int(fid), []).append((k, t, float(uv[j, 0]), float(uv[j, 1]), float(xy[j, 0]),
                                                    float(xy[j, 1])))
    return tr


def _frames_at(sim, times):
    idx = []
    for t in times:
        k = int(np.argmin(np.abs(sim.cam_t - t)))
        assert abs(sim.cam_t[k] - t) < 1e-9
        idx.append(k)
    return idx


def _feed_imu_until(sim, mgrs, t_from, t_to):
    lag = 1.0 / sim.imu_rate + 1e-9
    for i, t in enumerate(sim.imu_t):
        if t_from + lag <= t < t_to + lag:
            for m in mgrs:
                m.feed_measurement_imu(t, sim.wm[i], sim.am[i])


def _used(res):
    return [(r["featid"], r["used"], r["to_delete"]) for r in res]


def test_updater_level_calls_match_oracle(euroc_yaml):
    import uvio_amd as U
    from oracle import oracle as O
    from uvio_amd.sim import SimStream
    opts = U.load_options(euroc_yaml, max_msckf_in_update=60, max_slam_features=20, max_slam_in_update=10,
                          dt_slam_delay=100.0)  # no SLAM inside the frames: the landmarks come from the calls below
    n = 14
    sim = SimStream(opts, duration=(n + 6) / opts.track_frequency + 1.2, seed=11, spawn=40, frac_long=0.5)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    sim.run([g, o], n_frames=n, before_frame=lambda nf, t: _sync(g, o))
    _sync(g, o)
    ct = g.get_clone_times()
    assert len(ct) == opts.max_clone_size and np.allclose(ct, o.get_clone_times())
    window = _frames_at(sim, ct)
    t_last, i_next = float(ct[-1]), window[-1] + 1
    tracks = _tracks(sim, opts, window)
    nxt = set(int(f) for k in range(sim.K) for f in sim.frames[i_next][k][0])
    longf = sorted(f for f, m in tracks.items() if len(set(x[1] for x in m)) >= 6)
    # delayed-init candidates: long tracks that continue into the next frame; MSCKF: the other long ones
    dset = [(f, tracks[f]) for f in longf if f in nxt][:8]
    mset = [(f, tracks[f]) for f in longf if f not in dict(dset)][:40]
    short = [(10 ** 9 + k, tracks[f][:1]) for k, f in enumerate(longf[:2])]  # one measurement: too few
    assert len(dset) >= 4 and len(mset) >= 20

    # UpdaterMSCKF::update
    rg, ro = g.msckf_update(mset + short), o.msckf_update(mset + short)
    assert _used(rg) == _used(ro)
    assert sum(r["used"] for r in rg) >= 10
    assert all(r["status"] == 1 for r in rg[-len(short):])
    _same_state(g, o)

    # UpdaterSLAM::delayed_init: accepted features become landmarks (3 more covariance columns each)
    _sync(g, o)
    N0 = g.cov_dim()
    rg, ro = g.slam_delayed_init(dset), o.slam_delayed_init(dset)
    assert _used(rg) == _used(ro)
    nlm = sum(r["used"] for r in rg)
    assert nlm >= 2 and g.cov_dim() == N0 + 3 * nlm
    _same_state(g, o)

    # Propagator::propagate_and_clone to the next frame
    _sync(g, o)
    t_next = float(sim.cam_t[i_next])
    _feed_imu_until(sim, [g, o], t_last, t_next)
    g.propagate_and_clone(t_next)
    o.propagate_and_clone(t_next)
    assert g.get_clone_times()[-1] == t_next
    _same_state(g, o)

    # UpdaterSLAM::update with the landmarks' tracks including the new frame
    _sync(g, o)
    tracks2 = _tracks(sim, opts, window + [i_next])
    lms = [(f, tracks2[f]) for (f, _), r in zip(dset, rg) if r["used"]]
    rg2, ro2 = g.slam_update(lms), o.slam_update(lms)
    assert _used(rg2) == _used(ro2)
    assert sum(r["used"] for r in rg2) >= 1
    _same_state(g, o)

    # UpdaterSLAM::change_anchors, StateHelper::marginalize_slam / marginalize_old_clone
    for step in ("slam_change_anchors", "marginalize_slam", "marginalize_old_clone"):
        _sync(g, o)
        getattr(g, step)()
        getattr(o, step)()
        _same_state(g, o)
    assert len(g.get_clone_times()) == opts.max_clone_size
    g.close()


def test_updater_level_rejects_unknown_slam_landmark(euroc_yaml):
    import uvio_amd as U
    from uvio_amd.sim import SimStream
    opts = U.load_options(euroc_yaml, max_msckf_in_update=60, max_slam_features=0)
    sim = SimStream(opts, duration=8 / opts.track_frequency + 1.2, seed=3, spawn=30)
    g = U.VioManager(opts)
    sim.run(g, n_frames=6)
    t = float(g.get_clone_times()[-1])
    with pytest.raises(RuntimeError, match="E_ARG"):
        g.slam_update([(987654321, [(0, t, 100.0, 100.0, 0.1, 0.1)])])
    with pytest.raises(RuntimeError, match="E_ARG"):
        g.msckf_update([(1, [(7, t, 100.0, 100.0, 0.1, 0.1)])])  # camera id out of range
    g.close()


def test_uwb_update_single_matches_oracle(euroc_yaml):
    """UpdaterUWB::update_single (UpdaterUWB.cpp:53-90) through the C ABI on a state snapshot, fixed and
    estimated anchors, one range consistent with the ground truth and one 20 m off (chi2-gated on both)."""
    import uvio_amd as U
    from uvio_amd import _native as N
    from oracle import oracle as O
    from uvio_amd.sim import SimStream
    from test_gpu_parity import make_anchors
    opts = U.load_options(euroc_yaml, max_msckf_in_update=60, max_slam_features=0, use_uwb=1,
                          do_calib_uwb_extrinsics=1, min_dist_to_use_uwb=0.05)
    for k, v in enumerate([0.05, -0.02, 0.03]):
        opts.p_IinU[k] = v
    anchors = make_anchors(N)
    n = 10
    sim = SimStream(opts, duration=(n + 2) / opts.track_frequency + 1.2, seed=4, spawn=40, anchors=anchors,
                    uwb_rate=10.0, uwb_sigma=0.1)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    sim.run([g, o], n_frames=n, before_frame=lambda nf, t: _sync(g, o),
            after_init=lambda m: m.try_to_initialize_uwb_anchors(anchors))
    t, _ = g.get_imu_state()
    p_U = sim.traj.R_ItoG(t) @ (-np.array(opts.p_IinU[:])) + sim.traj.pos(t)
    applied, gated = 0, 0
    for a in anchors:
        true = (1 + a.dist_bias) * np.linalg.norm(np.array(a.p_AinG[:]) - p_U) + a.const_bias
        for rng in (true + 0.05, true + 20.0):
            _sync(g, o)
            ag = g.uwb_update_single(t, a.id, rng)
            ao = o.uwb_update_single(t, a.id, rng)
            assert ag == ao
            applied += ag
            gated += not ag
            _same_state(g, o)
    assert applied >= 3 and gated >= 3
    g.close()


def test_fatal_error_stops_the_handle(euroc_yaml):
    """A negative covariance diagonal after an update is fatal in the reference (StateHelper.cpp:171-182,
    std::exit): the call returns UVIO_HP_E_NUMERIC and every later state-changing call UVIO_HP_E_STATE naming it,
    while the getters still read the state."""
    import uvio_amd as U
    from uvio_amd import _native as N
    from uvio_amd.sim import SimStream
    from test_gpu_parity import make_anchors
    opts = U.load_options(euroc_yaml, max_msckf_in_update=60, max_slam_features=0, use_uwb=1,
                          do_calib_uwb_extrinsics=1, min_dist_to_use_uwb=0.05)
    anchors = make_anchors(N)
    n = 8
    sim = SimStream(opts, duration=(n + 2) / opts.track_frequency + 1.2, seed=4, spawn=40, anchors=anchors,
                    uwb_rate=10.0, uwb_sigma=0.1)
    g = U.VioManager(opts)
    sim.run(g, n_frames=n, after_init=lambda m: m.try_to_initialize_uwb_anchors(anchors))
    x, _ = g.get_state_vector()
    P = g.get_cov()
    P[-1, -1] = -1.0  # the last variable (outside the range's columns) gets a negative variance
    g.set_state(x, g.get_fej_vector(), P)
    t, _ = g.get_imu_state()
    a = anchors[-1]
    p_U = sim.traj.R_ItoG(t) @ (-np.array(opts.p_IinU[:])) + sim.traj.pos(t)
    rng = (1 + a.dist_bias) * np.linalg.norm(np.array(a.p_AinG[:]) - p_U) + a.const_bias
    with pytest.raises(RuntimeError, match="E_NUMERIC"):
        g.uwb_update_single(t, a.id, rng)
    with pytest.raises(RuntimeError, match="E_STATE.*stopped"):
        g.uwb_update_single(t, a.id, rng)
    with pytest.raises(RuntimeError, match="E_STATE"):
        g.propagate_and_clone(t + 0.05)
    assert g.get_cov().shape == P.shape and np.all(np.isfinite(g.get_state_vector()[0]))
    g.close()
