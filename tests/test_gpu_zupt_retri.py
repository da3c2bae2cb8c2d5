"""GPU parity of the two per-frame steps added around the update: the zero-velocity update and the
re-triangulation of the active tracks, in lock-step with the oracle (tolerances as test_gpu_parity.py).

  * UpdaterZeroVelocity::try_update (UpdaterZeroVelocity.cpp:65-329, called from UVioManager.cpp:147-162):
    a stream that rests for its first second; the IMU-chi2 / velocity test and the disparity test decide
    identically on both sides frame by frame, and the accepted frames apply the same bias propagation and
    EKF update (a ZUPT frame returns before cloning).
  * VioManager::retriangulate_active_tracks (VioManagerHelper.cpp:190-388, inside the timed "re-tri & marg"
    bucket): the active tracks' positions (running linear triangulation per track, SLAM landmarks from the
    state) and their (u, v, depth) in camera 0 equal the oracle's after every frame: same track sets, values
    within 1e-9 relative.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import _check_lockstep, _rel, run_lockstep

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")


def _lockstep(opts, sim, n, renderer=None, after_init=None):
    def extra(g, o, a, b):
        a["active"], b["active"] = g.get_active_tracks(), o.get_active_tracks()
    return run_lockstep(opts, sim, n, renderer=renderer, after_init=after_init, extra=extra)


def _check_active(steps, min_tracks=20):
    seen = 0
    for k, (a, b) in enumerate(steps):
        ta, Pa, Da = a["active"]
        tb, Pb, Db = b["active"]
        assert ta == tb, k
        assert set(Pa) == set(Pb), (k, len(Pa), len(Pb), sorted(set(Pa) ^ set(Pb))[:10])
        assert set(Da) == set(Db), (k, sorted(set(Da) ^ set(Db))[:10])
        for fid in Pa:
            assert _rel(Pa[fid], Pb[fid]) < 1e-9, (k, fid, Pa[fid], Pb[fid])
        for fid in Da:
            assert _rel(Da[fid], Db[fid]) < 1e-9, (k, fid, Da[fid], Db[fid])
        seen = max(seen, len(Da))
    assert seen >= min_tracks, seen


def test_zupt_static_start_lockstep():
    import uvio_amd as U
    from uvio_amd.sim import SimStream
    opts = U.load_options(EUROC, try_zupt=1, zupt_only_at_beginning=1, zupt_chi2_multipler=1.0,
                          zupt_max_velocity=0.1, zupt_noise_multiplier=10.0, zupt_max_disparity=0.5,
                          max_msckf_in_update=100, max_slam_features=10, max_slam_in_update=5, dt_slam_delay=0.5)
    n = 45
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=60, frac_long=0.3, sigma_pix=0.3,
                    static_for=1.0)
    steps = _lockstep(opts, sim, n)
    zg = [a["timing"]["zupt"] for a, _ in steps]
    zo = [b["timing"]["zupt"] for _, b in steps]
    assert zg == zo
    assert sum(zg) >= 10, zg                      # the resting second is absorbed by zero-velocity updates
    assert sum(zg[-15:]) == 0                     # zupt_only_at_beginning: none once the platform moved
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 50
    _check_lockstep(steps)
    _check_active(steps)


def test_zupt_iros_config_disparity_images():
    """The shipped config/iros_2023_uvio ZUPT settings (disparity-only test: zupt_chi2_multipler 0, max
    disparity 1.5 px, only at the beginning) on downsampled mono images of a platform that rests first."""
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(os.path.join(ROOT, "configs", "iros_2023_uvio", "estimator_config.yaml"),
                          init_max_features=150, use_uwb=0)
    assert opts.try_zupt == 1 and opts.zupt_chi2_multipler == 0.0
    n = 30
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=4, static_for=1.0)
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"))
    zg = [a["timing"]["zupt"] for a, _ in steps]
    assert zg == [b["timing"]["zupt"] for _, b in steps]
    assert sum(zg) >= 4, zg
    assert sum(zg[-10:]) == 0
    _check_lockstep(steps)


def test_retriangulation_tracks_lockstep():
    import uvio_amd as U
    from uvio_amd.sim import SimStream
    opts = U.load_options(EUROC, max_msckf_in_update=100, max_slam_features=20, max_slam_in_update=10,
                          dt_slam_delay=0.3)
    n = 30
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=80, frac_long=0.3)
    steps = _lockstep(opts, sim, n)
    _check_lockstep(steps)
    _check_active(steps, min_tracks=100)


def test_retriangulation_images_lockstep():
    import sys
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    sys.path.insert(0, ROOT)
    import bench
    opts = bench.workload_options(U, "cfg2")
    n = 20
    sim = bench.make_stream(opts, n + 2, seed=5, workload="cfg2")
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"))
    _check_lockstep(steps)
    _check_active(steps, min_tracks=100)
