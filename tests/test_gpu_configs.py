"""GPU parity on the BASELINE.json configs 3-5: the HIP path against the oracle in
lock-step (tolerances and the rounding-tie steering as in test_gpu_parity.py) on streams shaped like

  cfg3  configs/tum_vi            stereo equidistant (fisheye) 512x512, T_cam_imu calibration
  cfg4  configs/uzhfpv_outdoor_45 stereo equidistant 640x480, extrinsics not calibrated, sigma_px 1.5
  cfg5  configs/rpng_sim_uwb      4 cameras (binocular: every feature in one camera), IMU intrinsics and
                                  g-sensitivity calibrated (Phi 39x39), 6 UWB anchors (2 fixed) from the
                                  config with ranges at 10 Hz

Clone counts and feature counts are the configs' own (the bench raises them to the BASELINE sizes), so
each run finishes in seconds on the oracle.  The image path of cfg3 (fisheye pyramids / tracks) is
checked bit-exact against the oracle tracker.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import _check_lockstep, _rel, _snap, run_lockstep

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(name):
    return os.path.join(ROOT, "configs", name, "estimator_config.yaml")


def _lockstep(opts, n_frames, anchors=False, **simkw):
    from uvio_amd.sim import SimStream
    anc = [opts.anchors[i] for i in range(opts.n_anchors)] if anchors else None
    s = SimStream(opts, duration=n_frames / opts.track_frequency + 1.2, seed=5, anchors=anc, **simkw)
    return run_lockstep(opts, s, n_frames)


def test_lockstep_cfg3_tum_vi_fisheye():
    import uvio_amd as U
    opts = U.load_options(_cfg("tum_vi"), max_msckf_in_update=150, max_slam_features=10, max_slam_in_update=5,
                          dt_slam_delay=0.3)
    steps = _lockstep(opts, 30, spawn=80, frac_long=0.2)
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 200
    assert sum(a["timing"]["n_slam"] for a, _ in steps) > 0
    _check_lockstep(steps)


def test_lockstep_cfg4_uzhfpv_no_extrinsics():
    import uvio_amd as U
    opts = U.load_options(_cfg("uzhfpv_outdoor_45"), max_msckf_in_update=150, max_slam_features=10,
                          max_slam_in_update=5, dt_slam_delay=0.3)
    steps = _lockstep(opts, 30, spawn=80, frac_long=0.2)
    # no extrinsic blocks: 15 IMU + 1 dt + 2 x 8 intrinsics before the clones
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 200
    _check_lockstep(steps)


def test_lockstep_cfg5_four_cameras_uwb_imu_intrinsics():
    import uvio_amd as U
    opts = U.load_options(_cfg("rpng_sim_uwb"), max_msckf_in_update=150, max_slam_features=10,
                          max_slam_in_update=5, dt_slam_delay=0.3, min_dist_to_use_uwb=0.05)
    steps = _lockstep(opts, 30, anchors=True, spawn=120, frac_long=0.2)
    # IMU 15 + Dw 6 + Da 6 + Tg 9 + R_GYROtoIMU 3 + dt 1 + 4 x 14 camera blocks + 4 x 5 unfixed anchors
    assert steps[0][0]["P"].shape[0] >= 15 + 24 + 1 + 56 + 20
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 50
    _check_lockstep(steps)


def test_lockstep_images_cfg5_four_cameras():
    """The full image path on the 4-camera rig (each camera tracked on its own, batched on the device) with
    UWB ranges and IMU intrinsics: track -> propagate -> MSCKF / SLAM / delayed init / UWB, lock-step."""
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(_cfg("rpng_sim_uwb"), init_max_features=600, max_msckf_in_update=150, max_slam_features=20,
                          max_slam_in_update=10, dt_slam_delay=0.5, min_dist_to_use_uwb=0.05)
    anc = [opts.anchors[i] for i in range(opts.n_anchors)]
    n = 24
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, anchors=anc, spawn=4)
    steps = run_lockstep(opts, s, n, renderer=SceneRenderer(opts, device="cuda"))
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 100
    assert sum(a["timing"]["n_slam_delayed"] for a, _ in steps) > 0
    _check_lockstep(steps)


def test_cfg5_long_run_matches_oracle_counts():
    """cfg5 shape past the clone-window fill (max_clones 30) with SLAM promotion and UWB: both run on their
    own; the update sets must agree frame by frame while the states stay close."""
    import uvio_amd as U
    from oracle import oracle as O
    from uvio_amd.sim import SimStream
    opts = U.load_options(_cfg("rpng_sim_uwb"), max_clone_size=30, max_msckf_in_update=200, dt_slam_delay=1.0)
    anc = [opts.anchors[i] for i in range(opts.n_anchors)]
    n = 70
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, anchors=anc, spawn=100, frac_lost=0.0,
                  frac_long=0.02)
    out = {"g": [], "o": []}
    g, o = U.VioManager(opts), O.OracleManager(opts)
    s.run(g, n_frames=n, on_frame=lambda nf, t: out["g"].append(_snap(g)))
    s.run(o, n_frames=n, on_frame=lambda nf, t: out["o"].append(_snap(o)))
    g.close()
    assert len(out["g"]) == len(out["o"]) == n
    for a, b in zip(out["g"], out["o"]):
        assert a["timing"]["n_msckf"] == b["timing"]["n_msckf"]
        assert a["x"].shape == b["x"].shape
    assert sum(a["timing"]["n_slam"] for a in out["g"]) > 0
    assert _rel(out["g"][-1]["x"], out["o"][-1]["x"]) < 1e-4


def test_upload_staging_recycling_is_invisible():
    """Large MSCKF batches write their tables straight into the upload staging ring; with a ring that
    recycles every few batches (UVIO_HP_STAGE_BYTES) the run must be bit-identical to the default one."""
    import uvio_amd as U
    from uvio_amd.sim import SimStream
    opts = U.load_options(_cfg("uzhfpv_outdoor_45"), max_msckf_in_update=400, max_slam_features=10,
                          max_slam_in_update=5, dt_slam_delay=0.3)
    n = 40
    runs = []
    for cap in (None, 1 << 20):
        if cap:
            os.environ["UVIO_HP_STAGE_BYTES"] = str(cap)
        try:
            s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=400, frac_long=0.2)
            g = U.VioManager(opts)
        finally:
            os.environ.pop("UVIO_HP_STAGE_BYTES", None)
        snaps = []
        s.run(g, n_frames=n, on_frame=lambda nf, t: snaps.append(_snap(g)))
        g.close()
        runs.append(snaps)
    assert max(a["timing"]["n_msckf"] for a in runs[0]) >= 256  # the direct-staging path ran
    # the small ring restarted, also between the update chain's blob and its first launch, whose copy of the blob
    # out of the previous epoch must precede the new epoch's upload (engine_chain.cpp, stage_flush(on_main))
    assert sum(a["timing"]["stage_restarts"] for a in runs[1]) > 0
    assert sum(a["timing"]["chain_blob_old_epoch"] for a in runs[1]) > 0
    assert sum(a["timing"]["stage_restarts"] for a in runs[1]) > sum(a["timing"]["stage_restarts"] for a in runs[0])
    for a, b in zip(*runs):
        assert np.array_equal(a["x"], b["x"]) and np.array_equal(a["P"], b["P"])


def test_tracks_bit_exact_cfg3_fisheye():
    """TrackKLT on rendered equidistant 512x512 stereo frames: ids and uv equal to the oracle tracker's after
    every frame, pyramids included (test_gpu_track.py does the same for the radtan EuRoC rig)."""
    import uvio_amd as U
    from oracle import oracle as O
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(_cfg("tum_vi"), init_max_features=400, max_msckf_in_update=100, max_slam_features=0)
    n = 15
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=4)
    r = SceneRenderer(opts, device="cuda")
    g, o = U.VioManager(opts), O.OracleManager(opts)
    checked = [0]

    def after(nf, t):
        for c in range(opts.num_cameras):
            ig, ug = g.get_tracks(c)
            io, uo = o.get_tracks(c)
            assert np.array_equal(ig, io), (nf, c)
            assert np.array_equal(ug, uo), (nf, c)
        for c in range(opts.num_cameras):
            for lvl in range(5):
                img_g, der_g = g.get_pyramid(c, lvl)
                img_o, der_o = o.get_pyramid(c, lvl)
                assert img_g.shape == img_o.shape and np.array_equal(img_g, img_o) and np.array_equal(der_g, der_o)
        checked[0] += 1

    s.run([g, o], n_frames=n, on_frame=after, renderer=r)
    ntr = sum(len(g.get_tracks(c)[0]) for c in range(2))
    g.close()
    assert checked[0] == n
    assert ntr > 300
