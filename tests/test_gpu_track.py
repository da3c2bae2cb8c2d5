"""GPU parity of the KLT front-end (kernels_track.hip + engine_track.cpp) against the oracle's TrackKLT
restatement (oracle/src/tracker*.cpp), on ray-cast synthetic images (uvio_amd/render.py).

Tolerances: the front-end is integer / byte work (histogram, pyramid, Scharr, FAST, LK window sums)
plus float / double tails whose operation order the device reproduces (cornerSubPix runs one thread
per point with the oracle's summation order; LK's float update is uniform across the wave), so
  * pyramids (equalized image + Scharr derivatives, every level): bit-exact;
  * tracks after every frame (ids and float uv): bit-exact;
the one exception the tests allow for is RANSAC: the 7-point solver's cubic uses acos / cos / pow,
whose device and glibc results can differ by an ulp, which can flip a borderline inlier.  The test
counts such flips instead of failing on them (observed: none).
The estimator on top is then checked lock-step exactly as tests/test_gpu_parity.py does for the
simulated-track input.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _setup(euroc_yaml, n_frames, **over):
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(euroc_yaml, **over)
    s = SimStream(opts, duration=n_frames / opts.track_frequency + 1.2, seed=5, spawn=10)
    return opts, s, SceneRenderer(opts, device="cuda")


def _frames(s, r, cams, n):
    for i in range(n):
        yield i, s.cam_t[i], [r.render(k, *s.camera_pose(i, k), frame_seed=i).cpu().numpy() for k in cams]


def _compare_tracks(g, o, cams):
    """(#tracks, #mismatched) over cameras; ids must agree as sets up to RANSAC flips."""
    n = bad = 0
    for c in cams:
        ig, ug = g.get_tracks(c)
        io, uo = o.get_tracks(c)
        n += len(io)
        if len(ig) == len(io) and np.array_equal(ig, io) and np.array_equal(ug, uo):
            continue
        mg = {int(i): k for k, i in enumerate(ig)}
        mo = {int(i): k for k, i in enumerate(io)}
        common = set(mg) & set(mo)
        bad += len(set(mg) ^ set(mo))
        bad += sum(1 for i in common if not np.array_equal(ug[mg[i]], uo[mo[i]]))
    return n, bad


@pytest.mark.parametrize("hist", [1, 0])
def test_pyramid_bit_exact(euroc_yaml, hist):
    import uvio_amd as U
    from oracle import oracle as O
    opts, s, r = _setup(euroc_yaml, 4, histogram_method=hist)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    for i, t, imgs in _frames(s, r, [0, 1], 2):
        g.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        o.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        for c in (0, 1):
            for level in range(5):
                ig, dg = g.get_pyramid(c, level)
                io, do = o.get_pyramid(c, level)
                assert ig.shape == io.shape
                assert np.array_equal(ig, io), (c, level)
                assert np.array_equal(dg, do), (c, level)


@pytest.mark.parametrize("stereo", [True, False])
def test_tracks_bit_exact(euroc_yaml, stereo):
    """TrackKLT over 25 frames (detection, stereo LK, temporal LK + RANSAC): same ids, same uv."""
    import uvio_amd as U
    from oracle import oracle as O
    over = {} if stereo else {"use_stereo": 0}
    opts, s, r = _setup(euroc_yaml, 26, init_max_features=200, **over)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    total = bad = 0
    for i, t, imgs in _frames(s, r, [0, 1], 25):
        g.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        o.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        n, b = _compare_tracks(g, o, [0, 1])
        total += n
        bad += b
    cells, intro = g.grid_stats()
    print("FAST cells %d, on std::sort's introsort path (> 16 candidates) %d" % (cells, intro))
    assert total > 25 * 2 * 50  # the scene keeps the tracker busy
    assert bad == 0, (bad, total)


def test_tracks_bit_exact_four_cameras():
    """The 4-camera rpng_sim rig (configs/rpng_sim_uwb, use_stereo 0: each camera tracked on its own,
    TrackKLT.cpp:85-89) on rendered 752x480 frames, one camera masked: every camera's ids and uv equal
    the oracle's after every frame.  The device runs the cameras' detections and temporal matchings as
    one batch; the ids follow the cameras' order, as in the oracle's serial loop."""
    import uvio_amd as U
    from oracle import oracle as O
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "rpng_sim_uwb",
                       "estimator_config.yaml")
    opts = U.load_options(cfg, init_max_features=800)
    assert opts.num_cameras == 4 and not opts.use_stereo
    n = 16
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=10)
    r = SceneRenderer(opts, device="cuda")
    g, o = U.VioManager(opts), O.OracleManager(opts)
    cams = [0, 1, 2, 3]
    mask = np.zeros((opts.cams[2].height, opts.cams[2].width), dtype=np.uint8)
    mask[:120, :] = 255
    masks = [None, None, mask, None]
    total = bad = 0
    per_cam = np.zeros(4, dtype=int)
    for i, t, imgs in _frames(s, r, cams, n):
        g.feed_measurement_camera(t, cams, imgs, masks=masks, allow_uninit=True)
        o.feed_measurement_camera(t, cams, imgs, masks=masks, allow_uninit=True)
        nt, b = _compare_tracks(g, o, cams)
        total += nt
        bad += b
        for c in cams:
            per_cam[c] += len(o.get_tracks(c)[0])
    cells, intro = g.grid_stats()
    print("FAST cells %d, on std::sort's introsort path (> 16 candidates) %d" % (cells, intro))
    assert np.all(per_cam > n * 40), per_cam  # every camera keeps tracks
    assert bad == 0, (bad, total)


@pytest.mark.parametrize("stereo", [True, False])
def test_tracks_blank_frames(euroc_yaml, stereo):
    """Empty inputs to the front-end: uniform frames (no FAST corner, every LK window below the eigenvalue
    threshold) between textured ones, and one camera blank while the other is not.  Detection finds no corner on
    a blank frame, and LK into one keeps only what the previous image's gradients and RANSAC let through; the
    ids and uv equal the oracle's after every frame."""
    import uvio_amd as U
    from oracle import oracle as O
    over = {} if stereo else {"use_stereo": 0}
    opts, s, r = _setup(euroc_yaml, 12, init_max_features=200, **over)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    blank = np.full((opts.cams[0].height, opts.cams[0].width), 128, dtype=np.uint8)
    plan = ["tt", "tt", "tt", "bb", "bb", "tt", "tt", "bt", "tb", "tt", "tt"]
    total, counts = 0, []
    for (i, t, imgs), p in zip(_frames(s, r, [0, 1], len(plan)), plan):
        imgs = [blank if p[k] == "b" else imgs[k] for k in range(2)]
        g.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        o.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        n, b = _compare_tracks(g, o, [0, 1])
        assert b == 0, (i, p, b, n)
        total += n
        counts.append((p, n))
    print("tracks per frame", counts)
    assert total > 0


def test_tracks_mono_masked(euroc_yaml):
    """Monocular feed with a user mask (TrackKLT mask path: kept points, grid cells, griding)."""
    import uvio_amd as U
    from oracle import oracle as O
    opts, s, r = _setup(euroc_yaml, 12, num_cameras=1, use_stereo=0, init_max_features=150)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    mask = np.zeros((opts.cams[0].height, opts.cams[0].width), dtype=np.uint8)
    mask[:, :200] = 255
    mask[300:, 500:] = 255
    for i, t, imgs in _frames(s, r, [0], 10):
        g.feed_measurement_camera(t, [0], imgs, masks=[mask], allow_uninit=True)
        o.feed_measurement_camera(t, [0], imgs, masks=[mask], allow_uninit=True)
        n, b = _compare_tracks(g, o, [0])
        assert n > 20
        assert b == 0
        ig, ug = g.get_tracks(0)
        assert not np.any((ug[:, 0] < 200)), "masked region must stay empty"


def test_lockstep_images(euroc_yaml):
    """Full image path (track -> propagate -> MSCKF / SLAM update) lock-step against the oracle."""
    import test_gpu_parity as P
    import uvio_amd as U
    from oracle import oracle as O
    opts, s, r = _setup(euroc_yaml, 30, init_max_features=200, max_msckf_in_update=200, max_slam_features=25,
                        max_slam_in_update=25, dt_slam_delay=1.0)
    bad = [0]

    def extra(g, o, a, b):
        bad[0] += _compare_tracks(g, o, [0, 1])[1]

    steps = P.run_lockstep(opts, s, 30, renderer=r, extra=extra)
    assert bad[0] == 0
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 0
    assert sum(a["timing"]["n_slam_delayed"] for a, _ in steps) > 0
    P._check_lockstep(steps)


def _predetect_pair(opts, s, r, n, subset_frame=None, subset=None):
    """Two estimators on one stream, one with the next-frame detection run ahead on the worker thread and the
    detection stream (the default), one with it off (UVIO_HP_NO_PREDETECT=1): after every frame the states,
    covariances, track ids and points must be bit-identical.  Frame `subset_frame` feeds only the cameras
    `subset` (a camera set different from the last feed's: the run-ahead result is discarded)."""
    import uvio_amd as U
    old = os.environ.pop("UVIO_HP_NO_PREDETECT", None)
    try:
        a = U.VioManager(opts)
        os.environ["UVIO_HP_NO_PREDETECT"] = "1"
        b = U.VioManager(opts)
    finally:
        os.environ.pop("UVIO_HP_NO_PREDETECT", None)
        if old is not None:
            os.environ["UVIO_HP_NO_PREDETECT"] = old
    for m in (a, b):
        m.initialize_with_gt(s.gt_state(s.t0))
    nf = 0
    n_msckf = 0
    for kind, t, i in s.events():
        if t < s.t0 - 0.4:
            continue
        if kind == "imu":
            for m in (a, b):
                m.feed_measurement_imu(t, s.wm[i], s.am[i])
            continue
        if kind != "cam" or t <= s.t0:
            continue
        nf += 1
        cams = list(subset) if nf == subset_frame else list(range(s.K))
        imgs = [r.render(k, *s.camera_pose(i, k), frame_seed=i).cpu().numpy() for k in cams]
        for m in (a, b):
            m.feed_measurement_camera(t, cams, imgs)
        xa, xb = a.get_state_vector()[0], b.get_state_vector()[0]
        assert np.array_equal(xa, xb), ("state", nf)
        assert np.array_equal(a.get_cov(), b.get_cov()), ("covariance", nf)
        for c in range(s.K):
            ia, ua = a.get_tracks(c)
            ib, ub = b.get_tracks(c)
            assert np.array_equal(ia, ib) and np.array_equal(ua, ub), ("tracks", nf, c)
        n_msckf += a.get_timing()["n_msckf"]
        if nf >= n:
            break
    a.close()
    b.close()
    assert nf == n and n_msckf > 0


def test_predetect_on_off_bit_identical_cfg1_mono(euroc_yaml):
    """cfg1 (EuRoC mono, bench.py): the detection run ahead under the update chain changes nothing"""
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(euroc_yaml, num_cameras=1, use_stereo=0, init_max_features=200, max_msckf_in_update=100,
                          max_slam_features=20, max_slam_in_update=10, dt_slam_delay=0.3)
    n = 24
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=4)
    _predetect_pair(opts, s, SceneRenderer(opts, device="cuda"), n)


def test_predetect_on_off_bit_identical_four_cameras():
    """the 4-camera rig (each camera tracked on its own, feed_multi), with one frame of 3 cameras"""
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "rpng_sim_uwb",
                       "estimator_config.yaml")
    opts = U.load_options(cfg, init_max_features=800, max_msckf_in_update=200, max_slam_features=20,
                          max_slam_in_update=10, dt_slam_delay=0.3)
    n = 20
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=4)
    _predetect_pair(opts, s, SceneRenderer(opts, device="cuda"), n, subset_frame=12, subset=[0, 2, 3])


def test_second_device_image_frames(euroc_yaml):
    """A manager created for GPU 1 (the N > 1 bench ranks' form) feeds image frames -- its tracker's run-ahead
    detection binds that device on the worker thread -- and its estimate equals the GPU 0 manager's bit for bit.
    Needs two GPUs (skipped on a one-GPU box)."""
    import torch
    import uvio_amd as U
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU")
    opts, s, r = _setup(euroc_yaml, 16, init_max_features=200, max_msckf_in_update=100, max_slam_features=20,
                        max_slam_in_update=10, dt_slam_delay=0.3)
    out = []
    for dev in (0, 1):
        m = U.VioManager(opts, device=dev)
        s.run(m, n_frames=14, renderer=r)
        out.append((m.get_state_vector()[0], m.get_cov(), m.get_tracks(0)))
        m.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2][0], out[1][2][0]) and np.array_equal(out[0][2][1], out[1][2][1])
