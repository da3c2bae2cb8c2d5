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
    assert np.all(per_cam > n * 40), per_cam  # every camera keeps tracks
    assert bad == 0, (bad, total)


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
