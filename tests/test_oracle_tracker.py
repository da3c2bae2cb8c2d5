"""Pins the oracle's restatement of the OpenCV primitives TrackKLT calls.

OpenCV is not in this image and the reference holds no tracker golden vectors, so the
restatement (oracle/src/tracker.cpp) is checked two independent ways:
  * against a second, vectorized numpy restatement written from the published definitions
    (bit-exact for the integer / byte primitives: equalizeHist, pyrDown, Scharr, FAST-9 score + NMS);
  * against known answers no implementation detail can change: constant and linear-ramp images
    through pyrDown / Scharr, corners of rendered rectangles for FAST, a rendered saddle point for
    cornerSubPix, rendered sub-pixel translations at every pyramid level for LK, exact epipolar
    geometry for the 7-point solver and injected outliers for RANSAC.
The device kernels are bit-exact against this restatement (tests/test_gpu_track.py).
"""
import numpy as np
import pytest

from oracle import oracle as O


def _rand_img(rng, h, w, kind="uniform"):
    if kind == "uniform":
        return rng.integers(0, 256, (h, w), dtype=np.uint8)
    if kind == "narrow":  # occupied bins with gaps, like a dim camera image
        return (rng.integers(0, 40, (h, w)) * 3 + 17).astype(np.uint8)
    if kind == "skewed":
        return np.clip(rng.exponential(30.0, (h, w)), 0, 255).astype(np.uint8)
    raise ValueError(kind)


# ------------------------------------------------------------------------------------------------
# equalizeHist (TrackKLT.cpp:59): LUT[i0] = 0, LUT[i] = sat_u8(round(cumsum(hist[i0+1..i]) * 255/(N-hist[i0])))
def _np_equalize(img):
    hist = np.bincount(img.ravel(), minlength=256)
    i0 = int(np.nonzero(hist)[0][0])
    total = img.size
    if hist[i0] == total:
        return np.full_like(img, i0)
    scale = np.float32(255.0) / np.float32(total - hist[i0])
    lut = np.zeros(256, dtype=np.int64)
    cs = np.cumsum(hist[i0 + 1:])
    lut[i0 + 1:] = np.clip(np.rint(cs.astype(np.float32) * scale), 0, 255)
    return lut[img].astype(np.uint8)


@pytest.mark.parametrize("kind", ["uniform", "narrow", "skewed"])
def test_equalize_hist_matches_definition(kind):
    rng = np.random.default_rng(1)
    for h, w in [(48, 64), (480, 752), (37, 53)]:
        img = _rand_img(rng, h, w, kind)
        out = O.equalize_hist(img)
        assert np.array_equal(out, _np_equalize(img))
        # the LUT is monotone, maps the lowest occupied level to 0 and the highest to 255
        order = np.argsort(img.ravel(), kind="stable")
        assert np.all(np.diff(out.ravel()[order].astype(int)) >= 0)
        assert out[img == img.min()].max() == 0 and out[img == img.max()].min() == 255


def test_equalize_hist_constant_image_is_unchanged():
    img = np.full((30, 40), 77, dtype=np.uint8)
    assert np.array_equal(O.equalize_hist(img), img)


# ------------------------------------------------------------------------------------------------
# pyrDown (BORDER_REFLECT_101 = numpy 'reflect'), [1 4 6 4 1]^2, (sum + 128) >> 8
def _np_pyr_down(img):
    k = np.array([1, 4, 6, 4, 1], dtype=np.int64)
    p = np.pad(img.astype(np.int64), 2, mode="reflect")
    h, w = img.shape
    rows = sum(k[i] * p[i:i + h, :] for i in range(5))
    full = sum(k[j] * rows[:, j:j + w] for j in range(5))
    return ((full[::2, ::2] + 128) >> 8).astype(np.uint8)


@pytest.mark.parametrize("shape", [(480, 752), (512, 512), (33, 47), (8, 9)])
def test_pyr_down_matches_definition(shape):
    img = _rand_img(np.random.default_rng(shape[0]), *shape)
    out = O.pyr_down(img)
    assert out.shape == ((shape[0] + 1) // 2, (shape[1] + 1) // 2)
    assert np.array_equal(out, _np_pyr_down(img))


def test_pyr_down_constant_and_ramp():
    assert np.all(O.pyr_down(np.full((41, 60), 200, np.uint8)) == 200)
    y, x = np.mgrid[0:60, 0:80]
    ramp = (x + 2 * y + 3).astype(np.uint8)  # max 80 + 118 + 3 < 256
    out = O.pyr_down(ramp)
    yy, xx = np.mgrid[0:out.shape[0], 0:out.shape[1]]
    inner = (slice(1, -1), slice(1, -1))  # reflect-101 bends the ramp at the border only
    assert np.array_equal(out[inner], (2 * xx + 4 * yy + 3)[inner].astype(np.uint8))


def test_pyramid_truncation_rule():
    # buildOpticalFlowPyramid(win 15, maxLevel 5) stops once the next level's side would be <= win
    # (SURVEY Appendix A): 752x480 -> levels 0-4, 512x512 -> 0-5, 640x480 -> 0-4
    assert O.pyramid_levels(752, 480) == 5
    assert O.pyramid_levels(512, 512) == 6
    assert O.pyramid_levels(640, 480) == 5
    assert O.pyramid_levels(376, 240) == 4  # downsample_cameras (VioManager.cpp:274) halves the input


# ------------------------------------------------------------------------------------------------
# Scharr: dx = [3 10 3]^T (x) [-1 0 1], dy its transpose, BORDER_REFLECT_101, unnormalized int16
def _np_scharr(img):
    p = np.pad(img.astype(np.int64), 1, mode="reflect")
    h, w = img.shape
    s = lambda dy, dx: p[1 + dy:1 + dy + h, 1 + dx:1 + dx + w]  # noqa: E731
    dx = 3 * (s(-1, 1) - s(-1, -1)) + 10 * (s(0, 1) - s(0, -1)) + 3 * (s(1, 1) - s(1, -1))
    dy = 3 * (s(1, -1) - s(-1, -1)) + 10 * (s(1, 0) - s(-1, 0)) + 3 * (s(1, 1) - s(-1, 1))
    return np.stack([dx, dy], axis=-1).astype(np.int16)


@pytest.mark.parametrize("shape", [(480, 752), (31, 45)])
def test_scharr_matches_definition(shape):
    img = _rand_img(np.random.default_rng(7), *shape)
    assert np.array_equal(O.scharr(img), _np_scharr(img))


def test_scharr_of_linear_ramp_is_the_exact_gradient():
    y, x = np.mgrid[0:40, 0:50]
    for a, b in [(1, 2), (3, 0), (0, 4), (2, 1)]:
        ramp = (a * x + b * y + 5).astype(np.uint8)
        d = O.scharr(ramp)[1:-1, 1:-1]
        assert np.all(d[..., 0] == 32 * a) and np.all(d[..., 1] == 32 * b)


# ------------------------------------------------------------------------------------------------
# FAST-9/16 with non-maximum suppression (Grider_GRID.h:125):
#   corner iff some arc of 9 contiguous circle pixels is all darker than v - thr or all brighter than
#   v + thr; score = the largest threshold at which it is still a corner; NMS keeps strict maxima.
CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def _np_fast(img, thr):
    img = img.astype(np.int64)
    h, w = img.shape
    c = img[3:h - 3, 3:w - 3]
    d = np.stack([c - img[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE])  # (16, h-6, w-6)
    dd = np.concatenate([d, d[:8]])
    arcs_dark = np.stack([dd[k:k + 9].min(axis=0) for k in range(16)]).max(axis=0)
    arcs_bright = np.stack([(-dd[k:k + 9]).min(axis=0) for k in range(16)]).max(axis=0)
    score = np.maximum(arcs_dark, arcs_bright) - 1
    sc = np.zeros((h, w), dtype=np.int64)
    sc[3:h - 3, 3:w - 3] = np.where(score >= thr, score, 0)
    kps = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = sc[y, x]
            if s == 0:
                continue
            nb = sc[y - 1:y + 2, x - 1:x + 2].copy()
            nb[1, 1] = -1
            if s > nb.max():
                kps.append((x, y, s))
    return np.array(kps, dtype=np.float32).reshape(-1, 3)


@pytest.mark.parametrize("thr", [10, 20, 40])
def test_fast_matches_definition(thr):
    rng = np.random.default_rng(thr)
    # blocky texture: corners, edges and flat areas at several contrasts
    img = np.kron(rng.integers(0, 256, (12, 16)), np.ones((5, 5), dtype=np.int64)).astype(np.uint8)
    img = np.clip(img.astype(int) + rng.integers(-6, 7, img.shape), 0, 255).astype(np.uint8)
    kp = O.fast(img, thr)
    ref = _np_fast(img, thr)
    assert len(kp) > 20
    assert np.array_equal(kp, ref)


def test_fast_roi_coordinates_and_border():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (60, 80), dtype=np.uint8)
    x0, y0, rw, rh = 17, 9, 30, 25
    kp = O.fast(img, 20, roi=(x0, y0, rw, rh))
    ref = _np_fast(img[y0:y0 + rh, x0:x0 + rw].copy(), 20)
    assert np.array_equal(kp, ref)  # ROI coordinates, pixels closer than 3 px to the ROI edge untested
    assert kp.size == 0 or (kp[:, 0].min() >= 3 and kp[:, 1].min() >= 3 and kp[:, 0].max() < rw - 3)


def test_fast_finds_rectangle_corners_only():
    img = np.full((80, 100), 60, dtype=np.uint8)
    rects = [(20, 15, 30, 25), (60, 40, 25, 30)]  # x, y, w, h
    corners = set()
    for x, y, w, h in rects:
        img[y:y + h, x:x + w] = 170
        corners |= {(x, y), (x + w - 1, y), (x, y + h - 1), (x + w - 1, y + h - 1)}
    # a binary rectangle's corner pixel and its edge neighbours tie (11 vs 10 dark circle pixels, same
    # contrast): a plateau, which strict NMS rejects entirely
    assert len(O.fast(img, 30)) == 0
    for x, y in corners:
        img[y, x] = 210  # a strict maximum at each corner
    kp = O.fast(img, 30)
    found = {(int(a), int(b)) for a, b, _ in kp}
    assert found == corners, (sorted(found), sorted(corners))
    assert np.all(kp[:, 2] == 210 - 60 - 1)  # score: the largest threshold that still passes (strict test)


def test_fast_nms_is_strict_on_plateaus():
    # two adjacent pixels with the same score: neither is a strict local maximum
    img = np.full((30, 30), 50, dtype=np.uint8)
    img[15, 14:16] = 220
    kp = O.fast(img, 20)
    assert not any(14 <= x <= 15 and y == 15 for x, y, _ in kp)


# ------------------------------------------------------------------------------------------------
# cornerSubPix(win 5, zero zone none, 20 iterations, eps 1e-3) converges to a rendered saddle point
@pytest.mark.parametrize("x0,y0", [(30.3, 25.7), (41.55, 33.2), (27.0, 31.9)])
def test_corner_subpix_converges_to_saddle(x0, y0):
    y, x = np.mgrid[0:60, 0:70].astype(np.float64)
    img = np.clip(np.rint(128 + 100 * np.tanh((x - x0) / 1.2) * np.tanh((y - y0) / 1.2)), 0, 255).astype(np.uint8)
    start = np.array([[np.round(x0) + 1.0, np.round(y0) - 1.0], [np.round(x0) - 1.0, np.round(y0) + 2.0]])
    out = O.corner_subpix(img, start)
    assert np.abs(out - np.array([x0, y0])).max() < 0.05, out


def test_corner_subpix_reverts_far_drift():
    # a flat region next to an edge: the estimate may not leave the 5 px half-window
    img = np.zeros((50, 50), np.uint8)
    img[:, 30:] = 255
    out = O.corner_subpix(img, [[15.0, 25.0]])
    assert np.abs(out[0] - [15.0, 25.0]).max() <= 5.0 + 1e-6


# ------------------------------------------------------------------------------------------------
# pyramidal LK recovers rendered sub-pixel translations at every pyramid depth
def _texture(h, w, tx=0.0, ty=0.0, seed=4):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    x, y = x - tx, y - ty
    f = np.zeros((h, w))
    for _ in range(14):
        lam = rng.uniform(10, 70)
        th = rng.uniform(0, np.pi)
        ph = rng.uniform(0, 2 * np.pi)
        f += rng.uniform(0.5, 1.0) * np.sin(2 * np.pi * (x * np.cos(th) + y * np.sin(th)) / lam + ph)
    f = 128 + 110 * f / np.abs(f).max()
    return np.clip(np.rint(f), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("max_level,t", [(0, (1.3, -0.6)), (1, (2.7, 1.9)), (2, (-5.2, 3.6)), (3, (9.4, -6.3)),
                                         (4, (15.2, 11.7))])
def test_lk_recovers_translation(max_level, t):
    h, w = 240, 320
    prev = _texture(h, w)
    nxt = _texture(h, w, *t)
    gy, gx = np.mgrid[70:171:25, 90:231:35]
    p0 = np.stack([gx.ravel(), gy.ravel()], 1).astype(np.float32) + 0.37
    p1, st = O.lk(prev, nxt, p0, max_level=max_level)
    assert st.all()
    err = np.abs(p1 - (p0 + np.array(t, dtype=np.float32)))
    assert np.median(err) < 0.03 and err.max() < 0.15, (err.max(), np.median(err))


def test_lk_rejects_points_leaving_the_image():
    prev = _texture(120, 160)
    nxt = _texture(120, 160, 2.0, 0.0)
    p0 = np.array([[80.0, 60.0], [-20.0, 60.0]], dtype=np.float32)
    _, st = O.lk(prev, nxt, p0, max_level=2)
    assert st[0] == 1 and st[1] == 0


# ------------------------------------------------------------------------------------------------
# 7-point solver and FM_RANSAC on normalized coordinates (TrackKLT.cpp:863-877)
def _two_views(rng, n):
    P = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(4, 8, n)], 1)
    ang = rng.uniform(-0.1, 0.1, 3)
    K = np.array([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]])
    R = np.eye(3) + np.sin(np.linalg.norm(ang)) / np.linalg.norm(ang) * K + \
        (1 - np.cos(np.linalg.norm(ang))) / np.linalg.norm(ang) ** 2 * K @ K
    t = rng.uniform(0.4, 0.8, 3) * rng.choice([-1, 1], 3)
    Q = P @ R.T + t
    x0 = P[:, :2] / P[:, 2:]
    x1 = Q[:, :2] / Q[:, 2:]
    E = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]]) @ R
    return x0, x1, E


def test_fundamental_7pt_exact_geometry():
    rng = np.random.default_rng(11)
    for _ in range(5):
        x0, x1, E = _two_views(rng, 7)
        Fs = O.fundamental_7pt(x0, x1)
        assert 1 <= len(Fs) <= 3
        h0 = np.hstack([x0, np.ones((7, 1))])
        h1 = np.hstack([x1, np.ones((7, 1))])
        En = E / np.linalg.norm(E)
        best = np.inf
        for F in Fs:
            assert np.abs(np.einsum("ij,jk,ik->i", h1, F, h0)).max() < 1e-9 * np.abs(F).max()
            assert abs(np.linalg.det(F)) < 1e-9 * np.abs(F).max() ** 3
            Fn = F / np.linalg.norm(F)
            best = min(best, np.abs(Fn - En).max(), np.abs(Fn + En).max())
        assert best < 1e-6  # the true essential matrix is one of the pencil's singular members


def test_ransac_rejects_injected_outliers():
    rng = np.random.default_rng(5)
    n, n_out = 150, 30
    f = 460.0
    x0, x1, E = _two_views(rng, n)
    x0 = x0 + rng.normal(0, 0.3 / f, x0.shape)
    x1 = x1 + rng.normal(0, 0.3 / f, x1.shape)
    moved = rng.choice(n, n_out, replace=False)
    x1[moved] += rng.uniform(20, 60, (n_out, 2)) / f * rng.choice([-1, 1], (n_out, 2))
    # the error RANSAC thresholds, under the TRUE geometry: max of the squared point-to-epipolar-line
    # distances in both images (a point moved along its epipolar line stays an inlier)
    h0 = np.hstack([x0, np.ones((n, 1))])
    h1 = np.hstack([x1, np.ones((n, 1))])
    l1, l0 = h0 @ E.T, h1 @ E
    r = np.einsum("ij,ij->i", h1, l1)
    err = np.maximum(r ** 2 / (l1[:, 0] ** 2 + l1[:, 1] ** 2), r ** 2 / (l0[:, 0] ** 2 + l0[:, 1] ** 2))
    thr = 2.0 / f
    bad = err > (8 * thr) ** 2
    assert bad.sum() >= n_out // 2
    m = O.ransac_mask(x0, x1, thr)
    assert m[bad].sum() == 0
    assert m[err < (0.5 * thr) ** 2].mean() > 0.8  # mask of the best minimal-sample (7-point) model


def test_ransac_needs_seven_points():
    rng = np.random.default_rng(6)
    x0, x1, _ = _two_views(rng, 6)
    assert O.ransac_mask(x0, x1, 0.01).sum() == 0


def test_oracle_tracker_threads_give_identical_tracks(euroc_yaml):
    """The CPU baseline runs the restated OpenCV calls (LK per point, pyrDown / Scharr per row) on
    num_opencv_threads = 4 threads, as the reference's configs do (config/euroc_mav/estimator_config.yaml:89):
    every work item is independent, so the tracks must not depend on the thread count."""
    import uvio_amd as U
    from oracle import oracle as O
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(euroc_yaml, init_max_features=200)
    n = 6
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=4)
    r = SceneRenderer(opts, device="cpu")
    frames = [[r.render(k, *sim.camera_pose(i, k), frame_seed=i).numpy() for k in range(2)] for i in range(n)]
    runs = []
    for threads in (1, 4):
        assert O.set_threads(threads) == threads
        o = O.OracleManager(opts)
        tr = []
        for i in range(n):
            o.feed_measurement_camera(sim.cam_t[i], [0, 1], frames[i], allow_uninit=True)
            tr.append([o.get_tracks(c) for c in (0, 1)])
        runs.append(tr)
    O.set_threads(1)
    total = 0
    for a, b in zip(*runs):
        for (ia, ua), (ib, ub) in zip(a, b):
            assert np.array_equal(ia, ib) and np.array_equal(ua, ub)
            total += len(ia)
    assert total > 200
