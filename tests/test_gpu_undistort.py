"""GPU parity of CamBase::undistort_f (ov_core/src/cam/CamBase.h:89; CamRadtan.h:99, CamEqui.h:108) through
uvio_hp_undistort, and of the tracker's database coordinates that come from the same device pass.

The device undistorts every point (LK's epilogue in the tracker); for the equidistant model the float
result can depend on the last bit of tan, which differs between the device's and the host's libm, so the
device flags the points whose double result lies within 2^-40 (relative) of a float rounding boundary and the
host recomputes those (hp_math.h cam_undistort_f).  The contract is bit-equality with the host restatement
(oracle/src/cam.h undistort_f) on every point, checked here on dense sub-pixel grids over each BASELINE
camera, past the image borders included.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cams(name):
    import uvio_amd as U
    opts = U.load_options(os.path.join(ROOT, "configs", name, "estimator_config.yaml"))
    return [opts.cams[c] for c in range(opts.num_cameras)]


def _differ(a, b):
    return (a.view(np.uint32) != b.view(np.uint32)) & ~(np.isnan(a) & np.isnan(b))


def _grid(cam, n_side, rng):
    w, h = cam.width, cam.height
    # 10 % past each border: LK can return points outside the image before the tracker drops them
    u = np.linspace(-0.1 * w, 1.1 * w, n_side, dtype=np.float64)
    v = np.linspace(-0.1 * h, 1.1 * h, n_side, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    uv = np.stack([uu.ravel(), vv.ravel()], 1) + rng.uniform(-0.5, 0.5, (n_side * n_side, 2))
    return uv.astype(np.float32)


@pytest.mark.parametrize("name", ["tum_vi", "uzhfpv_outdoor_45", "euroc_mav", "rpng_sim_uwb"])
def test_undistort_bit_exact(name):
    import uvio_amd as U
    from oracle import oracle as O
    rng = np.random.default_rng(7)
    total = flagged = 0
    for cam in _cams(name):
        uv = _grid(cam, 1000, rng)  # 1e6 points per camera
        got, amb = U.undistort(cam, uv, return_ambiguous=True)
        ref = O.camera_undistort(cam, uv)
        bad = np.flatnonzero(np.any(_differ(got, ref), axis=1))
        assert bad.size == 0, (name, int(cam.model), bad[:5], got[bad[:5]], ref[bad[:5]])
        if cam.model == 0:
            assert not amb.any()  # radtan: IEEE operations only, the same on both sides
        total += uv.shape[0]
        flagged += int(amb.sum())
    print("%s: %d points, %d recomputed on the host" % (name, total, flagged))
    assert flagged <= 1e-3 * total  # expected <= 2 x 2^-15 per point


def test_undistort_edge_cases():
    import uvio_amd as U
    from oracle import oracle as O
    cam = _cams("tum_vi")[0]
    cx, cy = cam.intrinsics[2], cam.intrinsics[3]
    uv = np.array([[cx, cy], [cx + 1e-6, cy], [np.nextafter(np.float32(cx), np.float32(1e9)), cy], [-1e4, 3e4],
                   [0.0, 0.0], [1e6, -1e6]], dtype=np.float32)
    got = U.undistort(cam, uv)
    ref = O.camera_undistort(cam, uv)
    assert not _differ(got, ref).any(), (got, ref)
    assert U.undistort(cam, np.zeros((0, 2), np.float32)).shape == (0, 2)
