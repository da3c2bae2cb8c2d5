"""GPU parity at the BASELINE.json sizes: the HIP path in lock-step with the oracle on the bench's own
workloads (bench.WORKLOADS), each run past the clone-window fill so that at least three
frames update with the full window:

  cfg1  EuRoC MH_01-shaped MONO images, 11 clones, <= 100 MSCKF + 50 SLAM
  cfg3  TUM-VI fisheye stereo images, 20 clones, 400 tracks / camera, <= 400 MSCKF
  cfg4i UZH-FPV stereo fisheye 640x480 images, 25 clones, 800 tracks (the bench line's TrackKLT stream)
  cfg4  UZH-FPV stereo fisheye tracks, 25 clones, 800 MSCKF features x 52 measurements
  cfg5i rpng_sim 4 cameras (752x480 images, each tracked on its own) + 6 UWB anchors, 30 clones
  cfg5  rpng_sim 4 cameras + 6 UWB anchors, IMU intrinsics + Tg, 30 clones, 1500 MSCKF features (tracks)
  iros  config/iros_2023_uvio as shipped (mono, downsample_cameras, ANCHORED_MSCKF_INVERSE_DEPTH MSCKF,
        GLOBAL_3D SLAM, 4 UWB anchors of which 2 fixed, initialized through try_to_initialize_uwb_anchors)

These put the large-batch device paths under the oracle: direct-to-staging batch tables and the parallel
chunk build (>= 256 features), k_gemm_HPg_tiled (m >= 4096 stacked rows), k_gram_mfma (m >= 8192) and the
information-form Cholesky factors of n > 135 columns.  Lock-step as in test_gpu_parity.py: before every
frame the oracle adopts the device's mean / FEJ values / covariance, both process the same frame.

Tolerances: the per-frame bounds of test_gpu_parity.py on EVERY frame (triangulation 1e-9 m, chi2 1e-11
relative, no accept / reject flip, state and covariance 1e-10 relative), with the oracle's rounding-tie
steering (test_gpu_parity.py docstring, oracle/src/flip.h): a feature on which the device and the oracle
disagree must be explained by ONE float cast within 1e-10 relative of its rounding midpoint, and with that
cast rounded the device's way the frame must meet the strict bounds.  The oracle compresses the ~80k stacked
rows of cfg4 / cfg5 with Givens rotations (UpdaterHelper.cpp:456-487) while the device forms their Gram in
information form.  Measured on MI355X (r02c): worst P 1.2e-12 (cfg4, 800 features x 52
measurements), 1.9e-13 (cfg5), 6.8e-13 (cfg3); worst state 2.2e-14.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import _check_lockstep, run_lockstep

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _lockstep(opts, sim, n_frames, renderer=None, after_init=None):
    return run_lockstep(opts, sim, n_frames, renderer=renderer, after_init=after_init)


def _stats(steps, max_clones):
    """per-frame summary; frames with the full window"""
    rows = []
    for k, (a, b) in enumerate(steps):
        rows.append((k, a["timing"]["n_clones"], a["timing"]["n_msckf"], a["timing"]["n_slam"],
                     a["timing"]["n_slam_delayed"]))
    full = [r for r in rows if r[1] >= max_clones + 1 and r[2] > 0]
    for r in rows:
        print("frame %3d clones %3d msckf %5d slam %3d delayed %3d" % r)
    return rows, full


def _check(steps, full, min_full=3):
    assert len(full) >= min_full, "only %d lock-step frames with the full clone window" % len(full)
    worst = _check_lockstep(steps)
    print("worst", worst)


def test_lockstep_cfg1_mono_images():
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    B = _bench()
    opts = B.workload_options(U, "cfg1")
    n = 24
    sim = B.make_stream(opts, n + 2, seed=5, workload="cfg1")
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"))
    rows, full = _stats(steps, opts.max_clone_size)
    assert steps[-1][0]["P"].shape[0] >= 15 + 1 + 14 + 6 * 11  # one camera's 14 calibration dims
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 0
    _check(steps, full)


def test_lockstep_cfg3_baseline_size():
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    B = _bench()
    opts = B.workload_options(U, "cfg3")
    n = 26
    sim = B.make_stream(opts, n + 2, seed=5, workload="cfg3")
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"))
    rows, full = _stats(steps, opts.max_clone_size)
    assert max(r[2] for r in rows) >= 100
    _check(steps, full)


def test_lockstep_cfg4_images_baseline_size():
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    B = _bench()
    opts = B.workload_options(U, "cfg4i")
    n = 30
    sim = B.make_stream(opts, n + 2, seed=5, workload="cfg4i")
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"))
    rows, full = _stats(steps, opts.max_clone_size)
    assert steps[-1][0]["P"].shape[0] >= 15 + 1 + 16 + 6 * 25  # 25 clones after the marginalization
    _check(steps, full)


def test_lockstep_cfg4_baseline_size():
    import uvio_amd as U
    B = _bench()
    opts = B.workload_options(U, "cfg4")
    n = 30
    sim = B.make_stream(opts, n + 2, seed=5, workload="cfg4")
    steps = _lockstep(opts, sim, n)
    rows, full = _stats(steps, opts.max_clone_size)
    assert max(r[2] for r in rows) == 800  # direct-to-staging tables, chunked build, tiled T GEMM, MFMA Gram
    assert max(a["timing"]["msckf_rows"] for a, _ in steps) >= 8192
    _check(steps, full)


def test_lockstep_cfg5_baseline_size():
    import uvio_amd as U
    B = _bench()
    opts = B.workload_options(U, "cfg5")
    n = 35
    sim = B.make_stream(opts, n + 2, seed=5, workload="cfg5")
    steps = _lockstep(opts, sim, n)
    rows, full = _stats(steps, opts.max_clone_size)
    assert max(r[2] for r in rows) == 1500
    assert steps[-1][0]["P"].shape[0] >= 15 + 24 + 1 + 56 + 6 * 31 + 20
    _check(steps, full)


def test_lockstep_cfg5_images_baseline_size():
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    B = _bench()
    opts = B.workload_options(U, "cfg5i")
    n = 34
    sim = B.make_stream(opts, n + 2, seed=5, workload="cfg5i")
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"))
    rows, full = _stats(steps, opts.max_clone_size)
    assert steps[-1][0]["P"].shape[0] >= 15 + 24 + 1 + 56 + 6 * 30 + 20
    _check(steps, full, min_full=2)


def _iros_anchors():
    """uwb_anchors.yaml of configs/iros_2023_uvio (the anchors the ROS topic would announce)"""
    import yaml
    from uvio_amd import _native as N
    with open(os.path.join(ROOT, "configs", "iros_2023_uvio", "uwb_anchors.yaml")) as f:
        doc = yaml.safe_load("".join(f.readlines()[1:]))
    out = []
    for k in sorted(doc):
        d = doc[k]
        a = N.Anchor()
        a.id, a.fix = int(d["id"]), 1 if d["fix"] else 0
        for i in range(3):
            a.p_AinG[i] = d["p_AinG"][i]
        a.const_bias, a.dist_bias = d["const_bias"], d["dist_bias"]
        for i, v in enumerate([d["prior_p_AinG_cov"]] * 3 + [d["prior_const_bias_cov"], d["prior_dist_bias_cov"]]):
            a.cov_diag[i] = v
        out.append(a)
    return out


def test_lockstep_iros_2023_uvio():
    """The config uvio ships (config/iros_2023_uvio): mono 752x480 downsampled to 376x240 on the device,
    MSCKF features as ANCHORED_MSCKF_INVERSE_DEPTH, UWB ranges to 4 anchors (2 fixed).  try_zupt is off here
    (UpdaterZeroVelocity is covered by its own test)."""
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    # the tracker keeps init_max_features tracks under initialize_with_gt (VioManager.cpp:131): 150 here so the
    # MSCKF update (not only the 40 SLAM slots) sees features
    opts = U.load_options(os.path.join(ROOT, "configs", "iros_2023_uvio", "estimator_config.yaml"), try_zupt=0,
                          min_dist_to_use_uwb=0.2, init_max_features=150)
    assert opts.downsample_cameras == 1 and opts.cams[0].width == 376 and opts.feat_rep_msckf == 4
    anchors = _iros_anchors()
    n = 30
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=4, anchors=anchors, uwb_rate=10.0,
                    uwb_sigma=0.1)
    steps = _lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"),
                      after_init=lambda m: m.try_to_initialize_uwb_anchors(anchors))
    rows, full = _stats(steps, opts.max_clone_size)
    # 2 unfixed anchors x 5 appended after their initialization
    assert steps[-1][0]["P"].shape[0] >= 15 + 14 + 10 + 6 * 10
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 50
    _check(steps, full)
