"""The per-frame timing CSV (VioManagerOptions record_timing_information / record_timing_filepath) against the
reference's schema and rows (VioManager.cpp:105-122 header, :631-644 rows): the file is replaced at creation,
its header names the reference's columns (the SLAM pair only with max_slam_features > 0), and every frame that
runs the whole update (clone window >= min(max_clone_size, 5), VioManager.cpp:360-363) appends one row of the
state time in the IMU clock (timestamp + t_ItoC, %.15f) and the stage times (%.5f) uvio_hp_get_timing reports.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")


def _run(tmp_path, slam):
    import uvio_amd as U
    from uvio_amd.sim import SimStream
    path = tmp_path / "sub" / "timing.csv"
    path.parent.mkdir()
    path.write_text("stale\n")
    opts = U.load_options(EUROC, max_msckf_in_update=60, max_slam_features=10 if slam else 0, max_slam_in_update=5,
                          dt_slam_delay=0.3, record_timing_information=1, record_timing_filepath=str(path).encode())
    n = 16
    sim = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, spawn=60, frac_long=0.3)
    g = U.VioManager(opts)
    frames = []

    def after(nf, t):
        # t_ItoC of the state (variable after the IMU's 16 values: configs/euroc_mav calibrates it)
        frames.append((g.get_timing(), g.get_imu_state()[0] + g.get_state_vector()[0][16]))

    sim.run(g, n_frames=n, on_frame=after)
    g.close()
    return opts, path.read_text().splitlines(), frames


@pytest.mark.parametrize("slam", [True, False])
def test_timing_csv_schema_and_rows(tmp_path, slam):
    opts, lines, frames = _run(tmp_path, slam)
    head = "# timestamp (sec),tracking,propagation,msckf update,"
    if slam:
        head += "slam update,slam delayed,"
    head += "re-tri & marg,total"
    assert lines[0] == head  # the stale file was replaced
    rows = [ln.split(",") for ln in lines[1:]]
    want = [(tm, t) for tm, t in frames if tm["n_clones"] >= min(opts.max_clone_size, 5)]
    assert opts.calib_camimu_dt is not None and len(want) >= 8 and len(rows) == len(want)
    cols = ["tracking", "propagation", "msckf_update"] + (["slam_update", "slam_delayed"] if slam else []) + \
           ["marg", "total"]
    for r, (tm, t) in zip(rows, want):
        assert len(r) == 1 + len(cols)
        assert r[0] == "%.15f" % t
        for c, v in zip(cols, r[1:]):
            assert v == "%.5f" % tm[c], (c, v, tm[c])
        vals = np.array([float(v) for v in r[1:]])
        assert np.all(vals >= 0) and vals[-1] >= vals[:-1].max()
