"""The device engine's start from rest (VioManager::try_to_initialize -> InertialInitializer /
StaticInitializer, engine_init.cpp) in lock-step with the oracle (tests/test_static_init.py pins the oracle):
a platform that rests for its first 2.2 s and then moves, mono downsampled images of the shipped
iros_2023_uvio config, no initialize_with_gt.  Both sides stay uninitialized on the same frames, initialize
on the same frame with the same state and covariance (computed independently on each side: the oracle does
not adopt the device's state before the device is initialized; the frame whose initializer succeeds ends
there and the next frame reports initialized, as the reference's single-threaded try_to_initialize), then the zero-velocity updates at rest and
the MSCKF updates once moving follow the strict lock-step bounds of test_gpu_parity.py."""
import os

import numpy as np
import pytest

from test_gpu_parity import _check_lockstep, _rel, _sim, run_lockstep

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IROS = os.path.join(ROOT, "configs", "iros_2023_uvio", "estimator_config.yaml")


def test_static_start_lockstep_images():
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    opts = U.load_options(IROS, init_max_features=100, use_uwb=0)
    n = 24
    sim = _sim(opts, n, spawn=4, static_for=1.2)
    steps = run_lockstep(opts, sim, n, renderer=SceneRenderer(opts, device="cuda"), init="static")
    flags = [a["init"] for a, _ in steps]
    assert flags == [b["init"] for _, b in steps]
    assert not flags[0] and flags[-1], flags
    k = flags.index(True)
    # the initializer succeeded one frame earlier: that frame ended there, with the initialized state and no clone
    # (VioManagerHelper.cpp:164,187 return false; thread_init_success reports it on the next frame, :91-93)
    a0, b0 = steps[k - 1]
    assert a0["timing"]["n_clones"] == 0 and b0["timing"]["n_clones"] == 0
    assert a0["timing"]["n_msckf"] == 0 and a0["timing"]["zupt"] == 0
    assert _rel(a0["x"], b0["x"]) < 1e-10 and _rel(a0["P"], b0["P"]) < 1e-10, (_rel(a0["x"], b0["x"]),)
    a, b = steps[k]
    # the first initialized frame: independent on both sides (propagation from the initializer's time and the
    # first clone; its zero-velocity check is skipped, VioManager.cpp:294 reads is_initialized_vio before :310)
    assert a["timing"]["n_clones"] == 1 and b["timing"]["n_clones"] == 1 and a["timing"]["zupt"] == 0
    assert _rel(a["x"], b["x"]) < 1e-10 and _rel(a["P"], b["P"]) < 1e-10, (_rel(a["x"], b["x"]), _rel(a["P"], b["P"]))
    assert sum(s[0]["timing"]["zupt"] for s in steps[k:]) >= 1
    assert sum(s[0]["timing"]["n_msckf"] for s in steps[k:]) > 20
    _check_lockstep(steps)
