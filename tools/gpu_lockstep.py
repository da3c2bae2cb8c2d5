"""Print the lock-step / free-run parity figures (used to set the tolerances in tests/test_gpu_parity.py)."""
import sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import numpy as np
import uvio_amd as U
import test_gpu_parity as T
from conftest import EUROC

for name, kw, simkw in [("msckf", dict(max_msckf_in_update=200, max_slam_features=0), dict(spawn=120)),
                        ("slam", dict(max_msckf_in_update=100, max_slam_features=20, max_slam_in_update=10,
                                      dt_slam_delay=0.3), dict(spawn=80, frac_long=0.3))]:
    opts = U.load_options(EUROC, **kw)
    steps = T._lockstep(opts, 30, **simkw)
    for k, (a, b) in enumerate(steps):
        try:
            p, c = T._compare_feats(a["feats"], b["feats"])
        except AssertionError as e:
            p, c = -1, str(e)
        print(name, "lock", k, a["timing"]["n_msckf"], a["timing"]["n_slam"], a["timing"]["n_slam_delayed"],
              b["timing"]["n_msckf"], b["timing"]["n_slam"], b["timing"]["n_slam_delayed"],
              "p %.2e" % p, "c", c, "x %.2e P %.2e" % (T._rel(a["x"], b["x"]) if a["x"].shape == b["x"].shape else -1,
                                                      T._rel(a["P"], b["P"]) if a["P"].shape == b["P"].shape else -1))
    G, O = T._free_run(opts, 30, **simkw)
    for k, (a, b) in enumerate(zip(G, O)):
        ok = a["x"].shape == b["x"].shape
        print(name, "free", k, a["timing"]["n_msckf"], b["timing"]["n_msckf"], "x %.2e" % (T._rel(a["x"], b["x"]) if ok else -1),
              "pose %.2e %.2e" % T._pose_err(a, b))
