"""Diagnostic: the device chain (update_frame) against the per-updater path (UVIO_HP_NO_CHAIN) on the same
stream with stale frames, device only: first differing frame, per-kind differences."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import uvio_amd as U  # noqa: E402
from test_gpu_parity import _rel, _sim, _snap  # noqa: E402

opts = U.load_options(os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml"), max_msckf_in_update=100,
                      max_slam_features=20, max_slam_in_update=10, dt_slam_delay=0.3)
stale_at = [int(a) for a in sys.argv[1:]] or [12, 18]
n = 30
s = _sim(opts, n, spawn=80, frac_long=0.3)
cams = list(range(s.K))
ga = U.VioManager(opts)
os.environ["UVIO_HP_NO_CHAIN"] = "1"
gb = U.VioManager(opts)
del os.environ["UVIO_HP_NO_CHAIN"]
rows = []


def before(nf, t):
    gb.set_state(ga.get_state_vector()[0], ga.get_fej_vector(), ga.get_cov())
    if nf in stale_at:
        i = int(np.argmin(np.abs(np.asarray(s.cam_t) - t)))
        for m in (ga, gb):
            try:
                m.feed_measurement_simulation(0.5 * (s.cam_t[i - 3] + s.cam_t[i - 4]), cams, s.frames[i - 3])
            except RuntimeError:
                pass


def after(nf, t):
    rows.append((_snap(ga), _snap(gb)))


s.run([ga, gb], n_frames=n, before_frame=before, on_frame=after)
for k, (a, b) in enumerate(rows):
    kg, ig, pg, sg, cg = a["frame"]
    ko, io, po, so, co = b["frame"]
    tg = {(int(kg[q]), int(ig[q])): (pg[q], sg[q], cg[q]) for q in range(len(ig))}
    to = {(int(ko[q]), int(io[q])): (po[q], so[q], co[q]) for q in range(len(io))}
    worst = {}
    for key, (p1, s1, c1) in tg.items():
        if key not in to:
            worst.setdefault(key[0], []).append(("missing", key[1]))
            continue
        p2, s2, c2 = to[key]
        d = (float(np.abs(p1 - p2).max()) if s1 != 1 else 0.0, abs(c1 - c2) / max(abs(c2), 1.0), int(s1), int(s2))
        if d[0] > 0 or d[1] > 0 or s1 != s2:
            worst.setdefault(key[0], []).append((key[1],) + d)
    for key in to:
        if key not in tg:
            worst.setdefault(key[0], []).append(("extra", key[1]))
    print("frame %2d x %.1e P %.1e msckf %3d slam %2d delayed %2d" % (k, _rel(a["x"], b["x"]), _rel(a["P"], b["P"]),
          a["timing"]["n_msckf"], a["timing"]["n_slam"], a["timing"]["n_slam_delayed"]),
          {kk: v[:6] for kk, v in worst.items()} if worst else "")
