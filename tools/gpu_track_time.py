"""Per-frame timing of the image path (product) on rendered frames: tracking / total, syncs."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import uvio_amd as U  # noqa: E402
from uvio_amd.render import SceneRenderer  # noqa: E402
from uvio_amd.sim import SimStream  # noqa: E402

EUROC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "euroc_mav",
                     "estimator_config.yaml")
nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 80
opts = U.load_options(EUROC, init_max_features=400, max_msckf_in_update=200, max_slam_features=50,
                      max_slam_in_update=25, dt_slam_delay=1.0, record_timing=1)
s = SimStream(opts, duration=nfr / opts.track_frequency + 1.2, seed=5, spawn=10)
r = SceneRenderer(opts, device="cuda")
frames = [[r.render(k, *s.camera_pose(i, k), frame_seed=i) for k in range(2)] for i in range(nfr)]
torch.cuda.synchronize()
g = U.VioManager(opts)
g.initialize_with_gt(s.gt_state(s.t0))
tr, tot, wall, allt = [], [], [], []
nf = 0
for kind, t, i in s.events():
    if t < s.t0 - 0.4:
        continue
    if kind == "imu":
        g.feed_measurement_imu(t, s.wm[i], s.am[i])
    elif kind == "cam":
        if t <= s.t0:
            continue
        t0 = time.perf_counter()
        g.feed_measurement_camera_device(t, [0, 1], frames[i])
        wall.append(time.perf_counter() - t0)
        tm = g.get_timing()
        allt.append(tm)
        tr.append(tm["tracking"])
        tot.append(tm["total"])
        nf += 1
        if nf >= nfr:
            break
k = 20
x = g.get_imu_state()[1]
gt = s.gt_state(s.cam_t[nf - 1])
print("frames %d  track %.3f ms  total %.3f ms  wall %.3f ms  fps %.1f  pos err %.4f m  tracks %d/%d" % (
    nf, 1e3 * np.mean(tr[k:]), 1e3 * np.mean(tot[k:]), 1e3 * np.mean(wall[k:]), 1.0 / np.mean(wall[k:]),
    np.abs(x[4:7] - gt[5:8]).max(), len(g.get_tracks(0)[0]), len(g.get_tracks(1)[0])))
for key in ["tracking", "propagation", "msckf_update", "slam_update", "slam_delayed", "marg", "total", "n_msckf",
            "n_slam", "n_slam_delayed", "msckf_rows", "k_feat_launches", "device_syncs", "sync_wait"]:
    print("  %-16s %10.4f" % (key, np.mean([a[key] for a in allt[k:]]) * (1e3 if isinstance(allt[0][key], float) else 1)))
