"""Determinism check: the same cfg2 image stream through the binding twice (host images), with and without the
tracker's predetect; first differing frame and magnitude."""
import os
import sys
import numpy as np
sys.path.insert(0, ".")
import bench as B
import uvio_amd as U


def run(n, device_imgs, env=None):
    if env:
        os.environ.update(env)
    opts = B.workload_options(U, "cfg2")
    sim = B.make_stream(opts, n + 4, seed=5, workload="cfg2")
    import torch
    fr = B.Frames(sim, torch.device("cuda", 0))
    frames = fr if device_imgs else {i: [im.cpu().numpy() for im in fr[i]] for i in range(n + 4)}
    m = U.VioManager(opts)
    d = B.Driver(sim, m, frames, device_imgs=device_imgs)
    xs = []
    for _ in range(n):
        d.step()
        xs.append(m.get_imu_state()[1].copy())
    m.close()
    if env:
        for k in env:
            os.environ.pop(k)
    return np.array(xs)


n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
a = run(n, False)
b = run(n, False)
c = run(n, True)
d = run(n, False, {"UVIO_HP_NO_PREDETECT": "1"})
for name, y in (("host twice", b), ("device feed", c), ("no predetect", d)):
    diff = np.abs(a - y).max(axis=1)
    bad = np.nonzero(diff > 0)[0]
    print("%-14s first differing frame %s  max diff %.3e" % (name, bad[0] if len(bad) else None, diff.max()), flush=True)
