"""Per-stage frame timings (the reference CSV schema, VioManager.cpp:631-644) of a bench workload.

usage: python tools/stage_times.py cfg4 [frames] [record_timing]
record_timing 2 waits for the device at every stage boundary, so each stage includes its kernels."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import uvio_amd as U  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rt = int(sys.argv[3]) if len(sys.argv) > 3 else 2
import torch  # noqa: E402,F401
opts = bench.workload_options(U, wl)
opts.record_timing = rt
warm = int(opts.max_clone_size) + 8
sim = bench.make_stream(opts, warm + n + 2, seed=5, workload=wl)
images = bench.WORKLOADS[wl][1] == "images"
frames = bench.render_frames(sim, warm + n + 2, torch.device("cuda", 0)) if images else None
mgr = U.VioManager(opts)
drv = bench.Driver(sim, mgr, frames)
for _ in range(warm):
    drv.step()
keys = ["tracking", "propagation", "msckf_update", "slam_update", "slam_delayed", "marg", "total", "sync_wait",
        "k_feat_s"]
acc = {k: [] for k in keys + ["device_syncs", "n_msckf", "msckf_rows"]}
for _ in range(n):
    drv.step()
    tm = mgr.get_timing()
    for k in acc:
        acc[k].append(tm[k])
print("%s  record_timing %d  frames %d" % (wl, rt, n))
for k in keys:
    print("  %-14s %8.3f ms" % (k, 1e3 * np.mean(acc[k])))
for k in ["device_syncs", "n_msckf", "msckf_rows"]:
    print("  %-14s %8.1f" % (k, np.mean(acc[k])))
mgr.close()  # prints the UVIO_HP_HOST_PROF sections when enabled
