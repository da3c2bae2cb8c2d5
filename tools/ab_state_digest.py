"""Digest of the filter after N frames of a bench workload (state vector, FEJ vector, covariance, active tracks),
to compare two builds of the library bit for bit (UVIO_HP_LIB selects the library).

usage: python tools/ab_state_digest.py WORKLOAD FRAMES"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import uvio_amd as U  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 40
opts = bench.workload_options(U, wl)
sim = bench.make_stream(opts, frames, seed=5, workload=wl)
images = bench.WORKLOADS[wl][1] == "images"
fr = bench.Frames(sim, "cuda") if images else None
if fr is not None:
    fr.prerender(0, frames)
mgr = U.VioManager(opts)
drv = bench.Driver(sim, mgr, fr)
h = hashlib.sha256()
for k in range(frames):
    drv.step()
    x, meta = mgr.get_state_vector()
    h.update(x.tobytes())
    h.update(meta.tobytes())
h.update(mgr.get_fej_vector().tobytes())
h.update(np.ascontiguousarray(mgr.get_cov()).tobytes())
if images:
    t, P, D = mgr.get_active_tracks()
    for k in sorted(P):
        h.update(np.uint64(k).tobytes())
        h.update(P[k].tobytes())
        if k in D:
            h.update(D[k].tobytes())
print("%s %d frames lib %s digest %s" % (wl, frames, os.path.basename(os.environ.get("UVIO_HP_LIB", "libuvio_hp.so")),
                                          h.hexdigest()[:24]))
