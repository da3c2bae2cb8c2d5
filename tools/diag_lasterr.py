"""Find which library call leaves a sticky HIP error (diagnostic)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import uvio_amd as U
from uvio_amd.render import SceneRenderer
from uvio_amd.sim import SimStream

hip = C.CDLL("libamdhip64.so")
EUROC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "euroc_mav", "estimator_config.yaml")
opts = U.load_options(EUROC, init_max_features=200, max_msckf_in_update=200, max_slam_features=25,
                      max_slam_in_update=25, dt_slam_delay=1.0)
s = SimStream(opts, duration=30 / 20 + 1.2, seed=5, spawn=10)
r = SceneRenderer(opts, device="cuda")
g = U.VioManager(opts)


def chk(what):
    e = hip.hipGetLastError()
    if e:
        print("sticky error", e, "after", what, flush=True)


class W:
    def __init__(self, m):
        self.m = m

    def __getattr__(self, k):
        f = getattr(self.m, k)
        if not callable(f):
            return f

        def w(*a, **kw):
            out = f(*a, **kw)
            chk(k)
            return out
        return w


s.run(W(g), n_frames=30, before_frame=lambda nf, t: (g.get_state_vector(), chk("gsv"), g.get_fej_vector(), chk("fej"), g.get_cov(), chk("cov")),
      on_frame=lambda nf, t: (print("frame", nf, flush=True), g.debug_last_msckf(), chk("dbg"), g.get_timing(), chk("tm")), renderer=r)
print("done")
