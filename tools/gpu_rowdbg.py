import os, sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import numpy as np
import uvio_amd as U
from oracle import oracle as O
from conftest import EUROC
from uvio_amd.sim import SimStream

FR = int(sys.argv[1]) if len(sys.argv) > 1 else 5
LOCK = len(sys.argv) > 2 and sys.argv[2] == "lock"
os.makedirs("gpurun_out", exist_ok=True)
for f in ("gpurun_out/g.bin", "gpurun_out/o.bin", "gpurun_out/gm.bin", "gpurun_out/om.bin"):
    if os.path.exists(f):
        os.remove(f)
opts = U.load_options(EUROC, max_msckf_in_update=200, max_slam_features=0)
s = SimStream(opts, duration=30 / opts.track_frequency + 1.2, seed=5, spawn=120)
g, o = U.VioManager(opts), O.OracleManager(opts)
Pbefore = {}


def before(nf, t):
    if LOCK:
        o.set_state(g.get_state_vector()[0], g.get_fej_vector(), g.get_cov())
    if nf == FR:
        os.environ["UVIO_HP_DUMP"] = "gpurun_out/g.bin"
        os.environ["ORC_DUMP"] = "gpurun_out/o.bin"
        os.environ["UVIO_HP_MEAS_DUMP"] = "gpurun_out/gm.bin"
        os.environ["ORC_MEAS_DUMP"] = "gpurun_out/om.bin"
        Pbefore["P"] = g.get_cov()


def after(nf, t):
    os.environ.pop("UVIO_HP_DUMP", None)
    os.environ.pop("ORC_DUMP", None)
    os.environ.pop("UVIO_HP_MEAS_DUMP", None)
    os.environ.pop("ORC_MEAS_DUMP", None)


s.run([g, o], n_frames=FR, before_frame=before, on_frame=after)


def read(path):
    a = np.fromfile(path, dtype=np.float64)
    k, out = 0, {}
    while k < len(a):
        fid, r, c = int(a[k]), int(a[k + 1]), int(a[k + 2])
        ids = a[k + 3:k + 3 + c].astype(int)
        k += 3 + c
        M = a[k:k + r * (c + 1)].reshape(r, c + 1)
        k += r * (c + 1)
        out[fid] = (ids, M)
    return out


