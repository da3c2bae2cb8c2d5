import sys, time, numpy as np
sys.path.insert(0, '.')
import uvio_amd as U
from oracle import oracle as O
from uvio_amd.sim import SimStream
rng = np.random.default_rng(0)
N, n, r = 266, 100, 100
A = rng.standard_normal((N, N)); P = A @ A.T / N + 1e-3*np.eye(N)
idx = rng.choice(N, n, replace=False).astype(np.int32); H = rng.standard_normal((r, n)); res = rng.standard_normal(r)
Pg, dxg = U.ekf_update(P, idx, H, res, 1.0); Po, dxo = O.ekf_update(P, idx, H, res, 1.0)
print('ekf rel', np.abs(Pg-Po).max()/np.abs(Po).max(), np.abs(dxg-dxo).max()/np.abs(dxo).max(), flush=True)
A = rng.standard_normal((2000, 41)); Rg = U.compress(A); Ro = O.compress(A)
s = np.sign(np.diag(Rg))*np.sign(np.diag(Ro)); print('compress rel', np.abs(Rg*s[:,None]-Ro).max()/np.abs(Ro).max(), flush=True)
opts = U.load_options('configs/euroc_mav/estimator_config.yaml', max_msckf_in_update=200, max_slam_features=0)
s = SimStream(opts, duration=3.0, spawn=200)
g = U.VioManager(opts); o = O.OracleManager(opts)
res = {}
def cb(tag, m):
    def f(nf, t):
        res.setdefault(tag, []).append((m.get_state_vector()[0], m.get_cov(), m.get_timing()))
    return f
t = time.time(); s.run(g, n_frames=40, on_frame=cb('g', g)); tg = time.time() - t
t = time.time(); s.run(o, n_frames=40, on_frame=cb('o', o)); to = time.time() - t
print('times gpu %.2f oracle %.2f' % (tg, to))
for k in range(0, 40, 4):
    a, b = res['g'][k], res['o'][k]
    print(k, a[0].shape, b[0].shape, 'x', np.abs(a[0]-b[0]).max(), 'P', np.abs(a[1]-b[1]).max()/np.abs(b[1]).max(), 'tot %.2f ms'%(a[2]['total']*1e3), a[2]['n_msckf'], b[2]['n_msckf'], a[2]['msckf_rows'], b[2]['msckf_rows'])
