"""cfg2l's ATE: the oracle (CPU, oracle/liboracle.so) on the cfg2l stream with the scene churn the workload uses
(churn = 3: texture panels redrawn under the tracks) and without it, same trajectory and seed.
usage: python tools/ate_churn.py [frames] [warmup]"""
import sys

sys.path.insert(0, ".")
import numpy as np

import bench as B
import uvio_amd as U
from oracle import oracle as O
from uvio_amd.evaluation import ate

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 150
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 40
O.set_threads(4)
for churn in (3, 0):
    opts = B.workload_options(U, "cfg2l")
    sim = B.make_stream(opts, warm + frames + 2, seed=5, workload="cfg2l", extra={"churn": churn})
    fr = B.Frames(sim, "cpu")
    host = {i: [im.numpy() for im in fr[i]] for i in range(warm + frames + 2)}
    mgr = O.OracleManager(opts)
    drv = B.Driver(sim, mgr, host, device_imgs=False)
    ep, gp, eq, gq = [], [], [], []
    nm = 0
    for k in range(warm + frames):
        t = drv.step()
        if k < warm:
            continue
        x = mgr.get_imu_state()[1]
        g = sim.gt_state(t)
        ep.append(x[4:7].copy())
        eq.append(x[0:4].copy())
        gp.append(g[5:8])
        gq.append(g[1:5])
    a = ate(ep, gp, eq, gq, align="posyaw")
    print("churn %d: ATE %.4f m, %.3f deg over %d frames (after %d)" % (churn, a["pos_m"], a["ori_deg"], frames, warm),
          flush=True)
