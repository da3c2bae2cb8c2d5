"""cfg5 (TrackSIM) with every UWB anchor fixed: the first frame whose IMU state is not finite, with the frame's
timing counters and the covariance diagonal's minimum, on the device (and the oracle for the same frames when
--oracle is given)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import bench as B
import uvio_amd as U

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
opts = B.workload_options(U, "cfg5", {"anchors_fix": 1})
sim = B.make_stream(opts, n + 60, seed=5, workload="cfg5")
mgr = U.VioManager(opts)
drv = B.Driver(sim, mgr, None)
for k in range(n + 40):
    try:
        drv.step()
    except RuntimeError as e:
        print("frame", k, "error", e)
        break
    x = mgr.get_imu_state()[1]
    P = mgr.get_cov()
    tm = mgr.get_timing()
    bad = not np.all(np.isfinite(x)) or not np.all(np.isfinite(P))
    if k % 20 == 0 or bad:
        print("frame %d t %.3f clones %d N %d msckf %d slam %d delayed %d minPdiag %.3e |v| %.3f finite %s" % (
            k, tm["timestamp"], tm["n_clones"], tm["cov_dim"], tm["n_msckf"], tm["n_slam"], tm["n_slam_delayed"],
            np.min(np.diag(P)), np.linalg.norm(x[7:10]), not bad), flush=True)
    if bad:
        break
