"""Diagnostic: lock-step cfg5 variants (4 cameras / UWB / IMU intrinsics toggled), first differing frame."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import uvio_amd as U  # noqa: E402
from oracle import oracle as O  # noqa: E402
from uvio_amd.sim import SimStream  # noqa: E402
from test_gpu_parity import _snap, _rel  # noqa: E402

CFG = os.path.join(ROOT, "configs", "rpng_sim_uwb", "estimator_config.yaml")


EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")


def run(name, uwb, cfg=CFG, **ov):
    kw = dict(max_msckf_in_update=150, max_slam_features=10, max_slam_in_update=5, dt_slam_delay=0.3,
              min_dist_to_use_uwb=0.05)
    kw.update(ov)
    opts = U.load_options(cfg, **kw)
    if not uwb:
        opts.use_uwb = 0
        opts.n_anchors = 0
    anc = [opts.anchors[i] for i in range(opts.n_anchors)] if uwb else None
    s = SimStream(opts, duration=30 / opts.track_frequency + 1.2, seed=5, anchors=anc, spawn=120, frac_long=0.2)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    res = {"first": None}

    def before(nf, t):
        o.set_state(g.get_state_vector()[0], g.get_fej_vector(), g.get_cov())

    def after(nf, t):
        a, b = _snap(g), _snap(o)
        ig, pg, sg, cg = a["feats"]
        io, po, so, co = b["feats"]
        mo = {int(i): k for k, i in enumerate(io)}
        bad = []
        for k, i in enumerate(ig):
            j = mo.get(int(i))
            if j is None or sg[k] != so[j] or (sg[k] != 1 and np.abs(pg[k] - po[j]).max() > 1e-6):
                bad.append((int(i), int(sg[k]), int(so[j]) if j is not None else None,
                            float(np.abs(pg[k] - po[j]).max()) if j is not None else None))
        x = _rel(a["x"], b["x"]) if a["x"].shape == b["x"].shape else -1
        if (bad or x > 1e-8) and res["first"] is None:
            res["first"] = nf
            print("  %s: frame %d  n_feats %d  bad %d %s  x %.2e  n_slam %d/%d delayed %d/%d" % (
                name, nf, len(ig), len(bad), bad[:4], x, a["timing"]["n_slam"], b["timing"]["n_slam"],
                a["timing"]["n_slam_delayed"], b["timing"]["n_slam_delayed"]))
            for (fid, sgg, soo, dp) in bad[:2]:
                k = list(ig).index(fid)
                print("    feat %d  g p %s chi2 %.4f | o p %s chi2 %.4f" % (fid, pg[k], cg[k], po[mo[fid]], co[mo[fid]]))
            if a["x"].shape == b["x"].shape and False:
                meta = a["meta"]
                off = 0
                for v in range(len(meta) // 3 if meta.ndim == 1 else len(meta)):
                    kind, cid, csz = (meta[3 * v:3 * v + 3] if meta.ndim == 1 else meta[v])
                    vl = {0: 16, 1: csz, 2: 4, 3: 7, 4: 3, 5: 5}.get(int(kind), csz)
                    d = np.abs(a["x"][off:off + vl] - b["x"][off:off + vl]).max()
                    if d > 1e-9:
                        print("    var %d kind %d id %d size %d diff %.2e" % (v, kind, cid, csz, d))
                    off += vl

    s.run([g, o], n_frames=30, before_frame=before, on_frame=after)
    g.close()
    print("%s: first bad frame %s" % (name, res["first"]), flush=True)


def uwb_only(name, cfg=CFG, n=14, **ov):
    kw = dict(max_msckf_in_update=0, max_slam_features=0, min_dist_to_use_uwb=0.05)
    kw.update(ov)
    opts = U.load_options(cfg, **kw)
    anc = [opts.anchors[i] for i in range(opts.n_anchors)]
    s = SimStream(opts, duration=n / opts.track_frequency + 1.2, seed=5, anchors=anc, spawn=40)
    g, o = U.VioManager(opts), O.OracleManager(opts)
    line = []

    def before(nf, t):
        o.set_state(g.get_state_vector()[0], g.get_fej_vector(), g.get_cov())

    def after(nf, t):
        a, b = _snap(g), _snap(o)
        x = _rel(a["x"], b["x"]) if a["x"].shape == b["x"].shape else -1
        P = _rel(a["P"], b["P"]) if a["P"].shape == b["P"].shape else -1
        line.append("%d:%.1e/%.1e" % (nf, x, P))

    s.run([g, o], n_frames=n, before_frame=before, on_frame=after)
    g.close()
    print(name, " ".join(line), flush=True)


for args in [("D-uwb+msckf", dict(max_msckf_in_update=150, do_calib_imu_intrinsics=0, do_calib_imu_g_sensitivity=0)),
             ("E-uwb+msckf-nodt", dict(max_msckf_in_update=150, do_calib_imu_intrinsics=0,
                                       do_calib_imu_g_sensitivity=0, do_calib_camera_timeoffset=0)),
             ("F-uwb+msckf-noext", dict(max_msckf_in_update=150, do_calib_imu_intrinsics=0,
                                        do_calib_imu_g_sensitivity=0, do_calib_camera_pose=0)),
             ("G-uwb+msckf-nointr", dict(max_msckf_in_update=150, do_calib_imu_intrinsics=0,
                                         do_calib_imu_g_sensitivity=0, do_calib_camera_intrinsics=0))]:
    try:
        uwb_only(args[0], **args[1])
    except Exception as e:  # noqa: BLE001
        print("%s: exception %s" % (args[0], e), flush=True)
