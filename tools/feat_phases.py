"""Per-phase cycle counts of the feature kernel (UVIO_HP_FEAT_TS debug dump) on a bench workload.

usage: python tools/feat_phases.py [cfg2|cfg3|cfg4|cfg5]"""
import os, sys
sys.path.insert(0, '.')
import numpy as np
os.makedirs("gpurun_out", exist_ok=True)
path = "gpurun_out/feat_ts.bin"
if os.path.exists(path):
    os.remove(path)
import bench, uvio_amd as U
wl = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
opts = bench.workload_options(U, wl)
warm = int(opts.max_clone_size) + 8
sim = bench.make_stream(opts, warm + 12, seed=5, workload=wl)
images = bench.WORKLOADS[wl][1] == "images"
frames = bench.Frames(sim, "cuda") if images else None
if frames is not None:
    frames.prerender(0, warm + 12)
mgr = U.VioManager(opts)
drv = bench.Driver(sim, mgr, frames)
for _ in range(warm):
    drv.step()
os.environ["UVIO_HP_FEAT_TS"] = path
for _ in range(10):
    drv.step()
os.environ.pop("UVIO_HP_FEAT_TS")
a = np.fromfile(path, dtype=np.int64).reshape(-1, 16)
names = ["setup", "geom", "jacob", "nullsp", "T/S", "chol", "output"]
for mode in sorted(set(a[:, 0])):
    for big in (False, True):
        sel = a[(a[:, 0] == mode) & ((a[:, 1] > 1) == big)]
        if len(sel) == 0:
            continue
        ts = sel[:, 4:12].astype(float)
        d = np.diff(ts, axis=1)
        d[d < 0] = np.nan
        print("mode %d %s launches-feats %d  meas %.1f nf %.1f | " % (mode, "batch" if big else "single", len(sel),
              sel[:, 2].mean(), sel[:, 3].mean()) + "  ".join("%s %.0f" % (n, v) for n, v in zip(names, np.nanmean(d, axis=0))),
              " total %.0f cyc" % np.nanmean(ts[:, 7] - ts[:, 0]))
        if mode == 3:  # nullspace sub-phases: reflectors formed (wave 0), barrier, applied
            sub = sel[:, [7, 12, 13, 14, 8]].astype(float)
            ds = np.diff(sub, axis=1)
            print("      nullspace: reflectors %.0f  barrier %.0f  apply %.0f  barrier %.0f  cyc" % tuple(np.nanmean(ds, axis=0)))
            continue
        c = sel[:, 12:16].astype(float)
        c = c[c[:, 3] > 0]
        if len(c):
            dc = np.diff(c, axis=1)
            print("      chi2: stage+S %.0f  ldl %.0f  chi2 %.0f  cyc (n=%d)" % tuple(list(np.mean(dc, axis=0)) + [len(c)]))
            k = int(np.argmax(c[:, 3] - c[:, 0]))
            print("      chi2 slowest feature (meas %d): stage+S %.0f  ldl %.0f  chi2 %.0f  cyc" % (
                sel[sel[:, 15] > 0][k, 2], *dc[k]))
