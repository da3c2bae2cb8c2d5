"""Headline benchmark: VIO frames/s of the full per-frame track -> propagate -> update loop.

Workload (BASELINE.json configs[1], SURVEY.md §8 cfg 2): EuRoC V1_02-shaped stereo 752x480 rig from
configs/euroc_mav (radtan, 2 cameras, 20 Hz, 200 Hz IMU), 11 clones (+1 at update time), up to 200
MSCKF features per update and 50 SLAM landmarks.  Input: a synthetic EuRoC-shaped stream
(uvio_amd/sim.py: seeded smooth trajectory, IMU from analytic derivatives + the config's noise
densities) whose camera images are ray-cast from a textured room (uvio_amd/render.py) and are
resident in HBM before the timed region.  One step = one camera frame: the IMU samples since the
last frame, then VioManager::feed_measurement_camera (TrackKLT on the device: equalizeHist, pyramid,
FAST grid detection, cornerSubPix, stereo + temporal pyramidal LK, RANSAC) -> propagate + clone ->
MSCKF update -> SLAM update / delayed init -> marginalize.  The tracker keeps 200 features per
camera (init_max_features 400: initialize_with_gt keeps the initializer's count, VioManager.cpp:131).

Other workloads (--workload, SURVEY.md §8 cfg 3-5; parity-test cases and stress lines, not the headline):
  cfg3  TUM-VI room1-shaped stereo fisheye 512x512 images (configs/tum_vi), 20 clones, 400 tracks per
        camera, <= 400 MSCKF + 50 SLAM (LDS-tiled KLT stress)
  cfg4  UZH-FPV outdoor_45-shaped stereo fisheye rig (configs/uzhfpv_outdoor_45), 25 clones, 800 MSCKF
        features per update, each seen in all 26 clones x 2 cameras (TrackSIM feed: the backend stress case)
  cfg5  rpng_sim 4-camera rig + 6 UWB anchors (configs/rpng_sim_uwb), IMU intrinsics + g-sensitivity
        calibrated, 30 clones, 1500 MSCKF features per update (each in one camera), UWB ranges at 10 Hz

Frames/s is whole-job throughput: every rank runs its own estimator on its own stream (independent
replicas, weak scaling), value = total frames / max-over-ranks wall time.

roofline: the feature launch group (k_feature: triangulation + LM, Jacobians, left-nullspace
reflections; then k_gemm_HPg + k_chi2: the batched chi2 gate, both on the FP64 matrix cores), timed with HIP events on
the library's stream around the group; achieved = the algorithmic FP64 FLOPs of the group
(SURVEY.md §8(d) F_feat formula on the actual feature shapes) / event time.  cpu_baseline: the oracle/
CPU restatement (single-threaded, as the reference estimator is) on a bounded sample of the same
image stream, rank 0 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = os.path.join(ROOT, "configs")
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense peak (vector = matrix on gfx950)

# workload -> (config dir, camera input, option overrides, SimStream arguments, description)
WORKLOADS = {
    "cfg2": ("euroc_mav", "images",
             dict(init_max_features=400, max_msckf_in_update=200, max_slam_features=50, max_slam_in_update=25,
                  dt_slam_delay=1.0),
             dict(spawn=4),
             "cfg2 EuRoC V1_02-shaped stereo 752x480 images, 11 clones, <=200 MSCKF + 50 SLAM"),
    "cfg3": ("tum_vi", "images",
             dict(max_clone_size=20, init_max_features=800, num_pts=400, max_msckf_in_update=400,
                  max_slam_features=50, max_slam_in_update=25, dt_slam_delay=1.0),
             dict(spawn=4),
             "cfg3 TUM-VI room1-shaped stereo fisheye 512x512 images, 20 clones, 400 tracks/cam, <=400 MSCKF + 50 SLAM"),
    "cfg4": ("uzhfpv_outdoor_45", "tracks",
             dict(max_clone_size=25, max_msckf_in_update=800, max_slam_features=50, max_slam_in_update=25,
                  dt_slam_delay=1.0),
             dict(spawn=800, frac_lost=0.0, frac_long=0.02),
             "cfg4 UZH-FPV outdoor_45-shaped stereo fisheye 640x480 tracks, 25 clones, 800 MSCKF feats x 52 meas"),
    "cfg5": ("rpng_sim_uwb", "tracks",
             dict(max_clone_size=30, max_msckf_in_update=1500, max_slam_features=50, max_slam_in_update=25,
                  dt_slam_delay=1.0),
             dict(spawn=1500, frac_lost=0.0, frac_long=0.02, uwb=True),
             "cfg5 rpng_sim 4-cam 752x480 tracks + 6 UWB anchors (2 fixed), IMU intrinsics, 30 clones, 1500 MSCKF feats"),
}


def workload_options(U, name):
    cfg, _, ov, _, _ = WORKLOADS[name]
    return U.load_options(os.path.join(CONFIGS, cfg, "estimator_config.yaml"), record_timing=1, **ov)


def cfg2_options(U):
    return workload_options(U, "cfg2")


def make_stream(opts, n_frames, seed, workload="cfg2"):
    from uvio_amd.sim import SimStream
    kw = dict(WORKLOADS[workload][3])
    anchors = None
    if kw.pop("uwb", False):
        anchors = [opts.anchors[i] for i in range(opts.n_anchors)]
    # image workloads: the simulated tracks are not used (the images are); keep their generation small
    return SimStream(opts, duration=n_frames / opts.track_frequency + 1.0, seed=seed, anchors=anchors, **kw)


def render_frames(sim, n_frames, device):
    """All camera images of the first n_frames frames, resident in HBM (u8 tensors)."""
    import torch
    from uvio_amd.render import SceneRenderer
    r = SceneRenderer(sim.opts, device=device)
    frames = [[r.render(k, *sim.camera_pose(i, k), frame_seed=i) for k in range(sim.K)]
              for i in range(min(n_frames, len(sim.cam_t)))]
    torch.cuda.synchronize(device)
    return frames


class Driver:
    """Feeds one stream into one manager frame by frame (events precomputed).  frames: per camera frame
    the list of device images (feed_measurement_camera_device) or of host arrays (feed_measurement_camera)."""

    def __init__(self, sim, mgr, frames, device_imgs=True):
        """frames=None: the stream's simulated tracks (TrackSIM feed), packed per frame beforehand."""
        self.sim, self.mgr, self.frames, self.device_imgs = sim, mgr, frames, device_imgs
        if frames is None:
            from uvio_amd.manager import pack_sim_frame
            self.packed = [pack_sim_frame(f) for f in sim.frames]
        self.ev = [e for e in sim.events() if e[1] >= sim.t0 - 0.4]
        self.k = 0
        mgr.initialize_with_gt(sim.gt_state(sim.t0))

    def step(self):
        """Feed events up to and including the next camera frame; returns its timestamp."""
        sim, mgr = self.sim, self.mgr
        while True:
            kind, t, i = self.ev[self.k]
            self.k += 1
            if kind == "imu":
                mgr.feed_measurement_imu(t, sim.wm[i], sim.am[i])
            elif kind == "uwb":
                mgr.feed_measurement_uwb(t, sim.uwb[i][1], sim.uwb[i][2])
            elif t > sim.t0:
                cams = list(range(sim.K))
                if self.frames is None:
                    mgr.feed_measurement_simulation_packed(t, cams, *self.packed[i])
                elif self.device_imgs:
                    mgr.feed_measurement_camera_device(t, cams, self.frames[i])
                else:
                    mgr.feed_measurement_camera(t, cams, self.frames[i])
                return t


# newest first: the PMC passes of the current kernels (tools/gpu_final.sh), then earlier rounds'
PMC_FILES = {"cfg2": ["profiles/r01g_pmc_traffic_cfg2.json", "profiles/r01f_pmc_traffic_cfg2.json",
                      "profiles/r01e_pmc_traffic.json"],
             "cfg4": ["profiles/r01g_pmc_traffic_cfg4.json", "profiles/r01f_pmc_traffic_cfg4.json",
                      "profiles/r01_pmc_traffic_cfg4.json"]}


def pmc_traffic(workload):
    """(HBM bytes per feature-group launch, source) from the committed rocprofv3 PMC passes (FETCH_SIZE x2 +
    WRITE_SIZE, tools/pmc_summary.py) of this workload, or (None, None) if absent."""
    for path in PMC_FILES.get(workload, ["profiles/r01_pmc_traffic_%s.json" % workload]):
        try:
            with open(os.path.join(ROOT, path)) as f:
                return json.load(f)["feature_group_traffic"], path
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def max_over_ranks(x, device="cuda"):
    """Whole-job wall time: the slowest rank's (one all-reduce, outside the timed region)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--cpu-frames", type=int, default=None,
                    help="timed oracle frames for cpu_baseline (0 = skip; default: ~10-30 s of CPU work per workload)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg2")
    ap.add_argument("--shard", action="store_true",
                    help="one stream, MSCKF features sharded across the ranks (SURVEY §8e; strong scaling)")
    ap.add_argument("--shard-min", type=int, default=64, help="smallest MSCKF update that is sharded")
    args = ap.parse_args()
    if args.cpu_frames is None:
        args.cpu_frames = {"cfg2": 120, "cfg3": 60, "cfg4": 3, "cfg5": 2}[args.workload]
    # stdout carries exactly the one JSON line: whatever the libraries print (RCCL's version banner at
    # communicator creation, ...) goes to stderr
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import uvio_amd as U

    wl = args.workload
    images = WORKLOADS[wl][1] == "images"
    opts = workload_options(U, wl)
    n_frames = args.warmup + args.steps
    # replicas: one stream per rank; --shard: every rank runs the same stream and splits its MSCKF updates
    sim = make_stream(opts, n_frames + 2, seed=5 if args.shard else 5 + rank, workload=wl)
    frames = render_frames(sim, n_frames + 2, torch.device("cuda", local)) if images else None
    mgr = U.VioManager(opts, device=local)
    if args.shard:
        from uvio_amd.manager import shard_unique_id
        uid = [shard_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        mgr.enable_feature_sharding(rank, world, backend="rccl", unique_id=uid[0], min_features=args.shard_min)
    drv = Driver(sim, mgr, frames)
    for _ in range(args.warmup):
        drv.step()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    acc = {"k_feat_s": 0.0, "k_feat_flops": 0.0, "k_feat_launches": 0, "rows": 0, "n_msckf": 0, "n_slam": 0,
           "cols": 0, "cov_dim": 0, "tracks": 0, "tracking_s": 0.0}
    pos_err = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t = drv.step()
        tm = mgr.get_timing()
        acc["k_feat_s"] += tm["k_feat_s"]
        acc["k_feat_flops"] += tm["k_feat_flops"]
        acc["k_feat_launches"] += tm["k_feat_launches"]
        acc["rows"] += tm["msckf_rows"]
        acc["n_msckf"] += tm["n_msckf"]
        acc["n_slam"] += tm["n_slam"]
        acc["cols"] = max(acc["cols"], tm["msckf_cols"])
        acc["cov_dim"] = max(acc["cov_dim"], tm["cov_dim"])
        acc["tracking_s"] += tm["tracking"]
        _, x = mgr.get_imu_state()
        pos_err.append(x[4:7] - sim.traj.pos(t))
    barrier()
    t1 = time.perf_counter()
    elapsed = max_over_ranks(t1 - t0)
    ate = float(np.sqrt(np.mean(np.sum(np.array(pos_err) ** 2, axis=1))))

    if rank == 0:
        # replicas: world streams were processed; --shard: one stream, split
        value = (1 if args.shard else world) * args.steps / elapsed
        launches = max(acc["k_feat_launches"], 1)
        avg_s = acc["k_feat_s"] / launches
        flops_per_launch = acc["k_feat_flops"] / launches
        achieved = flops_per_launch / avg_s / 1e12 if avg_s > 0 else 0.0
        ntr = sum(len(mgr.get_tracks(c)[0]) for c in range(opts.num_cameras)) if images else None
        cpu = None
        if args.cpu_frames > 0:
            # the oracle needs only the clone window filled; fewer warm-up frames bound its run time
            cpu_warm = args.warmup if images else min(args.warmup, int(opts.max_clone_size) + 3)
            cpu = cpu_baseline(opts, wl, cpu_warm, args.cpu_frames, frames)
        traffic, traffic_src = pmc_traffic(wl)
        out = {
            "metric": "VIO frames/sec (track+propagate+update) at clones x feats",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if args.shard else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic %s-shaped stream (uvio_amd/sim.py, seed 5+rank) with ray-cast images "
                     "(uvio_amd/render.py) resident in HBM, TrackKLT front-end" % WORKLOADS[wl][0]) if images else
                    ("synthetic %s-shaped stream (uvio_amd/sim.py, seed 5+rank): simulated feature tracks "
                     "(TrackSIM feed, VioManager::feed_measurement_simulation)%s" %
                     (WORKLOADS[wl][0], " + UWB ranges" if opts.use_uwb else "")),
            "config": {"workload": WORKLOADS[wl][4],
                       "track_features_per_cam": int(opts.init_max_features) // int(opts.num_cameras) if images else None,
                       "tracks_last_frame": ntr, "mean_tracking_ms": 1e3 * acc["tracking_s"] / args.steps,
                       "clones": int(opts.max_clone_size), "cameras": int(opts.num_cameras),
                       "max_msckf_in_update": int(opts.max_msckf_in_update),
                       "max_slam_features": int(opts.max_slam_features),
                       "mean_msckf_feats": acc["n_msckf"] / args.steps, "mean_slam_feats": acc["n_slam"] / args.steps,
                       "mean_msckf_rows": acc["rows"] / args.steps, "H_cols": acc["cols"],
                       "state_dim": acc["cov_dim"],
                       "parallelism": ("feature-shard%d" % world) if args.shard else ("replicas%d" % world)},
            "ate_rmse_m": ate,
            "roofline": {"kernel": "feature linearize + chi2 launch group (k_feature, k_gemm_HPg, k_chi2)",
                         "bound": "mfma",
                         "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                         "avg_launch_us": avg_s * 1e6, "flops_per_launch": flops_per_launch},
            "cpu_baseline": cpu,
        }
        result_out.write(json.dumps(out) + "\n")
        result_out.flush()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(opts, wl, warmup, frames, dev_frames):
    """oracle/ (the CPU restatement) on the same stream (rank 0's), one thread, bounded sample."""
    from oracle import oracle as O
    sim = make_stream(opts, warmup + frames + 2, seed=5, workload=wl)
    if dev_frames is not None:
        frames = max(1, min(frames, len(dev_frames) - warmup - 2))
        host = [[im.cpu().numpy() for im in fr] for fr in dev_frames[:warmup + frames + 2]]
    else:
        host = None
    mgr = O.OracleManager(opts)
    drv = Driver(sim, mgr, host, device_imgs=False)
    for _ in range(warmup):
        drv.step()
    t0 = time.perf_counter()
    for _ in range(frames):
        drv.step()
    dt = time.perf_counter() - t0
    return {"value": frames / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "%d frames of the %s %s stream after %d warm-up frames, oracle/liboracle.so (g++ -O3)" %
                      (frames, wl, "image" if dev_frames is not None else "track", warmup)}


if __name__ == "__main__":
    main()
