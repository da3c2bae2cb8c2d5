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

EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense peak (vector = matrix on gfx950)


def cfg2_options(U):
    return U.load_options(EUROC, init_max_features=400, max_msckf_in_update=200, max_slam_features=50,
                          max_slam_in_update=25, dt_slam_delay=1.0, record_timing=1)


def make_stream(opts, n_frames, seed):
    from uvio_amd.sim import SimStream
    # the simulated tracks are not used (the images are); keep their generation small
    return SimStream(opts, duration=n_frames / opts.track_frequency + 1.0, seed=seed, spawn=4)


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
        self.sim, self.mgr, self.frames, self.device_imgs = sim, mgr, frames, device_imgs
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
                if self.device_imgs:
                    mgr.feed_measurement_camera_device(t, cams, self.frames[i])
                else:
                    mgr.feed_measurement_camera(t, cams, self.frames[i])
                return t


PMC_FILE = "profiles/r01_pmc_traffic.json"


def pmc_traffic():
    """HBM bytes per feature-group launch from the committed rocprofv3 PMC passes (FETCH_SIZE x2 +
    WRITE_SIZE, tools/pmc_summary.py) of this workload, or None if absent."""
    try:
        with open(os.path.join(ROOT, PMC_FILE)) as f:
            return json.load(f)["feature_group_traffic"]
    except (OSError, KeyError, ValueError):
        return None


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
    ap.add_argument("--cpu-frames", type=int, default=120, help="timed oracle frames for cpu_baseline (0 = skip)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import uvio_amd as U

    opts = cfg2_options(U)
    n_frames = args.warmup + args.steps
    sim = make_stream(opts, n_frames + 2, seed=5 + rank)
    frames = render_frames(sim, n_frames + 2, torch.device("cuda", local))
    mgr = U.VioManager(opts, device=local)
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
        value = world * args.steps / elapsed
        launches = max(acc["k_feat_launches"], 1)
        avg_s = acc["k_feat_s"] / launches
        flops_per_launch = acc["k_feat_flops"] / launches
        achieved = flops_per_launch / avg_s / 1e12 if avg_s > 0 else 0.0
        ntr = sum(len(mgr.get_tracks(c)[0]) for c in range(opts.num_cameras))
        cpu = None
        if args.cpu_frames > 0:
            cpu = cpu_baseline(opts, args.warmup, args.cpu_frames, frames)
        out = {
            "metric": "VIO frames/sec (track+propagate+update) at clones x feats",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic EuRoC-shaped stream (uvio_amd/sim.py, seed 5+rank) with ray-cast images "
                    "(uvio_amd/render.py) resident in HBM, TrackKLT front-end",
            "config": {"workload": "cfg2 EuRoC V1_02-shaped stereo 752x480 images, 11 clones, <=200 MSCKF + 50 SLAM",
                       "track_features_per_cam": int(opts.init_max_features) // int(opts.num_cameras),
                       "tracks_last_frame": ntr, "mean_tracking_ms": 1e3 * acc["tracking_s"] / args.steps,
                       "clones": int(opts.max_clone_size), "cameras": int(opts.num_cameras),
                       "max_msckf_in_update": int(opts.max_msckf_in_update),
                       "max_slam_features": int(opts.max_slam_features),
                       "mean_msckf_feats": acc["n_msckf"] / args.steps, "mean_slam_feats": acc["n_slam"] / args.steps,
                       "mean_msckf_rows": acc["rows"] / args.steps, "H_cols": acc["cols"],
                       "state_dim": acc["cov_dim"], "parallelism": "replicas%d" % world},
            "ate_rmse_m": ate,
            "roofline": {"kernel": "feature linearize + chi2 launch group (k_feature, k_gemm_HPg, k_chi2)",
                         "bound": "mfma",
                         "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": pmc_traffic(),
                         "traffic_source": PMC_FILE if pmc_traffic() is not None else None,
                         "avg_launch_us": avg_s * 1e6, "flops_per_launch": flops_per_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(opts, warmup, frames, dev_frames):
    """oracle/ (the CPU restatement) on the same image stream (rank 0's), one thread, bounded sample."""
    from oracle import oracle as O
    frames = max(1, min(frames, len(dev_frames) - warmup - 2))
    sim = make_stream(opts, warmup + frames + 2, seed=5)
    host = [[im.cpu().numpy() for im in fr] for fr in dev_frames[:warmup + frames + 2]]
    mgr = O.OracleManager(opts)
    drv = Driver(sim, mgr, host, device_imgs=False)
    for _ in range(warmup):
        drv.step()
    t0 = time.perf_counter()
    for _ in range(frames):
        drv.step()
    dt = time.perf_counter() - t0
    return {"value": frames / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "%d frames of the cfg2 image stream after %d warm-up frames, oracle/liboracle.so (g++ -O3)" %
                      (frames, warmup)}


if __name__ == "__main__":
    main()
