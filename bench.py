"""Headline benchmark: VIO frames/s of the full per-frame track -> propagate -> update loop.

Workload at N = 1: cfg3 (BASELINE.json configs[2], SURVEY.md §8 cfg 3), the largest single-GPU configuration of
BASELINE.json: a TUM-VI room1-shaped stereo fisheye 512x512 rig from configs/tum_vi (equidistant, 2 cameras,
20 Hz, 200 Hz IMU), 20 clones (+1 at update time), 400 tracks per camera, up to 400 MSCKF features per update
and 50 SLAM landmarks.  Input: a synthetic stream (uvio_amd/sim.py: seeded smooth trajectory, IMU from analytic
derivatives + the config's noise densities) whose camera images are ray-cast from a textured room
(uvio_amd/render.py) and are resident in HBM before the timed region.  One step = one camera frame: the IMU
samples since the last frame, then VioManager::feed_measurement_camera (TrackKLT on the device: equalizeHist,
pyramid, FAST grid detection, cornerSubPix, stereo + temporal pyramidal LK, RANSAC) -> propagate + clone ->
MSCKF update -> SLAM update / delayed init -> marginalize.  The same frames are then fed once more as host
images (uvio_hp_feed_camera, the reference caller's form: the library uploads them) into a second estimator;
that rate is reported as "host_feed" (PCIe-inclusive, never "value").

Steady state: the warm-up runs at least --warmup frames and then until the clone window is full
(max_clones + 1 clones at update time) and the SLAM slots are >= 90 % populated (at most --max-warmup
frames); the line reports the effective warm-up and whether steady state was reached.

Multi-GPU (--gpus N > 1; launched either by torch.distributed.run, or by this script itself, which then
spawns N worker processes before any GPU call): value = one independent cfg3 estimator per GPU (the N = 1
workload on every rank, seed 5 + rank; scaling "weak", value = all ranks' frames / the slowest rank's time), so
the per-N values of one command compare like with like.  In the same job the line's "feature_sharded" object
measures the north star's feature-sharded update: every rank runs the same BASELINE stream --
cfg4 (UZH-FPV, 25 clones x 800 features per update) at N <= 4, cfg5 (rpng_sim 4 cameras + UWB, 30 clones x 1500
features) at N > 4 -- and each MSCKF update's per-feature linearization, chi2 gate and Gram are split across the
ranks with one RCCL all-reduce (scaling "strong"), next to rank 0's unsharded time on the same stream.  --shard
makes the sharded run the value instead.

Other workloads (--workload, SURVEY.md §8 cfg 1-5; parity-test cases and stress lines):
  cfg1  EuRoC MH_01-shaped MONO 752x480 images (configs/euroc_mav, max_cameras 1), 11 clones, <= 100 MSCKF
  cfg2  EuRoC V1_02-shaped stereo 752x480 images (configs/euroc_mav), 11 clones, <= 200 MSCKF + 50 SLAM
  cfg2l cfg2 with track loss (scene churn: each texture panel redraws every 8 frames), 400 tracks
  cfg3t cfg3's rig and window with a TrackSIM feed at BASELINE's MSCKF load: 400 features per update, each seen
        in every clone by both cameras (the N = 1 line's "msckf_load" companion, --msckf-load-steps)
  cfg4 / cfg5  the backend stress at BASELINE's feature counts: TrackSIM feed with 800 / 1500 MSCKF features
        per update, each seen in every clone (26 clones x 2 cameras / 31 clones x 1 of 4 cameras, + 6 UWB
        anchors and IMU intrinsics + g-sensitivity at cfg5) -- the shapes BASELINE.json's cfg4 / cfg5 name
  cfg4i UZH-FPV outdoor_45-shaped stereo fisheye 640x480 images (configs/uzhfpv_outdoor_45), 25 clones,
        800 tracks, <= 800 MSCKF + 50 SLAM (TrackKLT front-end on rendered images)
  cfg5i rpng_sim 4-camera 752x480 images, each camera tracked on its own (configs/rpng_sim_uwb), + 6 UWB
        anchors at 10 Hz, IMU intrinsics + g-sensitivity calibrated, 30 clones, 1500 tracks
  (cfg4t / cfg5t, the names of cfg4 / cfg5 in rounds 1-3, and cfg4 / cfg5 images of round 3 = cfg4i / cfg5i)

roofline: live HIP-event timing of the kernel classes (uvio_hp_set_kernel_timing) over the timed region;
achieved = algorithmic FLOPs (FP64 classes) or bytes (tracker classes) of the class's launches (SURVEY.md
§8(d), formulas in DESIGN.md §6) / their summed event time; "roofline" is the class with the largest device
time in this run (the EKF-update chain aggregate excluded, its LDL factor is its own class), "rooflines" lists
every class.  traffic = HBM bytes per launch from the committed rocprofv3 PMC passes of the same workload
(profiles/, FETCH_SIZE x 2 + WRITE_SIZE); mfma_util = SQ_VALU_MFMA_BUSY_CYCLES of the class's kernels over
(launch duration x shader clock x 256 CUs), from the same committed passes.  cpu_baseline: the oracle/ CPU
restatement on a bounded sample of the same stream, rank 0 only.  ate: posyaw-aligned ATE RMSE against the
stream's ground truth (ov_eval's definition, uvio_amd/evaluation.py).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = os.path.join(ROOT, "configs")
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense peak (vector = matrix on gfx950), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak, MI355X_MICROARCH.md "HBM"

# workload -> (config dir, camera input, option overrides, SimStream arguments, description)
WORKLOADS = {
    "cfg1": ("euroc_mav", "images",
             dict(num_cameras=1, use_stereo=0, init_max_features=200, max_msckf_in_update=100, max_slam_features=50,
                  max_slam_in_update=25, dt_slam_delay=1.0),
             dict(spawn=4),
             "cfg1 EuRoC MH_01-shaped mono 752x480 images, 11 clones, <=100 MSCKF + 50 SLAM"),
    "cfg2": ("euroc_mav", "images",
             dict(init_max_features=400, max_msckf_in_update=200, max_slam_features=50, max_slam_in_update=25,
                  dt_slam_delay=1.0),
             dict(spawn=4),
             "cfg2 EuRoC V1_02-shaped stereo 752x480 images, 11 clones, <=200 MSCKF + 50 SLAM"),
    # cfg2 with real track loss: 400 stereo tracks over a scene whose texture panels each redraw every 8 frames
    # at their own phase (render.py churn), so a track lives a few frames and is lost with several observations
    # (round 4's churn 3 lost most tracks after 2 observations: 1.3 rows per feature)
    "cfg2l": ("euroc_mav", "images",
              dict(init_max_features=800, max_msckf_in_update=200, max_slam_features=50, max_slam_in_update=25,
                   dt_slam_delay=1.0),
              dict(spawn=4, churn=8),
              "cfg2l EuRoC V1_02-shaped stereo 752x480 images with track loss (scene churn 1/8 per frame), 400 "
              "tracks, 11 clones, <=200 MSCKF + 50 SLAM"),
    "cfg3": ("tum_vi", "images",
             dict(max_clone_size=20, init_max_features=800, num_pts=400, max_msckf_in_update=400,
                  max_slam_features=50, max_slam_in_update=25, dt_slam_delay=1.0),
             dict(spawn=4),
             "cfg3 TUM-VI room1-shaped stereo fisheye 512x512 images, 20 clones, 400 tracks/cam, <=400 MSCKF + 50 SLAM"),
    # cfg3 at BASELINE's MSCKF load (the N = 1 line's "msckf_load" companion): the TUM-VI stereo rig and window
    # of cfg3 with a TrackSIM feed whose every update holds 400 MSCKF features seen in every clone by both
    # cameras (up to 400 x 81 = 32,400 stacked rows), so the MFMA paths (tiled T GEMM,
    # MFMA Gram, information-form factors) run every frame
    "cfg3t": ("tum_vi", "tracks",
              dict(max_clone_size=20, max_msckf_in_update=400, max_slam_features=50, max_slam_in_update=25,
                   dt_slam_delay=1.0),
              dict(spawn=400, frac_lost=0.0, frac_long=0.02),
              "cfg3t TUM-VI room1-shaped stereo fisheye 512x512 tracks, 20 clones, 400 MSCKF feats x 42 meas + 50 SLAM"),
    # the backend stress at the BASELINE feature counts: every MSCKF update holds 800 / 1500 features seen in
    # every clone (TrackSIM feed); the feature-sharded multi-GPU lines run these
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
    "cfg4i": ("uzhfpv_outdoor_45", "images",
              dict(max_clone_size=25, init_max_features=800, num_pts=400, max_msckf_in_update=800, max_slam_features=50,
                   max_slam_in_update=25, dt_slam_delay=1.0),
              dict(spawn=4),
              "cfg4i UZH-FPV outdoor_45-shaped stereo fisheye 640x480 images, 25 clones, 800 tracks (400/cam), "
              "<=800 MSCKF + 50 SLAM"),
    "cfg5i": ("rpng_sim_uwb", "images",
              dict(max_clone_size=30, init_max_features=1500, num_pts=375, max_msckf_in_update=1500,
                   max_slam_features=50, max_slam_in_update=25, dt_slam_delay=1.0),
              dict(spawn=4, uwb=True),
              "cfg5i rpng_sim 4-cam 752x480 images (each camera tracked on its own) + 6 UWB anchors (2 fixed), IMU "
              "intrinsics, 30 clones, 1500 tracks (375/cam), <=1500 MSCKF + 50 SLAM"),
}

# names of rounds 1-3 (the TrackSIM stress lines were cfg4t / cfg5t)
ALIASES = {"cfg4t": "cfg4", "cfg5t": "cfg5"}
# oracle frames in the cpu_baseline sample (~10-30 s of CPU work per workload)
CPU_CV_THREADS = 4  # num_opencv_threads of every reference config
CPU_FRAMES = {"cfg1": 150, "cfg2": 120, "cfg2l": 60, "cfg3": 60, "cfg4i": 20, "cfg5i": 10, "cfg3t": 6, "cfg4": 3,
              "cfg5": 2}
# shader clock for cycle counts (MI355X peak engine clock, MI355X_MICROARCH.md) and the CU count
SCLK_HZ = 2.4e9
N_CU = 256
SIMD_PER_CU = 4


def _kv(items):
    out = {}
    for it in items:
        k, v = it.split("=", 1)
        try:
            out[k] = json.loads(v)
        except ValueError:
            out[k] = v
    return out


def workload_options(U, name, extra=None):
    """the workload's options; extra: further overrides (ablations), "anchors_fix" = 0/1 sets every UWB anchor's
    fix flag (uwb_anchors.yaml "fix")"""
    cfg, _, ov, _, _ = WORKLOADS[name]
    ov = dict(ov, **(extra or {}))
    fix = ov.pop("anchors_fix", None)
    opts = U.load_options(os.path.join(CONFIGS, cfg, "estimator_config.yaml"), record_timing=1, **ov)
    if fix is not None:
        for i in range(opts.n_anchors):
            opts.anchors[i].fix = int(fix)
    return opts


def cfg2_options(U):
    return workload_options(U, "cfg2")


def make_stream(opts, n_frames, seed, workload="cfg2", extra=None):
    from uvio_amd.sim import SimStream
    kw = dict(WORKLOADS[workload][3], **(extra or {}))
    anchors = None
    if kw.pop("uwb", False):
        anchors = [opts.anchors[i] for i in range(opts.n_anchors)]
    churn = kw.pop("churn", 0)
    # image workloads: the simulated tracks are not used (the images are); keep their generation small
    sim = SimStream(opts, duration=n_frames / opts.track_frequency + 1.0, seed=seed, anchors=anchors, **kw)
    sim.churn = churn  # scene churn of the rendered images (render.py)
    return sim


class Frames:
    """Camera images of the stream's frames as u8 CUDA tensors, rendered on first use and kept resident."""

    def __init__(self, sim, device):
        import torch
        from uvio_amd.render import SceneRenderer
        self.sim, self.device, self.torch = sim, device, torch
        self.r = SceneRenderer(sim.opts, device=device, churn=getattr(sim, "churn", 0))
        self.cache = {}

    def __getitem__(self, i):
        if i not in self.cache:
            self.cache[i] = [self.r.render(k, *self.sim.camera_pose(i, k), frame_seed=i) for k in range(self.sim.K)]
        return self.cache[i]

    def prerender(self, lo, hi):
        for i in range(lo, min(hi, len(self.sim.cam_t))):
            self[i]
        self.torch.cuda.synchronize(self.device)


class Driver:
    """Feeds one stream into one manager frame by frame (events precomputed).  frames: per camera frame
    the list of device images (feed_measurement_camera_device) or of host arrays (feed_measurement_camera);
    None: the stream's simulated tracks (TrackSIM feed), packed per frame beforehand."""

    def __init__(self, sim, mgr, frames, device_imgs=True):
        self.sim, self.mgr, self.frames, self.device_imgs = sim, mgr, frames, device_imgs
        if frames is None:
            from uvio_amd.manager import pack_sim_frame
            self.packed = [pack_sim_frame(f) for f in sim.frames]
        self.ev = [e for e in sim.events() if e[1] >= sim.t0 - 0.4]
        # runs of consecutive IMU events go in as one feed_measurement_imu_batch call (index of the run's
        # first event -> (t, wm, am) arrays, events in the run)
        self.imu_runs = {}
        k = 0
        while k < len(self.ev):
            j = k
            while j < len(self.ev) and self.ev[j][0] == "imu":
                j += 1
            if j > k:
                idx = [self.ev[q][2] for q in range(k, j)]
                self.imu_runs[k] = (np.array([self.ev[q][1] for q in range(k, j)]), np.ascontiguousarray(sim.wm[idx]),
                                    np.ascontiguousarray(sim.am[idx]), j - k)
            k = max(j, k + 1)
        self.k = 0
        self.frame = -1  # index of the last fed camera frame
        mgr.initialize_with_gt(sim.gt_state(sim.t0))

    def next_frame(self):
        """index of the camera frame the next step() feeds"""
        k = self.k
        while True:
            kind, t, i = self.ev[k]
            k += 1
            if kind == "cam" and t > self.sim.t0:
                return i

    def step(self):
        """Feed events up to and including the next camera frame; returns its timestamp."""
        sim, mgr = self.sim, self.mgr
        while True:
            run = self.imu_runs.get(self.k)
            if run is not None:
                mgr.feed_measurement_imu_batch(run[0], run[1], run[2])
                self.k += run[3]
                continue
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
                self.frame = i
                return t


# committed rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE / FP64 MFMA, tools/pmc_summary.py), newest first.  The
# workload names cfg4 / cfg5 changed meaning in r04 (TrackSIM stress, before: images), so only r04+ passes count
# for them and for their image variants
PMC_MIN_TAG = {"cfg4": "r04", "cfg5": "r04", "cfg4i": "r04", "cfg5i": "r04"}


def pmc_files(workload):
    names = sorted((f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc_traffic_%s.json" % workload)
                    and f >= PMC_MIN_TAG.get(workload, "")), reverse=True)
    return [os.path.join("profiles", f) for f in names]


# the kernels one timed "launch" of a class (one HIP-event pair around a launch chain, kprof.h) contains exactly
# once: their PMC launch count is the class's group count
CLASS_GROUP_KERNELS = {"feature": ["k_feature"], "chi2": ["k_chi2"], "gram": ["k_gram", "k_gram_mfma"],
                       "ekf_update": ["k_ekf_fact", "k_info_P"], "ldl": ["k_ekf_fact"], "lk": ["k_lk"],
                       "pyramid": ["k_hist_multi"], "fast": ["k_fast_score"], "subpix": ["k_subpix"]}


def pmc_class_traffic(workload, name, kernels):
    """(HBM bytes per launch group of the kernel class, MFMA busy cycles per launch group or None, source file)
    from the newest PMC summary holding it: the members' summed counters over the number of groups
    (CLASS_GROUP_KERNELS)."""
    for path in pmc_files(workload):
        try:
            with open(os.path.join(ROOT, path)) as f:
                k = json.load(f)["kernels"]
        except (OSError, KeyError, ValueError):
            continue
        hit = [n for n in kernels if n in k]
        groups = sum(k[n]["launches"] for n in CLASS_GROUP_KERNELS.get(name, kernels[:1]) if n in k)
        if not hit or groups == 0:
            continue
        tot = sum(k[n]["traffic"] * k[n]["launches"] for n in hit)
        busy = None
        if any("mfma_busy_cycles" in k[n] for n in hit):
            busy = sum(k[n].get("mfma_busy_cycles", 0.0) * k[n]["launches"] for n in hit) / groups
        return tot / groups, busy, path
    return None, None, None


def library_sha16():
    """sha256 (16 hex) of the product library this process loads (the build tools/prof_summary.py records)."""
    import hashlib
    from uvio_amd import _native as N
    try:
        return hashlib.sha256(open(N.LIB_PATH, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def committed_class_times(workload, classes):
    """Per-class device time per frame (us) from the newest committed rocprofv3 per-frame summary of this workload
    made with THIS library build (profiles/rNN*_<workload>_per_frame.txt, tools/prof_summary.py over a kernel trace
    of the same bench command; its 'library sha256' line must equal the loaded library's), summed over the class's
    kernels; ({class: us}, path, why) or ({}, None, why).  rocprof's device timestamps rank the classes without the
    dispatch gap that the live HIP-event pairs include (the event before a launch completes when the previous kernel
    does, so each timed launch also carries its ~5 us dispatch gap).  A summary of another build, or one whose
    format does not parse, is skipped and `why` says so (the caller then ranks by the live timing)."""
    d = os.path.join(ROOT, "profiles")
    names = sorted((f for f in os.listdir(d) if f.endswith("_%s_per_frame.txt" % workload) and f >= "r05"),
                   reverse=True)
    sha = library_sha16()
    why = "no committed per-frame summary of %s" % workload
    for f in names:
        per, fsha = {}, None
        try:
            with open(os.path.join(d, f)) as fh:
                for line in fh:
                    if line.startswith("library sha256 "):
                        fsha = line.split()[2]
                        continue
                    if "n/frame" not in line or "per frame" not in line:
                        continue
                    head, rest = line.split("n/frame", 1)
                    kname = head.strip().split("<")[0]
                    us = float(rest.split("per frame")[1].split("us")[0])
                    per[kname] = per.get(kname, 0.0) + us
        except (OSError, ValueError, IndexError):
            why = "profiles/%s does not parse" % f
            continue
        if fsha is None or fsha != sha:
            if not why.startswith("newest"):
                why = "newest summary profiles/%s is of another build (%s, loaded %s)" % (f, fsha, sha)
            continue
        if per:
            return ({c: sum(per.get(k, 0.0) for k in ks) for c, ks in classes.items()}, os.path.join("profiles", f),
                    "same build (library sha256 %s)" % sha)
    return {}, None, why


def max_over_ranks(x, device="cuda"):
    """Whole-job wall time: the slowest rank's (one all-reduce, outside the timed region)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_true(flag, device="cuda"):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return flag
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def spawn_workers(n, argv, script=None):
    """--gpus N without a launcher: N worker processes (one per GPU) started before this process touches the
    GPU; rank 0's JSON line is passed through, the exit code is the worst of the workers'."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].communicate()[0]
    rcs = [p.wait() for p in procs]
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def roofline_entry(name, st, wl):
    bound = st["bound"]
    secs = st["seconds"]
    n = max(st["launches"], 1)
    avg = secs / n
    if bound == "mfma":
        per = st["flops"] / n
        achieved = per / avg / 1e12 if avg > 0 else 0.0
        peak, unit = FP64_PEAK_TFLOPS, "TFLOP/s"
    else:
        per = st["bytes"] / n
        achieved = per / avg / 1e9 if avg > 0 else 0.0
        peak, unit = HBM_PEAK_GBS, "GB/s"
    traffic, busy, src = pmc_class_traffic(wl, name, st["kernels"])
    e = {"kernel": name, "kernels": st["kernels"], "bound": bound, "achieved": achieved, "peak": peak, "unit": unit,
         "frac": achieved / peak, "traffic": traffic, "traffic_source": src, "launches": st["launches"],
         "avg_launch_us": avg * 1e6, ("flops_per_launch" if bound == "mfma" else "bytes_per_launch"): per,
         "device_s": secs}
    if bound == "mfma":
        # SQ_VALU_MFMA_BUSY_CYCLES is summed over the SIMDs (k_gram_mfma: 509.6 MFLOP / 2048 FLOP per
        # v_mfma_f64_16x16x4f64 x 64 cycles = the counter's value), so per launch group it is divided by the chip's
        # SIMD cycles in this run's average launch time: the whole-chip MFMA utilisation of the class
        e["mfma_busy_cycles_per_launch"] = busy
        e["mfma_util"] = busy / (avg * SCLK_HZ * N_CU * SIMD_PER_CU) if (busy is not None and avg > 0) else None
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=40, help="minimum warm-up frames (then until steady state)")
    ap.add_argument("--max-warmup", type=int, default=200, help="warm-up cap while waiting for steady state")
    ap.add_argument("--cpu-frames", type=int, default=None,
                    help="timed oracle frames for cpu_baseline (0 = skip; default: ~10-30 s of CPU work per workload)")
    ap.add_argument("--workload", choices=["auto"] + sorted(WORKLOADS) + sorted(ALIASES), default="auto",
                    help="auto: cfg3 at 1 GPU, feature-sharded cfg4 at 2-4 GPUs, cfg5 beyond")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="override an estimator option of the workload (ablations; the line records it)")
    ap.add_argument("--sim", action="append", default=[], metavar="KEY=VALUE",
                    help="override a SimStream argument of the workload (ablations; the line records it)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N > 1 on fewer GPUs (tests only): ranks share the visible GPUs, torch.distributed over gloo "
                         "and the sharded update's all-reduce through the host callback instead of RCCL")
    ap.add_argument("--no-host-feed", action="store_true",
                    help="skip the second timed pass that feeds the frames as host images (uvio_hp_feed_camera)")
    ap.add_argument("--replicas", action="store_true", help="(the N > 1 default) one independent estimator per GPU")
    ap.add_argument("--shard", action="store_true",
                    help="value = the feature-sharded run of --workload (every rank one stream, MSCKF updates split; "
                         "also at N = 1 as an RCCL world of 1)")
    ap.add_argument("--sharded-steps", type=int, default=100,
                    help="N > 1: timed frames of the feature-sharded companion run (0 = skip)")
    ap.add_argument("--shard-min", type=int, default=64, help="smallest MSCKF update that is sharded")
    ap.add_argument("--msckf-load-steps", type=int, default=60,
                    help="N = 1 cfg3 line: timed frames of the cfg3t companion at BASELINE's MSCKF load (0 = skip)")
    ap.add_argument("--ktime-period", type=int, default=None,
                    help="kernel-class event timing on every k-th frame of the timed region (0 = off; default: every "
                         "frame for --steps <= 50, else every 10th)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if args.gpus > 1:
            return spawn_workers(args.gpus, sys.argv[1:])
        world = 1
    if args.gpus != world:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # N > 1: value = one independent cfg3 estimator per GPU (weak scaling: the same per-rank work as the N = 1
    # line); the north star's feature-sharded update (cfg4 at N <= 4, cfg5 beyond) is measured in the same job as
    # the line's "feature_sharded" object, with its 1-GPU time on the same stream
    shard = args.shard
    wl = ALIASES.get(args.workload, args.workload)
    if wl == "auto":
        wl = ("cfg4" if world <= 4 else "cfg5") if (shard and world > 1) else "cfg3"
    if args.cpu_frames is None:
        args.cpu_frames = CPU_FRAMES[wl]
    if args.ktime_period is None:
        args.ktime_period = 1 if args.steps <= 50 else 10
    # stdout carries exactly the one JSON line: whatever the libraries print (RCCL's version banner at
    # communicator creation, ...) goes to stderr
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    if world > 1:
        if args.rehearse:
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import uvio_amd as U
    from uvio_amd.evaluation import ate as ate_fn

    images = WORKLOADS[wl][1] == "images"
    opt_set, sim_set = _kv(args.set), _kv(args.sim)
    opts = workload_options(U, wl, opt_set)
    max_warm = max(args.warmup, args.max_warmup)
    n_frames = max_warm + args.steps + 2
    # replicas: one stream per rank; sharded: every rank runs the same stream and splits its MSCKF updates
    sim = make_stream(opts, n_frames + 2, seed=5 if shard else 5 + rank, workload=wl, extra=sim_set)
    dev = torch.device("cuda", local)
    frames = Frames(sim, dev) if images else None
    if frames is not None:
        frames.prerender(0, args.warmup + 2)
    mgr = U.VioManager(opts, device=local)
    if shard:
        from uvio_amd.manager import shard_unique_id
        uid = [shard_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        if args.rehearse:
            mgr.enable_feature_sharding(rank, world, backend="host", min_features=args.shard_min)
        else:
            mgr.enable_feature_sharding(rank, world, backend="rccl", unique_id=uid[0], min_features=args.shard_min)
    drv = Driver(sim, mgr, frames)

    # warm-up: at least --warmup frames, then until the clone window is full and the SLAM slots are populated
    want_slam = int(0.9 * opts.max_slam_features)
    warm, steady = 0, False
    while True:
        drv.step()
        warm += 1
        tm = mgr.get_timing()
        ok = tm["n_clones"] >= opts.max_clone_size + 1 and tm["n_slam"] >= want_slam
        if warm >= args.warmup:
            steady = all_ranks_true(ok, dev)
            if steady or warm >= max_warm:
                break
    if frames is not None:
        nxt = drv.next_frame()
        frames.prerender(nxt, nxt + args.steps + 1)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    acc = {"rows": 0, "n_msckf": 0, "n_slam": 0, "cols": 0, "cov_dim": 0, "tracking_s": 0.0, "syncs": 0,
           "sync_wait": 0.0}
    stages = ("propagation", "msckf_update", "slam_update", "slam_delayed", "marg", "total", "chain_wait")
    stage_s = dict.fromkeys(stages, 0.0)
    est_p, est_q, gt_p, gt_q = [], [], [], []
    mgr.set_kernel_timing(args.ktime_period)
    ks0 = mgr.kernel_stats(flush=True)
    # a torch kernel marks the start of the timed region in kernel traces (tools/prof_summary.py and
    # tools/gap_summary.py count from the last torch kernel), so TrackSIM workloads' warm-up stays out too
    torch.ones(1, device=dev).add_(1)
    barrier()
    # inside the timed loop only what a driver of the library does per frame: the feed and the state / timing
    # read-out; the ground truth and the statistics are computed afterwards
    rec = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t = drv.step()
        rec.append((t, mgr.get_timing_raw(), mgr.get_imu_state()[1]))
    barrier()
    t1 = time.perf_counter()
    for t, tmr, x in rec:
        tm = tmr.as_dict()
        acc["rows"] += tm["msckf_rows"]
        acc["n_msckf"] += tm["n_msckf"]
        acc["n_slam"] += tm["n_slam"]
        acc["cols"] = max(acc["cols"], tm["msckf_cols"])
        acc["cov_dim"] = max(acc["cov_dim"], tm["cov_dim"])
        acc["tracking_s"] += tm["tracking"]
        acc["syncs"] += tm["device_syncs"]
        acc["sync_wait"] += tm["sync_wait"]
        for k in stages:
            stage_s[k] += tm[k]
        est_q.append(x[0:4].copy())
        est_p.append(x[4:7].copy())
        g = sim.gt_state(t)
        gt_q.append(g[1:5])
        gt_p.append(g[5:8])
    elapsed = max_over_ranks(t1 - t0)
    ks1 = mgr.kernel_stats(flush=True)
    acc_ate = ate_fn(est_p, gt_p, est_q, gt_q, align="posyaw")
    raw = ate_fn(est_p, gt_p, align="none")
    ntr = sum(len(mgr.get_tracks(c)[0]) for c in range(opts.num_cameras)) if images else None
    host_feed = None
    if frames is not None and world == 1 and not args.no_host_feed:
        mgr.close()
        host_feed = host_feed_pass(U, opts, sim, frames, warm, args.steps, barrier, x_ref=[r[2] for r in rec])
    msckf_load = None
    if world == 1 and wl == "cfg3" and not shard and args.msckf_load_steps > 0:
        mgr.close()
        msckf_load = msckf_load_companion(U, args, dev)
    sharded = None
    if world > 1 and not shard and args.sharded_steps > 0:
        mgr.close()
        frames = None
        sharded = sharded_companion(U, args, world, rank, dev, barrier)

    if rank == 0:
        # replicas: world streams were processed; sharded: one stream, split
        value = (1 if shard else world) * args.steps / elapsed
        ks = {}
        for k, a in ks1.items():
            b = ks0[k]
            ks[k] = dict(a, launches=a["launches"] - b["launches"], seconds=a["seconds"] - b["seconds"],
                         flops=a["flops"] - b["flops"], bytes=a["bytes"] - b["bytes"])
        rl = {k: roofline_entry(k, v, wl) for k, v in ks.items() if v["launches"] > 0}
        # the dominant kernel class (the EKF-update chain aggregate is excluded: it contains the LDL class and
        # several latency-bound kernels): by device time in the committed same-code rocprof summary of this
        # workload when there is one, else by this run's live HIP-event time
        cand = {k: v for k, v in rl.items() if k != "ekf_update"}
        prof_t, prof_src, prof_why = committed_class_times(wl, {k: v["kernels"] for k, v in cand.items()})
        if prof_t:
            dom = max(cand, key=lambda k: prof_t.get(k, 0.0))
            dom_by = {"source": prof_src, "why": prof_why,
                      "device_us_per_frame": {k: round(v, 1) for k, v in prof_t.items()}}
        else:
            dom = max(cand, key=lambda k: cand[k]["device_s"]) if cand else None
            dom_by = {"source": "live HIP-event time of this run", "why": prof_why}
        cpu = None
        if args.cpu_frames > 0:
            # the oracle needs only the clone window filled; fewer warm-up frames bound its run time
            cpu_warm = warm if images else min(warm, int(opts.max_clone_size) + 3)
            cpu = cpu_baseline(opts, wl, cpu_warm, args.cpu_frames, frames, sim_set)
        out = {
            "metric": "VIO frames/sec (track+propagate+update) at clones x feats",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": warm,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if shard else "weak",
            "value_definition": ("feature-sharded: every rank runs the same stream, each MSCKF update split across the "
                                 "ranks (one RCCL all-reduce); value = frames of that one stream / wall time") if shard
                                else ("one independent estimator per GPU on its own stream (the N = 1 workload, seed 5 + "
                                      "rank), value = all ranks' frames / the slowest rank's wall time; the north star's "
                                      "feature-sharded update at N > 1 is the feature_sharded object"),
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic %s-shaped stream (uvio_amd/sim.py, seed %s) with ray-cast images "
                     "(uvio_amd/render.py) resident in HBM, TrackKLT front-end" %
                     (WORKLOADS[wl][0], "5" if shard else "5+rank")) if images else
                    ("synthetic %s-shaped stream (uvio_amd/sim.py, seed %s): simulated feature tracks "
                     "(TrackSIM feed, VioManager::feed_measurement_simulation)%s" %
                     (WORKLOADS[wl][0], "5" if shard else "5+rank", " + UWB ranges" if opts.use_uwb else "")),
            "config": {"workload": WORKLOADS[wl][4],
                       "steady": steady, "warmup_requested": args.warmup,
                       "track_features_per_cam": int(opts.init_max_features) // int(opts.num_cameras) if images else None,
                       "tracks_last_frame": ntr, "mean_tracking_ms": 1e3 * acc["tracking_s"] / args.steps,
                       "clones": int(opts.max_clone_size), "cameras": int(opts.num_cameras),
                       "max_msckf_in_update": int(opts.max_msckf_in_update),
                       "max_slam_features": int(opts.max_slam_features),
                       "mean_msckf_feats": acc["n_msckf"] / args.steps, "mean_slam_feats": acc["n_slam"] / args.steps,
                       "mean_msckf_rows": acc["rows"] / args.steps, "H_cols": acc["cols"],
                       "state_dim": acc["cov_dim"], "host_waits_per_frame": acc["syncs"] / args.steps,
                       "host_wait_ms_per_frame": 1e3 * acc["sync_wait"] / args.steps,
                       "stage_ms": {k: round(1e3 * v / args.steps, 4) for k, v in stage_s.items()},
                       "parallelism": ("feature-shard%d" % world) if shard else ("replicas%d" % world),
                       "overrides": {"options": opt_set, "sim": sim_set} if (opt_set or sim_set) else None},
            "ate_rmse_m": acc_ate["pos_m"],
            "ate": {"align": "posyaw (ov_eval AlignTrajectory.cpp:84-106)", "pos_rmse_m": acc_ate["pos_m"],
                    "ori_rmse_deg": acc_ate["ori_deg"], "unaligned_pos_rmse_m": raw["pos_m"],
                    "frames": args.steps,
                    "note": (None if args.steps >= 100 else
                             "fewer than 100 frames: the posyaw alignment absorbs the drift of so short a segment, "
                             "the number says nothing about accuracy (the 300-frame default line is the accuracy check)")},
            "roofline": rl.get(dom),
            "roofline_selected_by": dom_by,
            "rooflines": rl,
            "host_feed": host_feed,
            "feature_sharded": sharded,
            "msckf_load": msckf_load,
            "cpu_baseline": cpu,
        }
        result_out.write(json.dumps(out) + "\n")
        result_out.flush()
    if world > 1:
        dist.destroy_process_group()
    return 0


def msckf_load_companion(U, args, dev):
    """cfg3 at BASELINE's MSCKF load (workload cfg3t): the same rig, window and limits as the cfg3 line, fed
    TrackSIM tracks so that every update holds 400 MSCKF features seen in all 21 clones by both cameras.  Its own
    frame rate, per-class rooflines (live HIP-event timing) and dominant class, as the main line reports them."""
    import torch
    wl = "cfg3t"
    opts = workload_options(U, wl)
    warm = int(opts.max_clone_size) + 4
    steps = args.msckf_load_steps
    sim = make_stream(opts, warm + steps + 4, seed=5, workload=wl)
    mgr = U.VioManager(opts, device=dev.index)
    drv = Driver(sim, mgr, None)
    for _ in range(warm):
        drv.step()
    mgr.set_kernel_timing(1 if steps <= 50 else 5)
    ks0 = mgr.kernel_stats(flush=True)
    torch.cuda.synchronize()
    acc = {"n_msckf": 0, "rows": 0, "cols": 0}
    stages = ("tracking", "propagation", "msckf_update", "slam_update", "slam_delayed", "marg", "chain_wait")
    st = dict.fromkeys(stages, 0.0)
    rec = []
    t0 = time.perf_counter()
    for _ in range(steps):
        drv.step()
        rec.append(mgr.get_timing_raw())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ks1 = mgr.kernel_stats(flush=True)
    mgr.close()
    for r in rec:
        tm = r.as_dict()
        acc["n_msckf"] += tm["n_msckf"]
        acc["rows"] += tm["msckf_rows"]
        acc["cols"] = max(acc["cols"], tm["msckf_cols"])
        for k in stages:
            st[k] += tm[k]
    rl = {}
    for k, a in ks1.items():
        b = ks0[k]
        d = dict(a, launches=a["launches"] - b["launches"], seconds=a["seconds"] - b["seconds"],
                 flops=a["flops"] - b["flops"], bytes=a["bytes"] - b["bytes"])
        if d["launches"] > 0:
            rl[k] = roofline_entry(k, d, wl)
    cand = {k: v for k, v in rl.items() if k != "ekf_update"}
    prof_t, prof_src, prof_why = committed_class_times(wl, {k: v["kernels"] for k, v in cand.items()})
    if prof_t:
        dom = max(cand, key=lambda k: prof_t.get(k, 0.0))
        dom_by = {"source": prof_src, "why": prof_why, "device_us_per_frame": {k: round(v, 1) for k, v in prof_t.items()}}
    else:
        dom = max(cand, key=lambda k: cand[k]["device_s"]) if cand else None
        dom_by = {"source": "live HIP-event time of this run", "why": prof_why}
    return {"workload": WORKLOADS[wl][4], "steps": steps, "warmup": warm, "value": steps / el, "unit": "frames/s",
            "ms_per_step": 1e3 * el / steps, "mean_msckf_feats": acc["n_msckf"] / steps,
            "mean_msckf_rows": acc["rows"] / steps, "H_cols": acc["cols"],
            "stage_ms": {k: round(1e3 * v / steps, 4) for k, v in st.items()},
            "roofline": rl.get(dom), "roofline_selected_by": dom_by, "rooflines": rl,
            "note": "TrackSIM feed (VioManager::feed_measurement_simulation) of a cfg3-shaped stream: every MSCKF update "
                    "at BASELINE's 400 features; the line's value is the image-fed cfg3 run"}


def sharded_companion(U, args, world, rank, dev, barrier):
    """The feature-sharded MSCKF update at this world size: every rank runs the same BASELINE
    stream (cfg4 at N <= 4, cfg5 beyond) and splits each update's features (one RCCL all-reduce per update);
    then rank 0 alone runs the same stream unsharded on its GPU (the other ranks wait), for the speedup."""
    import torch
    import torch.distributed as dist
    from uvio_amd.manager import shard_unique_id
    wl = "cfg4" if world <= 4 else "cfg5"
    opts = workload_options(U, wl)
    warm = int(opts.max_clone_size) + 4
    steps = args.sharded_steps
    sim = make_stream(opts, warm + steps + 4, seed=5, workload=wl)

    def run(mgr, sync):
        drv = Driver(sim, mgr, None)
        for _ in range(warm):
            drv.step()
        sync()
        t0 = time.perf_counter()
        n_msckf = 0
        for _ in range(steps):
            drv.step()
            n_msckf += mgr.get_timing_raw().n_msckf
        sync()
        return time.perf_counter() - t0, n_msckf / steps, mgr.get_imu_state()[1]

    mgr = U.VioManager(opts, device=dev.index)
    if args.rehearse:
        mgr.enable_feature_sharding(rank, world, backend="host", min_features=args.shard_min)
    else:
        uid = [shard_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        mgr.enable_feature_sharding(rank, world, backend="rccl", unique_id=uid[0], min_features=args.shard_min)
    el, nm, x_sh = run(mgr, barrier)
    el = max_over_ranks(el)
    mgr.close()
    out = None
    if rank == 0:
        m1 = U.VioManager(opts, device=dev.index)
        el1, _, x_1 = run(m1, lambda: torch.cuda.synchronize())
        m1.close()
        out = {"workload": WORKLOADS[wl][4], "scaling": "strong", "n_gpus": world, "steps": steps, "warmup": warm,
               "value": steps / el, "unit": "frames/s", "ms_per_step": 1e3 * el / steps,
               "single_gpu_value": steps / el1, "speedup": el1 / el, "mean_msckf_feats": nm,
               "final_imu_state_max_abs_diff_vs_single": float(np.max(np.abs(x_sh - x_1))),
               "note": "every rank runs the same stream; each MSCKF update's feature linearization, chi2 gate and "
                       "Gram are split over the ranks with one RCCL all-reduce (SURVEY.md §8e); single_gpu_value: "
                       "rank 0 alone, unsharded, same stream, same job"}
    dist.barrier()
    return out


def host_feed_pass(U, opts, sim, frames, warm, steps, barrier, x_ref):
    """The same frames once more, fed as host u8 images through uvio_hp_feed_camera (the reference caller's
    form, SURVEY.md §8b: the library uploads each image) into a fresh estimator: the PCIe-inclusive frame rate.
    The host copies of the images are made before the timed region; the estimate must equal the device-feed
    run's (same inputs, same library)."""
    host = {i: [im.cpu().numpy() for im in v] for i, v in frames.cache.items()}
    mgr = U.VioManager(opts, device=0)
    drv = Driver(sim, mgr, host, device_imgs=False)
    for _ in range(warm):
        drv.step()
    xs = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        drv.step()
        xs.append(mgr.get_imu_state()[1])
    barrier()
    t1 = time.perf_counter()
    mgr.close()
    same = all(np.array_equal(a, b) for a, b in zip(xs, x_ref))
    img_bytes = sum(im.nbytes for im in host[next(iter(host))])
    return {"value": steps / (t1 - t0), "unit": "frames/s", "ms_per_step": 1e3 * (t1 - t0) / steps,
            "bytes_uploaded_per_frame": img_bytes, "estimate_equal_to_device_feed": same,
            "note": "uvio_hp_feed_camera with pageable host images, same frames and warm-up as value's run"}


def cpu_baseline(opts, wl, warmup, frames, dev_frames, sim_set=None):
    """oracle/ (the CPU restatement) on the same stream (rank 0's), one thread, bounded sample."""
    from oracle import oracle as O
    # the reference's configs run OpenCV on num_opencv_threads = 4 (config/*/estimator_config.yaml:87-89): the
    # oracle's restated parallel OpenCV calls (LK per point, pyrDown / Scharr per row) use as many; the estimator
    # itself is single-threaded in the reference
    threads = O.set_threads(CPU_CV_THREADS)
    sim = make_stream(opts, warmup + frames + 2, seed=5, workload=wl, extra=sim_set)
    host = None
    if dev_frames is not None:
        host = {}
        for i in range(warmup + frames + 2):
            host[i] = [im.cpu().numpy() for im in dev_frames[i]]
    mgr = O.OracleManager(opts)
    drv = Driver(sim, mgr, host, device_imgs=False)
    for _ in range(warmup):
        drv.step()
    t0 = time.perf_counter()
    for _ in range(frames):
        drv.step()
    dt = time.perf_counter() - t0
    O.set_threads(1)
    return {"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
            "sample": "%d frames of the %s %s stream after %d warm-up frames, oracle/liboracle.so (g++ -O3): the "
                      "tracker's OpenCV-parallel calls on %d threads (num_opencv_threads), the estimator on one (as "
                      "the reference)" % (frames, wl, "image" if dev_frames is not None else "track", warmup, threads)}


if __name__ == "__main__":
    sys.exit(main())
