"""The ROS-free serial runner (uvio_amd/uvio_run_asl, csrc/run_asl.cpp; the reference's
ov_msckf/src/ros1_serial_msckf.cpp:127-275 with an ASL folder instead of a rosbag) on a synthetic EuRoC-format
folder generated here: IMU CSV, two cameras' PNG images rendered from the textured room, ASL ground truth.

CPU: the runner parses the folder and decodes every PNG (--dry-run) -- message counts, stereo pairing and the
pixel sum of the decoded images equal what was written.
GPU: the runner's trajectory (ov_eval format, ground-truth initialized) equals, bit for bit, the estimate of the
same messages fed through the Python binding in the same order (host images, uvio_hp_feed_camera), and agrees
with the oracle (the CPU restatement, tracker included) fed the same messages in the same order: a free run of
the whole serial loop, poses within 1e-5 m / rad on every frame (ros1_serial_msckf.cpp:160-275)."""
import json
import os
import re
import struct
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")
RUNNER = os.path.join(ROOT, "uvio_amd", "uvio_run_asl")
N_FRAMES = 30


def write_png(path, img):
    """8-bit grayscale PNG, every scanline with filter 0 except a few with filter 1 / 2 (exercises the decoder)"""
    h, w = img.shape
    rows = []
    for y in range(h):
        r = img[y].astype(np.int16)
        ft = y % 3
        if ft == 1:
            d = (r - np.concatenate([[0], r[:-1]])) & 255
        elif ft == 2:
            d = (r - (img[y - 1].astype(np.int16) if y > 0 else 0)) & 255
        else:
            d = r
        rows.append(bytes([ft]) + d.astype(np.uint8).tobytes())

    def chunk(t, data):
        c = t + data
        return struct.pack(">I", len(data)) + c + struct.pack(">I", zlib.crc32(c) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(b"".join(rows), 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def _ns(t):
    return int(round(t * 1e9))


@pytest.fixture(scope="module")
def asl(tmp_path_factory):
    """(folder, ground-truth CSV, opts, sim, written images) of a short EuRoC-shaped stereo stream"""
    import uvio_amd as U
    from uvio_amd.render import SceneRenderer
    from uvio_amd.sim import SimStream
    opts = U.load_options(EUROC, init_max_features=200, max_msckf_in_update=100, max_slam_features=20,
                          max_slam_in_update=10, dt_slam_delay=0.3)
    # the runner reads a config folder: a copy of the EuRoC one with the same values as the binding's options
    base = tmp_path_factory.mktemp("asl")
    cfg = base / "config"
    cfg.mkdir()
    src = os.path.dirname(EUROC)
    for name in os.listdir(src):
        with open(os.path.join(src, name)) as f:
            text = f.read()
        if name == "estimator_config.yaml":
            for key, val in (("init_max_features", 200), ("max_msckf_in_update", 100), ("max_slam", 20),
                             ("max_slam_in_update", 10), ("dt_slam_delay", 0.3)):
                text, n = re.subn(r"(?m)^%s:.*$" % key, "%s: %s" % (key, val), text)
                assert n == 1, key
        with open(cfg / name, "w") as f:
            f.write(text)
    sim = SimStream(opts, duration=N_FRAMES / opts.track_frequency + 1.2, seed=5, spawn=4)
    r = SceneRenderer(opts, device="cpu")
    mav = base / "mav0"
    imgs = {}
    (mav / "imu0").mkdir(parents=True)
    with open(mav / "imu0" / "data.csv", "w") as f:
        f.write("#timestamp [ns],w_RS_S_x [rad s^-1],w_RS_S_y [rad s^-1],w_RS_S_z [rad s^-1],"
                "a_RS_S_x [m s^-2],a_RS_S_y [m s^-2],a_RS_S_z [m s^-2]\n")
        for i, t in enumerate(sim.imu_t):
            if t < sim.t0 - 0.4:
                continue
            f.write("%d,%s\n" % (_ns(t), ",".join(repr(float(v)) for v in np.r_[sim.wm[i], sim.am[i]])))
    for k in range(2):
        d = mav / ("cam%d" % k) / "data"
        d.mkdir(parents=True)
        with open(mav / ("cam%d" % k) / "data.csv", "w") as f:
            f.write("#timestamp [ns],filename\n")
            for i, t in enumerate(sim.cam_t[:N_FRAMES + 1]):
                if t <= sim.t0:
                    continue
                img = np.asarray(r.render(k, *sim.camera_pose(i, k), frame_seed=i)).astype(np.uint8)
                name = "%d.png" % _ns(t)
                write_png(str(d / name), img)
                imgs[(k, i)] = img
                f.write("%d,%s\n" % (_ns(t), name))
    gt = base / "gt.csv"
    with open(gt, "w") as f:
        f.write("#timestamp,p_x,p_y,p_z,q_w,q_x,q_y,q_z,v_x,v_y,v_z,b_w_x,b_w_y,b_w_z,b_a_x,b_a_y,b_a_z\n")
        for t in sim.imu_t:
            g = sim.gt_state(t)  # [t, q_GtoI (JPL xyzw = Hamilton q_ItoG), p, v, bg, ba]
            q = g[1:5]
            row = np.r_[g[5:8], q[3], q[:3], g[8:11], g[11:14], g[14:17]]
            f.write("%d,%s\n" % (_ns(t), ",".join(repr(float(v)) for v in row)))
    return str(base), str(gt), opts, sim, imgs, str(cfg / "estimator_config.yaml")


def _timing_config(cfg, path):
    """a copy of the runner's config that also writes the reference's timing CSV (VioManager.cpp:105-122)"""
    d = os.path.dirname(cfg)
    with open(cfg) as f:
        text = f.read()
    text += "\nrecord_timing_information: true\nrecord_timing_filepath: \"%s\"\n" % path
    out = os.path.join(d, "estimator_config_timing.yaml")
    with open(out, "w") as f:
        f.write(text)
    return out


def test_runner_dry_run_parses_and_decodes(asl):
    from uvio_amd import build
    build.build_runner()
    folder, gt, opts, sim, imgs, cfg = asl
    out = subprocess.check_output([RUNNER, cfg, folder, "--gt", gt, "--dry-run"], timeout=120)
    s = json.loads(out.decode().strip().splitlines()[-1])
    for k, v in s["options"].items():  # the config copy carries the binding's options
        assert v == getattr(opts, k), k
    n_imu = int(np.sum(sim.imu_t >= sim.t0 - 0.4))
    last_cam = max(1e-9 * _ns(sim.cam_t[i]) for (k, i) in imgs)
    assert s["dry_run"] and s["gt_states"] == len(sim.imu_t)
    assert s["frames"] == len(imgs) // 2 and s["images"] == len(imgs) and s["skipped_unsynced"] == 0
    imu_t = np.array([1e-9 * _ns(t) for t in sim.imu_t])
    assert s["imu"] == int(np.sum((sim.imu_t >= sim.t0 - 0.4) & (imu_t <= last_cam))) <= n_imu
    assert s["pixel_sum"] == int(sum(int(im.astype(np.uint64).sum()) for im in imgs.values()))


def test_runner_rejects_a_bad_png(asl, tmp_path):
    from uvio_amd import build
    build.build_runner()
    folder, gt, opts, sim, imgs, cfg = asl
    bad = tmp_path / "x"
    os.makedirs(bad / "mav0" / "imu0")
    for k in range(2):
        os.makedirs(bad / "mav0" / ("cam%d" % k) / "data")
        with open(bad / "mav0" / ("cam%d" % k) / "data.csv", "w") as f:
            f.write("#t,f\n1000000000,a.png\n")
        with open(bad / "mav0" / ("cam%d" % k) / "data" / "a.png", "wb") as f:
            f.write(b"not a png")
    with open(bad / "mav0" / "imu0" / "data.csv", "w") as f:
        f.write("#t\n1000000000,0,0,0,0,0,9.81\n")
    p = subprocess.run([RUNNER, EUROC, str(bad), "--dry-run"], capture_output=True, timeout=60)
    assert p.returncode == 2 and b"not a PNG" in p.stderr


@pytest.mark.gpu
def test_runner_matches_the_binding(asl, tmp_path):
    """the C++ runner and the Python binding, same folder, same order: identical trajectories"""
    import uvio_amd as U
    folder, gt, opts, sim, imgs, cfg = asl
    traj = tmp_path / "traj.txt"
    tcsv = tmp_path / "timing.csv"
    subprocess.check_call([RUNNER, _timing_config(cfg, str(tcsv)), folder, "--gt", gt, "--out", str(traj)], timeout=300)
    est = np.loadtxt(traj, ndmin=2)
    # the timing CSV in the reference's schema: one row per updated frame once the clone window holds 5 clones
    with open(tcsv) as f:
        lines = f.read().strip().splitlines()
    assert lines[0].startswith("# timestamp (sec),tracking,propagation,msckf update,slam update,slam delayed,")
    rows = np.array([[float(v) for v in l.split(",")] for l in lines[1:]])
    assert rows.shape[1] == 8 and len(rows) >= len(est) - 6 and np.all(rows[:, 1:] >= 0)
    assert np.all(np.diff(rows[:, 0]) > 0)
    assert len(est) >= N_FRAMES - 3
    ref = _serial_feed(U.VioManager(opts), folder, gt, sim, imgs)
    assert ref.shape == est.shape
    assert np.array_equal(ref[:, 1:], est[:, 1:]) and np.allclose(ref[:, 0], est[:, 0], atol=1e-9)


def _serial_feed(m, folder, gt, sim, imgs):
    """the runner's message order through a manager's Python surface: IMU rows and camera pairs in time order
    (IMU first at equal times), GT init at the first pair; returns the ov_eval rows [t, p, q] of every frame"""
    imu = np.loadtxt(os.path.join(folder, "mav0", "imu0", "data.csv"), delimiter=",", ndmin=2)
    gts = np.loadtxt(gt, delimiter=",", ndmin=2)
    gt_t = 1e-9 * gts[:, 0]
    cams = sorted({i for (k, i) in imgs})
    ev = [(1e-9 * r[0], 0, r) for r in imu] + [(1e-9 * _ns(sim.cam_t[i]), 1, i) for i in cams]
    ev.sort(key=lambda e: (e[0], e[1]))
    last_cam = max(e[0] for e in ev if e[1] == 1)
    rows = []
    for t, kind, p in ev:
        if t > last_cam:
            break
        if kind == 0:
            m.feed_measurement_imu(t, p[1:4], p[4:7])
            continue
        if not m.initialized():
            j = int(np.argmin(np.abs(gt_t - t)))
            ts = gt_t[j] if abs(gt_t[j] - t) < 0.10 else t
            v = gts[j]
            m.initialize_with_gt(np.r_[ts, v[5:8], v[4], v[1:4], v[8:17]])
        try:  # the runner goes on after E_STATE / E_ORDER (a ground-truth state a little after the frame)
            rc = m.feed_measurement_camera(t, [0, 1], [imgs[(0, p)], imgs[(1, p)]], allow_uninit=True)
        except RuntimeError as e:
            assert "E_ORDER" in str(e), e
            rc = -1
        if m.initialized() and rc == 0:
            ts, x = m.get_imu_state()
            rows.append(np.r_[ts, x[4:7], x[0:4]])
    m.close()
    return np.array(rows)


@pytest.mark.gpu
def test_runner_matches_the_oracle(asl, tmp_path):
    """the C++ runner (HIP path) against the oracle fed the same folder's messages in the same order: same frames,
    poses within 1e-5 m / rad on every frame (a free run of track -> propagate -> update, no state adoption)"""
    from oracle import oracle as O
    folder, gt, opts, sim, imgs, cfg = asl
    traj = tmp_path / "traj.txt"
    subprocess.check_call([RUNNER, cfg, folder, "--gt", gt, "--out", str(traj)], timeout=300)
    est = np.loadtxt(traj, ndmin=2)
    orc = _serial_feed(O.OracleManager(opts), folder, gt, sim, imgs)
    assert orc.shape == est.shape and len(est) >= N_FRAMES - 3
    assert np.allclose(orc[:, 0], est[:, 0], atol=1e-9)
    dp = np.max(np.linalg.norm(orc[:, 1:4] - est[:, 1:4], axis=1))
    # quaternion distance as a small angle (q and -q are the same rotation)
    dots = np.abs(np.sum(orc[:, 4:8] * est[:, 4:8], axis=1))
    dth = float(np.max(2.0 * np.arccos(np.clip(dots, -1.0, 1.0))))
    print("runner vs oracle over %d frames: max |dp| %.2e m, max dtheta %.2e rad" % (len(est), dp, dth))
    assert dp < 1e-5 and dth < 1e-5, (dp, dth)
