"""Synthetic EuRoC/TUM/UZH-shaped input streams (harness, not the measured path).

Follows the pattern of the reference Simulator (ov_msckf/src/sim/Simulator.cpp:35-470) and TrackSIM
(ov_core/src/track/TrackSIM.cpp:30-79): a smooth ground-truth trajectory, IMU readings from its
analytic derivatives plus white noise and bias random walk with the config's noise densities, and
per-camera feature tracks (id, uv) of 3D points projected through each camera model with sigma_pix
pixel noise.  uv_norm is NOT supplied: the library undistorts like TrackSIM does.

Track life cycle knobs reproduce the BASELINE.json update shapes (C clones x F MSCKF features):
each frame spawns ``spawn`` new points in front of camera 0; a point lives ``life`` frames (mostly
max_clones+1, so it reaches the marginalized clone with a full track and enters the MSCKF update as a
"max track"; some shorter ones arrive as "lost" tracks; some longer ones feed SLAM).
"""
import numpy as np

G = 9.81


def skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def rot_2_quat(R):
    """JPL quaternion of R (quat_ops.h:88)."""
    T = np.trace(R)
    q = np.zeros(4)
    if R[0, 0] >= T and R[0, 0] >= R[1, 1] and R[0, 0] >= R[2, 2]:
        q[0] = np.sqrt((1 + 2 * R[0, 0] - T) / 4)
        q[1] = (R[0, 1] + R[1, 0]) / (4 * q[0])
        q[2] = (R[0, 2] + R[2, 0]) / (4 * q[0])
        q[3] = (R[1, 2] - R[2, 1]) / (4 * q[0])
    elif R[1, 1] >= T and R[1, 1] >= R[0, 0] and R[1, 1] >= R[2, 2]:
        q[1] = np.sqrt((1 + 2 * R[1, 1] - T) / 4)
        q[0] = (R[0, 1] + R[1, 0]) / (4 * q[1])
        q[2] = (R[1, 2] + R[2, 1]) / (4 * q[1])
        q[3] = (R[2, 0] - R[0, 2]) / (4 * q[1])
    elif R[2, 2] >= T and R[2, 2] >= R[0, 0] and R[2, 2] >= R[1, 1]:
        q[2] = np.sqrt((1 + 2 * R[2, 2] - T) / 4)
        q[0] = (R[0, 2] + R[2, 0]) / (4 * q[2])
        q[1] = (R[1, 2] + R[2, 1]) / (4 * q[2])
        q[3] = (R[0, 1] - R[1, 0]) / (4 * q[2])
    else:
        q[3] = np.sqrt((1 + T) / 4)
        q[0] = (R[1, 2] - R[2, 1]) / (4 * q[3])
        q[1] = (R[2, 0] - R[0, 2]) / (4 * q[3])
        q[2] = (R[0, 1] - R[1, 0]) / (4 * q[3])
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


def quat_2_rot(q):
    qv = q[:3]
    return (2 * q[3] ** 2 - 1) * np.eye(3) - 2 * q[3] * skew(qv) + 2 * np.outer(qv, qv)


class Trajectory:
    """Seeded smooth SE(3): sum of sinusoids in a ~10 x 10 x 3 m room, +-30 deg/s rotations.

    static_until: the platform rests until this time and then starts moving smoothly over `ramp` seconds
    (a C2 time warp tau(t) with tau' = smoothstep), e.g. to exercise the zero-velocity update."""

    def __init__(self, seed=5, speed=1.0, static_until=None, ramp=1.0):
        self.static_until, self.ramp = static_until, ramp
        rng = np.random.default_rng(seed)
        self.ap = rng.uniform(0.5, 1.5, (3, 3)) * np.array([[2.0], [2.0], [0.4]]) * speed
        self.wp = rng.uniform(0.2, 0.6, (3, 3))
        self.php = rng.uniform(0, 2 * np.pi, (3, 3))
        self.ae = rng.uniform(0.05, 0.25, (3, 2)) * np.array([[1.0], [0.4], [0.4]])
        self.we = rng.uniform(0.3, 0.9, (3, 2))
        self.phe = rng.uniform(0, 2 * np.pi, (3, 2))

    def warp(self, t):
        """(tau, dtau/dt, d2tau/dt2)"""
        if self.static_until is None:
            return t, 1.0, 0.0
        t0, T = self.static_until, self.ramp
        x = (t - t0) / T
        if x <= 0:
            return t0, 0.0, 0.0
        if x >= 1:
            return t0 + 0.5 * T + (t - t0 - T), 1.0, 0.0
        return t0 + T * (x ** 3 - 0.5 * x ** 4), 3 * x ** 2 - 2 * x ** 3, (6 * x - 6 * x ** 2) / T

    def pos(self, t):
        tau = self.warp(t)[0]
        return np.sum(self.ap * np.sin(self.wp * tau + self.php), axis=1)

    def vel(self, t):
        tau, d1, _ = self.warp(t)
        return d1 * np.sum(self.ap * self.wp * np.cos(self.wp * tau + self.php), axis=1)

    def acc(self, t):
        tau, d1, d2 = self.warp(t)
        return (d1 * d1 * np.sum(-self.ap * self.wp ** 2 * np.sin(self.wp * tau + self.php), axis=1) +
                d2 * np.sum(self.ap * self.wp * np.cos(self.wp * tau + self.php), axis=1))

    def euler(self, t):
        tau = self.warp(t)[0]
        return np.sum(self.ae * np.sin(self.we * tau + self.phe), axis=1)

    def R_ItoG(self, t):
        yaw, pitch, roll = self.euler(t)
        cz, sz = np.cos(yaw), np.sin(yaw)
        cy, sy = np.cos(pitch), np.sin(pitch)
        cx, sx = np.cos(roll), np.sin(roll)
        Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
        Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
        Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
        # camera looks roughly along +x of the body; body z up
        return Rz @ Ry @ Rx

    def omega_I(self, t, h=1e-5):
        R0 = self.R_ItoG(t - h)
        R1 = self.R_ItoG(t + h)
        Rm = self.R_ItoG(t)
        dR = (R1 - R0) / (2 * h)
        W = Rm.T @ dR
        return np.array([W[2, 1] - W[1, 2], W[0, 2] - W[2, 0], W[1, 0] - W[0, 1]]) * 0.5


def cam_project(cam, p_C):
    """distort(p_C / z) with the camera model (CamRadtan.h:127 / CamEqui.h:136), vectorized."""
    v = np.array(cam.intrinsics[:])
    x = p_C[:, 0] / p_C[:, 2]
    y = p_C[:, 1] / p_C[:, 2]
    if cam.model == 0:
        r2 = x * x + y * y
        x1 = x * (1 + v[4] * r2 + v[5] * r2 * r2) + 2 * v[6] * x * y + v[7] * (r2 + 2 * x * x)
        y1 = y * (1 + v[4] * r2 + v[5] * r2 * r2) + v[6] * (r2 + 2 * y * y) + 2 * v[7] * x * y
    else:
        r = np.sqrt(x * x + y * y)
        th = np.arctan(r)
        thd = th + v[4] * th ** 3 + v[5] * th ** 5 + v[6] * th ** 7 + v[7] * th ** 9
        c = np.where(r > 1e-8, thd / np.maximum(r, 1e-12), 1.0)
        x1, y1 = x * c, y * c
    return np.stack([v[0] * x1 + v[2], v[1] * y1 + v[3]], axis=1)


def cam_backproject_approx(cam, uv):
    """Pinhole back-projection ignoring distortion (only used to seed point positions)."""
    v = np.array(cam.intrinsics[:])
    return np.stack([(uv[:, 0] - v[2]) / v[0], (uv[:, 1] - v[3]) / v[1], np.ones(len(uv))], axis=1)


class SimStream:
    """Pre-generated synthetic stream for one run (deterministic for a seed)."""

    def __init__(self, opts, duration=6.0, cam_rate=None, imu_rate=200.0, seed=5, spawn=200, life_full=None,
                 frac_lost=0.10, frac_long=0.05, sigma_pix=1.0, depth=(5.0, 7.0), noisy_imu=True, speed=1.0,
                 anchors=None, uwb_rate=10.0, uwb_sigma=0.5, static_for=None):
        """static_for: seconds after the start (t0 = 1 s) during which the platform rests (ZUPT workloads)."""
        self.opts = opts
        self.rng = np.random.default_rng(seed + 1000)
        self.traj = Trajectory(seed, speed, static_until=(1.0 + static_for) if static_for else None)
        self.cam_rate = cam_rate if cam_rate else (opts.track_frequency if opts.track_frequency > 0 else 20.0)
        self.imu_rate = imu_rate
        self.K = opts.num_cameras
        self.stereo = bool(opts.use_stereo) and self.K == 2
        self.life_full = life_full if life_full else opts.max_clone_size + 1
        self.t0 = 1.0
        # extrinsics R_ItoC, p_IinC
        self.R_ItoC, self.p_IinC = [], []
        for i in range(self.K):
            c = opts.cams[i]
            self.R_ItoC.append(quat_2_rot(np.array(c.q_ItoC[:])))
            self.p_IinC.append(np.array(c.p_IinC[:]))
        # IMU
        n_imu = int(duration * imu_rate) + 2
        self.imu_t = self.t0 - 0.5 + np.arange(n_imu) / imu_rate
        self.bg0 = np.zeros(3)
        self.ba0 = np.zeros(3)
        wm, am = [], []
        bg, ba = self.bg0.copy(), self.ba0.copy()
        dt = 1.0 / imu_rate
        for t in self.imu_t:
            R_ItoG = self.traj.R_ItoG(t)
            w = self.traj.omega_I(t)
            a = R_ItoG.T @ (self.traj.acc(t) + np.array([0, 0, G]))
            if noisy_imu:
                wn = w + bg + opts.sigma_w / np.sqrt(dt) * self.rng.standard_normal(3)
                an = a + ba + opts.sigma_a / np.sqrt(dt) * self.rng.standard_normal(3)
                bg = bg + opts.sigma_wb * np.sqrt(dt) * self.rng.standard_normal(3)
                ba = ba + opts.sigma_ab * np.sqrt(dt) * self.rng.standard_normal(3)
            else:
                wn, an = w, a
            wm.append(wn)
            am.append(an)
        self.wm = np.array(wm)
        self.am = np.array(am)
        # camera frames
        n_cam = int((duration - 0.6) * self.cam_rate)
        self.cam_t = self.t0 + (np.arange(n_cam) + 1) / self.cam_rate
        self.frames = []
        alive = []  # (id, p_G, death_frame, cam or -1)
        next_id = 0
        for k, t in enumerate(self.cam_t):
            R_ItoG = self.traj.R_ItoG(t)
            p_IinG = self.traj.pos(t)
            # spawn
            cams_spawn = [0] if self.stereo or self.K == 1 else list(range(self.K))
            for cs in cams_spawn:
                nsp = spawn if self.stereo or self.K == 1 else max(spawn // self.K, 1)
                cam = opts.cams[cs]
                uv = np.stack([self.rng.uniform(20, cam.width - 20, nsp), self.rng.uniform(20, cam.height - 20, nsp)], 1)
                b = cam_backproject_approx(cam, uv)
                d = self.rng.uniform(depth[0], depth[1], nsp)
                p_C = b * d[:, None]
                R_GtoC = self.R_ItoC[cs] @ R_ItoG.T
                p_CinG = p_IinG - R_GtoC.T @ self.p_IinC[cs]
                p_G = (R_GtoC.T @ p_C.T).T + p_CinG
                u = self.rng.uniform(0, 1, nsp)
                lives = np.where(u < frac_lost, self.rng.integers(3, self.life_full, nsp),
                                 np.where(u < frac_lost + frac_long, self.rng.integers(3 * self.life_full, 5 * self.life_full, nsp),
                                          self.life_full))
                for j in range(nsp):
                    alive.append((next_id, p_G[j], k + int(lives[j]), -1 if (self.stereo or self.K == 1) else cs))
                    next_id += 1
            alive = [a for a in alive if a[2] > k]
            frame = []
            ids_all = np.array([a[0] for a in alive], dtype=np.uint64)
            P = np.array([a[1] for a in alive]) if alive else np.zeros((0, 3))
            owner = np.array([a[3] for a in alive], dtype=np.int64)
            for i in range(self.K):
                cam = opts.cams[i]
                R_GtoC = self.R_ItoC[i] @ R_ItoG.T
                p_CinG = p_IinG - R_GtoC.T @ self.p_IinC[i]
                p_C = (R_GtoC @ (P - p_CinG).T).T
                ok = p_C[:, 2] > 0.2
                if not (self.stereo or self.K == 1):
                    ok &= owner == i
                uv = np.zeros((len(P), 2))
                if ok.any():
                    uv[ok] = cam_project(cam, p_C[ok])
                uv += sigma_pix * self.rng.standard_normal(uv.shape)
                ok &= (uv[:, 0] >= 0) & (uv[:, 0] < cam.width) & (uv[:, 1] >= 0) & (uv[:, 1] < cam.height)
                frame.append((ids_all[ok].copy(), uv[ok].astype(np.float32)))
            self.frames.append(frame)
        # UWB ranges (uvio): (1+beta)|p_A - p_U| + gamma + N(0, sigma^2)
        self.uwb = []
        if anchors:
            p_IinU = np.array(opts.p_IinU[:])
            t = self.t0 + 0.5 / uwb_rate
            while t < self.cam_t[-1] if len(self.cam_t) else False:
                R_ItoG = self.traj.R_ItoG(t)
                p_U = R_ItoG @ (-p_IinU) + self.traj.pos(t)
                ids, rs = [], []
                for a in anchors:
                    d = np.linalg.norm(np.array(a.p_AinG[:]) - p_U)
                    ids.append(int(a.id))
                    rs.append((1 + a.dist_bias) * d + a.const_bias + uwb_sigma * self.rng.standard_normal())
                self.uwb.append((t, ids, rs))
                t += 1.0 / uwb_rate

    def camera_pose(self, i, k):
        """(R_GtoC, p_CinG) of camera k at camera frame i (ground truth)."""
        t = self.cam_t[i]
        R_ItoG = self.traj.R_ItoG(t)
        p_IinG = self.traj.pos(t)
        R_GtoC = self.R_ItoC[k] @ R_ItoG.T
        return R_GtoC, p_IinG - R_GtoC.T @ self.p_IinC[k]

    def gt_state(self, t):
        """[t, q_GtoI, p_IinG, v_IinG, bg, ba] (initialize_with_gt input, VioManagerHelper.cpp:40)."""
        R_ItoG = self.traj.R_ItoG(t)
        q = rot_2_quat(R_ItoG.T)
        return np.concatenate([[t], q, self.traj.pos(t), self.traj.vel(t), self.bg0, self.ba0])

    def events(self):
        """Time-ordered (kind, t, payload) events: 'imu', 'cam' (frame index), 'uwb'."""
        ev = [("imu", t, i) for i, t in enumerate(self.imu_t)]
        ev += [("cam", t, k) for k, t in enumerate(self.cam_t)]
        ev += [("uwb", u[0], j) for j, u in enumerate(self.uwb)]
        # camera / UWB events are released one IMU period late so the IMU buffer already holds a
        # reading past their timestamp (as run_simulation.cpp / Simulator::get_next_cam ensure)
        order = {"imu": 0, "uwb": 1, "cam": 2}
        lag = 1.0 / self.imu_rate + 1e-9
        ev.sort(key=lambda e: (e[1] + (0.0 if e[0] == "imu" else lag), order[e[0]]))
        return ev

    def run(self, mgr, n_frames=None, on_frame=None, start_frame=0, before_frame=None, after_init=None, renderer=None,
            before_feed=None, init="gt"):
        """Drive one manager (or a list of managers in lock-step): initialize from ground truth at t0, then
        feed IMU / UWB / camera in time order.  before_frame(nf, t) runs before each camera feed,
        after_init(mgr) right after the ground-truth initialization (e.g. UWB anchor init), before_feed(mgr)
        right before each manager's camera feed (lock-step steering: the oracle, fed after the device, learns
        the device's results of the same frame).  With a
        renderer (uvio_amd.render.SceneRenderer) the managers get images (feed_measurement_camera)
        instead of the simulated tracks.  init="static" skips the ground-truth initialization: the camera
        feeds then run the managers' own initializer (VioManager::try_to_initialize, a stream that starts at
        rest) until it succeeds; after_init is not called."""
        mgrs = mgr if isinstance(mgr, (list, tuple)) else [mgr]
        static = init == "static"
        if static and renderer is None:
            raise ValueError("init='static' needs camera images (the simulated feed requires an initialized filter)")
        for m in mgrs:
            if static:
                continue
            m.initialize_with_gt(self.gt_state(self.t0))
            if after_init is not None:
                after_init(m)
        nf = 0
        for kind, t, i in self.events():
            if t < self.t0 - 0.4:
                continue
            if kind == "imu":
                for m in mgrs:
                    m.feed_measurement_imu(t, self.wm[i], self.am[i])
            elif kind == "uwb":
                for m in mgrs:
                    m.feed_measurement_uwb(t, self.uwb[i][1], self.uwb[i][2])
            else:
                if t <= self.t0:
                    continue
                if before_frame is not None:
                    before_frame(nf + 1, t)
                if renderer is not None:
                    imgs = [renderer.render(k, *self.camera_pose(i, k), frame_seed=i).cpu().numpy() for k in range(self.K)]
                    for m in mgrs:
                        if before_feed is not None:
                            before_feed(m)
                        m.feed_measurement_camera(t, list(range(self.K)), imgs, allow_uninit=static)
                else:
                    fr = self.frames[i]
                    for m in mgrs:
                        if before_feed is not None:
                            before_feed(m)
                        m.feed_measurement_simulation(t, list(range(self.K)), fr)
                nf += 1
                if on_frame is not None:
                    on_frame(nf, t)
                if n_frames is not None and nf >= n_frames:
                    break
        return nf
