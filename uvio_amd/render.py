"""Synthetic camera images for the KLT front-end (harness, not the measured path).

SURVEY.md §8(d): a procedural textured room is ray-cast through each camera's own model so that FAST
(threshold 10-50) finds >= num_pts corners per frame and the tracks obey the same projection the
estimator uses.  The room is an axis-aligned box; every face carries a random-gray tile pattern
(0.25 m tiles, corners for FAST) plus a finer value noise (texture for LK), and every image gets a
little seeded sensor noise.  Rays come from inverting the camera's distortion once per pixel grid
(fixed-point iteration as in cv::undistortPoints / fisheye::undistortPoints), so rendered corners land
where the estimator's distort() predicts them.

Rendering runs on torch (the GPU when present) so a few hundred stereo frames take seconds.

churn > 0 (track-loss streams): every face is cut into PANEL x PANEL m panels, and each panel redraws its
texture (tile values, tile-grid offset, noise) every `churn` frames at its own random phase, so about
1/churn of the scene changes under the tracks each frame.  A track on a redrawn panel loses its corner:
KLT drifts or fails and the RANSAC step drops it, as on real footage with occlusions and motion blur.
"""
import numpy as np
import torch

ROOM_MIN = (-9.0, -9.0, -2.0)
ROOM_MAX = (9.0, 9.0, 4.5)
TILE = 0.25
PANEL = 1.0


def _undistort_grid(cam):
    """Normalized (x, y) of every pixel centre of camera `cam` (uvio_hp_camera_t)."""
    v = np.array(cam.intrinsics[:], dtype=np.float64)
    W, H = cam.width, cam.height
    u, w = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    x0 = (u - v[2]) / v[0]
    y0 = (w - v[3]) / v[1]
    if cam.model == 0:
        x, y = x0.copy(), y0.copy()
        for _ in range(20):
            r2 = x * x + y * y
            icd = 1.0 / (1 + v[4] * r2 + v[5] * r2 * r2)
            dx = 2 * v[6] * x * y + v[7] * (r2 + 2 * x * x)
            dy = v[6] * (r2 + 2 * y * y) + 2 * v[7] * x * y
            x = (x0 - dx) * icd
            y = (y0 - dy) * icd
        return x, y
    thd = np.sqrt(x0 * x0 + y0 * y0)
    th = thd.copy()
    for _ in range(20):
        th2 = th * th
        f = th * (1 + v[4] * th2 + v[5] * th2 ** 2 + v[6] * th2 ** 3 + v[7] * th2 ** 4) - thd
        df = 1 + 3 * v[4] * th2 + 5 * v[5] * th2 ** 2 + 7 * v[6] * th2 ** 3 + 9 * v[7] * th2 ** 4
        th = th - f / df
    s = np.where(thd > 1e-12, np.tan(th) / np.maximum(thd, 1e-12), 1.0)
    return x0 * s, y0 * s


def _hash2(a, b, seed):
    h = (a * 73856093) ^ (b * 19349663) ^ (seed * 83492791)
    h = (h ^ (h >> 13)) * 1274126177
    h = h ^ (h >> 16)
    return (h & 0xFFFF).to(torch.float32) / 65535.0


class SceneRenderer:
    def __init__(self, opts, device=None, seed=1234, churn=0):
        self.device = torch.device(device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
        self.seed = seed
        self.churn = int(churn)
        self.rays = []
        self.sizes = []
        for i in range(opts.num_cameras):
            c = opts.cams[i]
            if opts.downsample_cameras:
                # the configured camera is the halved one (VioManagerOptions.h:251-260); the feed takes the raw
                # 2w x 2h image, so render at the raw resolution and intrinsics (exact: a power-of-two scale)
                from . import _native as N
                raw = N.Camera.from_buffer_copy(c)
                raw.width, raw.height = 2 * c.width, 2 * c.height
                for k in range(4):
                    raw.intrinsics[k] = 2.0 * c.intrinsics[k]
                c = raw
            x, y = _undistort_grid(c)
            d = np.stack([x, y, np.ones_like(x)], axis=-1)
            d /= np.linalg.norm(d, axis=-1, keepdims=True)
            self.rays.append(torch.tensor(d, dtype=torch.float32, device=self.device))
            self.sizes.append((c.width, c.height))
        self.lo = torch.tensor(ROOM_MIN, dtype=torch.float32, device=self.device)
        self.hi = torch.tensor(ROOM_MAX, dtype=torch.float32, device=self.device)

    def _texture(self, face, s, t, frame=0):
        seed = torch.full_like(face, self.seed)
        if self.churn > 0:
            # the panel's redraw epoch: floor((frame + phase) / churn), phase a per-panel hash in [0, churn)
            pi = torch.floor(s / PANEL).to(torch.int64) + 4096 * face
            pj = torch.floor(t / PANEL).to(torch.int64)
            phase = torch.floor(_hash2(pi, pj, self.seed + 3) * self.churn).to(torch.int64)
            epoch = torch.div(frame + phase, self.churn, rounding_mode="floor")
            seed = seed + 7919 * epoch
            # a new tile-grid offset per epoch moves the panel's corners
            s = s + TILE * _hash2(pi, pj, seed + 5)
            t = t + TILE * _hash2(pj, pi, seed + 11)
        si = torch.floor(s / TILE).to(torch.int64)
        ti = torch.floor(t / TILE).to(torch.int64)
        base = 35.0 + 185.0 * _hash2(si + 1000 * face, ti, seed)
        # value noise at 1/4 tile for LK texture
        fs, ft = s / (TILE / 4), t / (TILE / 4)
        i0, j0 = torch.floor(fs).to(torch.int64), torch.floor(ft).to(torch.int64)
        a, b = fs - i0, ft - j0
        n00 = _hash2(i0, j0, seed + 7 + face)
        n10 = _hash2(i0 + 1, j0, seed + 7 + face)
        n01 = _hash2(i0, j0 + 1, seed + 7 + face)
        n11 = _hash2(i0 + 1, j0 + 1, seed + 7 + face)
        n = (1 - a) * (1 - b) * n00 + a * (1 - b) * n10 + (1 - a) * b * n01 + a * b * n11
        return base + 36.0 * (n - 0.5)

    def render(self, k, R_GtoC, p_CinG, frame_seed=0):
        """u8 image (H, W) of camera k at pose (R_GtoC, p_CinG)."""
        R = torch.tensor(np.asarray(R_GtoC).T, dtype=torch.float32, device=self.device)  # C -> G
        o = torch.tensor(np.asarray(p_CinG), dtype=torch.float32, device=self.device)
        # (H, W, 3) in G; elementwise instead of a 3x3 matmul (keeps the harness off the BLAS
        # libraries, whose kernel lookup has failed for this shape on the box)
        rk = self.rays[k]
        d = rk[..., 0:1] * R[:, 0] + rk[..., 1:2] * R[:, 1] + rk[..., 2:3] * R[:, 2]
        inv = 1.0 / torch.where(d.abs() < 1e-9, torch.full_like(d, 1e-9), d)
        t1 = (self.lo - o) * inv
        t2 = (self.hi - o) * inv
        tfar = torch.maximum(t1, t2)  # exit distance per axis (camera is inside the box)
        tmin, axis = tfar.min(dim=-1)
        P = o + d * tmin[..., None]
        sign = torch.gather(d, -1, axis[..., None])[..., 0] > 0
        face = axis * 2 + sign.to(torch.int64)
        # in-plane coordinates of each face
        ax0 = torch.where(axis == 0, P[..., 1], P[..., 0])
        ax1 = torch.where(axis == 2, P[..., 1], P[..., 2])
        img = self._texture(face, ax0, ax1, frame_seed)
        g = torch.Generator(device=self.device)
        g.manual_seed(int(self.seed * 1000003 + frame_seed * 7 + k))
        img = img + 2.0 * torch.randn(img.shape, generator=g, device=self.device)
        return img.clamp(0, 255).round().to(torch.uint8)
