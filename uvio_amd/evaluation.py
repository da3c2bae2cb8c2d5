"""Trajectory accuracy as the reference's ov_eval computes it (host-side measurement, numpy).

Restates, for the metric's "ATE RMSE vs ref" (BASELINE.json):
  * AlignTrajectory::align_posyaw (ov_eval/src/alignment/AlignTrajectory.cpp:84-106) -> yaw-only
    Umeyama with known scale (AlignUtils::align_umeyama, AlignUtils.cpp:26-93, get_best_yaw
    AlignUtils.h:53-58), or align_posyaw_single (:56-82) on the first pose when n_aligned == 1;
  * ResultTrajectory::calculate_ate (ov_eval/src/calc/ResultTrajectory.cpp:82-109): per pose the
    position error |p_gt - p_est_aligned| and the orientation error |log(R_est_aligned^T R_gt)| in
    degrees, summarized as RMSE (Statistics::calculate, ov_eval/src/utils/Statistics.h:100-108).
  * Loader::load_data (ov_eval/src/utils/Loader.cpp:26-90) and AlignUtils::perform_association
    (ov_eval/src/alignment/AlignUtils.cpp:103-188, offset 0, max difference 0.02 s as ResultTrajectory.cpp:45
    calls it) for trajectory files in the ov_eval text format (`t x y z qx qy qz qw [covariances]`).
Poses are (p_IinG, q_GtoI) with the JPL quaternion convention of the estimator (quat_ops.h).
"""
import numpy as np


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def quat_2_rot(q):
    """JPL q_GtoI -> R_GtoI (quat_ops.h:152)."""
    q = np.asarray(q, dtype=np.float64)
    qv = q[:3]
    return (2 * q[3] ** 2 - 1) * np.eye(3) - 2 * q[3] * _skew(qv) + 2 * np.outer(qv, qv)


def rot_z(t):
    """quat_ops.h:623"""
    c, s = np.cos(t), np.sin(t)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def best_yaw(C):
    """AlignUtils::get_best_yaw (AlignUtils.h:53-58)"""
    return np.arctan2(C[0, 1] - C[1, 0], C[0, 0] + C[1, 1])


def log_so3(R):
    """|log_so3(R)| as quat_ops.h:273-310 computes it (the vee of R's antisymmetric part scaled by theta / (2 sin
    theta); the Taylor form near the identity, the axis form at pi), so that a matrix that is not exactly
    orthonormal (ov_eval applies it to un-normalized ground-truth quaternions) gives the reference's value"""
    R = np.asarray(R, dtype=np.float64)
    tr = float(np.trace(R))
    if tr + 1.0 < 1e-10:
        if abs(R[2, 2] + 1.0) > 1e-5:
            w = (np.pi / np.sqrt(2.0 + 2.0 * R[2, 2])) * np.array([R[0, 2], R[1, 2], 1.0 + R[2, 2]])
        elif abs(R[1, 1] + 1.0) > 1e-5:
            w = (np.pi / np.sqrt(2.0 + 2.0 * R[1, 1])) * np.array([R[0, 1], 1.0 + R[1, 1], R[2, 1]])
        else:
            w = (np.pi / np.sqrt(2.0 + 2.0 * R[0, 0])) * np.array([1.0 + R[0, 0], R[1, 0], R[2, 0]])
        return float(np.linalg.norm(w))
    tr_3 = tr - 3.0
    if tr_3 < -1e-7:
        theta = np.arccos((tr - 1.0) / 2.0)
        mag = theta / (2.0 * np.sin(theta))
    else:
        mag = 0.5 - tr_3 / 12.0
    return float(np.linalg.norm(mag * np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])))


def align_posyaw(p_est, p_gt, q_est=None, q_gt=None, n_aligned=-1):
    """(R, t) with p_gt ~ R p_est + t, R a rotation about gravity (z).  n_aligned == 1 aligns on the
    first pose only (needs the quaternions); otherwise Umeyama over all positions, yaw only."""
    p_est = np.asarray(p_est, dtype=np.float64)
    p_gt = np.asarray(p_gt, dtype=np.float64)
    if n_aligned == 1:
        g_rot = quat_2_rot(q_gt[0]).T  # R_ItoG (JPL)
        est_rot = quat_2_rot(q_est[0]).T
        R = rot_z(best_yaw(est_rot @ g_rot.T))
        return R, p_gt[0] - R @ p_est[0]
    n = min(len(p_est), len(p_gt))
    data, model = p_est[:n], p_gt[:n]
    mu_M, mu_D = model.mean(axis=0), data.mean(axis=0)
    C = (model - mu_M).T @ (data - mu_D) / n  # sum model_zc data_zc^T / n
    R = rot_z(best_yaw(n * C.T))
    return R, mu_M - R @ mu_D


def ate(p_est, p_gt, q_est=None, q_gt=None, align="posyaw"):
    """ATE RMSE: {"pos_m": ..., "ori_deg": ... (None without quaternions)} after posyaw alignment."""
    p_est = np.asarray(p_est, dtype=np.float64)
    p_gt = np.asarray(p_gt, dtype=np.float64)
    if align == "posyaw":
        R, t = align_posyaw(p_est, p_gt)
    elif align == "none":
        R, t = np.eye(3), np.zeros(3)
    else:
        raise ValueError(align)
    pa = p_est @ R.T + t
    pos = np.linalg.norm(p_gt - pa, axis=1)
    out = {"pos_m": float(np.sqrt(np.mean(pos ** 2))), "ori_deg": None, "align": align}
    if q_est is not None and q_gt is not None:
        # pose_ESTinGT orientation (ResultTrajectory.cpp:74): quat_multiply(q_est, Inv(q_ESTtoGT)), which normalizes
        # the product (quat_ops.h:180-195), so R_GtoI_aligned = R_GtoI(q_est / |q_est|) R^T; the ground truth's
        # quaternion is used as loaded (:93-94)
        ori = [np.degrees(log_so3((quat_2_rot(np.asarray(qe) / np.linalg.norm(qe)) @ R.T).T @ quat_2_rot(qg)))
               for qe, qg in zip(q_est, q_gt)]
        out["ori_deg"] = float(np.sqrt(np.mean(np.square(ori))))
    return out


def load_traj(path):
    """Loader::load_data (Loader.cpp:26-90): lines starting with '#' skipped, space-separated fields, a line with
    at least 8 numbers is (t, x y z, qx qy qz qw); returns (times (n,), poses (n, 7))."""
    times, poses = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("#"):
                continue
            vals = [float(v) for v in line.split(" ") if v.strip()][:20]
            if len(vals) >= 8:
                times.append(vals[0])
                poses.append(vals[1:8])
    if not times:
        raise ValueError("no poses in %s" % path)
    return np.array(times), np.array(poses)


def associate(est_t, est_poses, gt_t, gt_poses, offset=0.0, max_difference=0.02):
    """AlignUtils::perform_association (AlignUtils.cpp:103-188): for each estimate (in order) the closest ground
    truth within max_difference, the ground-truth pointer only advancing (injective); the matched estimates take
    the ground-truth times.  Returns (times, est_poses, gt_poses) of the matches."""
    out_t, out_e, out_g = [], [], []
    gp = 0
    ng = len(gt_t)
    for i in range(len(est_t)):
        te = est_t[i] + offset
        best_diff, best = max_difference, -1
        while gp < ng and gt_t[gp] < te and abs(gt_t[gp] - te) > max_difference:
            gp += 1
        while gp < ng and abs(gt_t[gp] - te) <= max_difference:
            if abs(gt_t[gp] - te) >= best_diff:
                break
            best_diff, best = abs(gt_t[gp] - te), gp
            gp += 1
        if best != -1:
            out_t.append(gt_t[best])
            out_e.append(est_poses[i])
            out_g.append(gt_poses[best])
    return np.array(out_t), np.array(out_e), np.array(out_g)


def ate_files(path_est, path_gt, align="posyaw"):
    """ResultTrajectory(path_est, path_gt, "posyaw") + calculate_ate (ResultTrajectory.cpp:26-109): load, associate,
    align, RMSE; also returns the number of associated poses."""
    te, pe = load_traj(path_est)
    tg, pg = load_traj(path_gt)
    t, e, g = associate(te, pe, tg, pg)
    out = ate(e[:, 0:3], g[:, 0:3], e[:, 3:7], g[:, 3:7], align=align)
    out["n_assoc"] = int(len(t))
    out["n_est"], out["n_gt"] = int(len(te)), int(len(tg))
    return out
