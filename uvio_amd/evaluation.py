"""Trajectory accuracy as the reference's ov_eval computes it (host-side measurement, numpy).

Restates, for the metric's "ATE RMSE vs ref" (BASELINE.json):
  * AlignTrajectory::align_posyaw (ov_eval/src/alignment/AlignTrajectory.cpp:84-106) -> yaw-only
    Umeyama with known scale (AlignUtils::align_umeyama, AlignUtils.cpp:26-93, get_best_yaw
    AlignUtils.h:53-58), or align_posyaw_single (:56-82) on the first pose when n_aligned == 1;
  * ResultTrajectory::calculate_ate (ov_eval/src/calc/ResultTrajectory.cpp:82-109): per pose the
    position error |p_gt - p_est_aligned| and the orientation error |log(R_est_aligned^T R_gt)| in
    degrees, summarized as RMSE (Statistics::calculate, ov_eval/src/utils/Statistics.h:100-108).
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
    """|log(R)| (rotation angle, radians)"""
    c = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
    return float(np.arccos(c))


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
        # pose_ESTinGT orientation: R_GtoI_aligned = R_GtoI_est R^T  (quat_multiply(q_est, Inv(q_ESTtoGT)))
        ori = [np.degrees(log_so3((quat_2_rot(qe) @ R.T).T @ quat_2_rot(qg))) for qe, qg in zip(q_est, q_gt)]
        out["ori_deg"] = float(np.sqrt(np.mean(np.square(ori))))
    return out
