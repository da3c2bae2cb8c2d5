"""Golden values for the ATE evaluator (uvio_amd/evaluation.py) on the reference's own ov_eval example pair:
ov_eval/example/stamped_traj_estimate.txt (a VINS-Mono MH_01 run, ov_eval/example/readme.txt) against
ov_data/euroc_mav/MH_01_easy.txt, the way `ov_eval error_singlerun posyaw` evaluates it
(ResultTrajectory.cpp:26-109).  Only VALUES are committed (tests/golden/ate_ov_eval_example.json) -- the two
trajectory files stay in /root/reference and are identified by their SHA-256.

Two independent computations:
  * uvio_amd.evaluation.ate_files: the restatement (association, yaw-only Umeyama through get_best_yaw,
    AlignUtils.h:53-58, RMSE);
  * procrustes_posyaw below: the same association, then the least-squares yaw / translation from an SVD of the
    2x2 horizontal cross-covariance (2-D Procrustes; z is untouched by a yaw), no shared code with the above.

Run in this container (the reference is only here): python tests/golden/make_ate_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"
EST = os.path.join(REF, "ov_eval", "example", "stamped_traj_estimate.txt")
GT = os.path.join(REF, "ov_data", "euroc_mav", "MH_01_easy.txt")
OUT = os.path.join(ROOT, "tests", "golden", "ate_ov_eval_example.json")


def sha256(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def procrustes_posyaw(p_est, p_gt, q_est, q_gt):
    """independent yaw-only alignment (SVD) and ATE RMSE; quaternions JPL q_GtoI [x y z w]"""
    me, mg = p_est.mean(0), p_gt.mean(0)
    H = (p_est[:, :2] - me[:2]).T @ (p_gt[:, :2] - mg[:2])
    U, _, Vt = np.linalg.svd(H)
    D = np.diag([1.0, np.sign(np.linalg.det(Vt.T @ U.T))])
    R2 = Vt.T @ D @ U.T
    yaw = float(np.arctan2(R2[1, 0], R2[0, 0]))
    R = np.eye(3)
    R[:2, :2] = R2
    t = mg - R @ me
    pa = p_est @ R.T + t
    pos = float(np.sqrt(np.mean(np.sum((p_gt - pa) ** 2, axis=1))))

    def rot(q):  # R_ItoG of a JPL q_GtoI [x y z w], by quat_2_Rot's expression (quat_ops.h:152-160) transposed:
        # for the un-normalized ground-truth quaternions the metric is defined by that expression
        v, w = np.asarray(q[:3]), q[3]
        K = np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
        return ((2 * w * w - 1) * np.eye(3) - 2 * w * K + 2 * np.outer(v, v)).T

    ang = []
    for qe, qg in zip(q_est, q_gt):
        # ov_eval's definition (ResultTrajectory.cpp:74,93-94): the aligned estimate's quaternion is normalized
        # (quat_multiply), the ground truth's used as loaded; the angle is |log| of the error matrix, i.e. the
        # antisymmetric part's axis vector times theta / (2 sin theta) (quat_ops.h:273-310; no angle here is
        # near pi)
        E = (R @ rot(qe / np.linalg.norm(qe))).T @ rot(qg)
        tr = np.trace(E)
        # the Taylor form where the trace is within 1e-7 of 3 (un-normalized ground truth can push it past 3)
        scale = np.arccos((tr - 1) / 2) / (2 * np.sin(np.arccos((tr - 1) / 2))) if tr - 3 < -1e-7 else 0.5 - (tr - 3) / 12
        v = np.array([E[2, 1] - E[1, 2], E[0, 2] - E[2, 0], E[1, 0] - E[0, 1]])
        ang.append(np.degrees(np.linalg.norm(v) * scale))
    return {"pos_m": pos, "ori_deg": float(np.sqrt(np.mean(np.square(ang)))), "yaw_rad": yaw, "t": t.tolist()}


def compute():
    from uvio_amd import evaluation as E
    r = E.ate_files(EST, GT)
    te, pe = E.load_traj(EST)
    tg, pg = E.load_traj(GT)
    t, e, g = E.associate(te, pe, tg, pg)
    R, tt = E.align_posyaw(e[:, :3], g[:, :3])
    ind = procrustes_posyaw(e[:, :3], g[:, :3], e[:, 3:7], g[:, 3:7])
    return {
        "source": {"estimate": "ov_eval/example/stamped_traj_estimate.txt", "estimate_sha256": sha256(EST),
                   "groundtruth": "ov_data/euroc_mav/MH_01_easy.txt", "groundtruth_sha256": sha256(GT)},
        "n_est": r["n_est"], "n_gt": r["n_gt"], "n_assoc": r["n_assoc"],
        "assoc_time_first": float(t[0]), "assoc_time_last": float(t[-1]),
        "evaluation": {"pos_m": r["pos_m"], "ori_deg": r["ori_deg"],
                       "yaw_rad": float(np.arctan2(R[1, 0], R[0, 0])), "t": tt.tolist()},
        "independent_svd": ind,
    }


if __name__ == "__main__":
    out = compute()
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
