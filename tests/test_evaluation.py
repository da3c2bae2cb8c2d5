"""The ATE evaluator behind the bench's accuracy figure (uvio_amd/evaluation.py, ov_eval's posyaw ATE:
ResultTrajectory.cpp:26-109, AlignTrajectory.cpp:84-106, AlignUtils.cpp:103-188), CPU only.

* synthetic: a trajectory moved by a known yaw and translation is aligned back exactly; noise-free ATE is 0;
  the association keeps ov_eval's injective closest-match rule;
* the reference's own example pair (ov_eval/example/stamped_traj_estimate.txt, a VINS-Mono MH_01 run, against
  ov_data/euroc_mav/MH_01_easy.txt): the committed values of tests/golden/ate_ov_eval_example.json (made by
  tests/golden/make_ate_golden.py, values only) are reproduced by evaluation.py and agree with an independent
  SVD (2-D Procrustes) alignment.  The trajectory files exist only in this container (/root/reference); where
  they are absent that part is skipped.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
GOLDEN = os.path.join(ROOT, "tests", "golden", "ate_ov_eval_example.json")


def _jpl_from_rot(R):
    """JPL q_GtoI of R_GtoI (rot_2_quat, quat_ops.h:88)"""
    from scipy.spatial.transform import Rotation
    x, y, z, w = Rotation.from_matrix(R.T).as_quat()  # Hamilton q_ItoG == JPL q_GtoI
    return np.array([x, y, z, w])


def test_posyaw_recovers_a_known_yaw_and_translation():
    from uvio_amd import evaluation as E
    rng = np.random.default_rng(3)
    n = 400
    s = np.linspace(0, 6 * np.pi, n)
    p_gt = np.c_[3 * np.cos(s), 2 * np.sin(1.3 * s), 0.5 * np.sin(0.7 * s) + 1.0]
    R_gt = [E.rot_z(0.3 * np.sin(k)) @ E.quat_2_rot(_jpl_from_rot(E.rot_z(0.1 * k))) for k in s]
    q_gt = np.array([_jpl_from_rot(R) for R in R_gt])
    yaw, t = 0.7, np.array([1.5, -2.0, 0.25])
    Rz = E.rot_z(yaw)
    # the estimate lives in a frame yawed / shifted from the ground truth's: p_gt = Rz p_est + t
    p_est = (p_gt - t) @ Rz
    q_est = np.array([_jpl_from_rot(E.quat_2_rot(q) @ Rz) for q in q_gt])
    R, tt = E.align_posyaw(p_est, p_gt)
    assert np.allclose(R, Rz, atol=1e-12) and np.allclose(tt, t, atol=1e-12)
    r = E.ate(p_est, p_gt, q_est, q_gt)
    assert r["pos_m"] < 1e-12 and r["ori_deg"] < 1e-5
    # noise: the RMSE is the noise's (about sqrt(3) sigma)
    p_n = p_est + rng.normal(0, 0.01, p_est.shape)
    r = E.ate(p_n, p_gt)
    assert 0.012 < r["pos_m"] < 0.022


def test_association_is_injective_and_closest():
    from uvio_amd import evaluation as E
    gt_t = np.arange(0.0, 10.0, 0.005)
    gt = np.c_[gt_t, np.zeros((len(gt_t), 6))]
    est_t = np.array([0.0011, 0.0012, 0.05, 0.5001, 3.3, 9.999, 12.0])
    est = np.c_[est_t, np.zeros((len(est_t), 6))]
    t, e, g = E.associate(est_t, est, gt_t, gt)
    # 0.0011 -> 0.0; 0.0012 -> the next one (the pointer only advances); 12.0 has no match within 0.02 s
    assert np.allclose(t, [0.0, 0.005, 0.05, 0.5, 3.3, 9.995])
    assert np.allclose(e[:, 0], est_t[:6])
    assert len(set(np.round(t, 6))) == len(t)


def _sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def test_reference_example_pair_matches_golden_and_independent_alignment():
    import make_ate_golden as M
    with open(GOLDEN) as f:
        gold = json.load(f)
    # the committed values: the restatement and the independent SVD agree
    ev, ind = gold["evaluation"], gold["independent_svd"]
    assert abs(ev["pos_m"] - ind["pos_m"]) < 1e-12 and abs(ev["ori_deg"] - ind["ori_deg"]) < 1e-9
    assert abs(ev["yaw_rad"] - ind["yaw_rad"]) < 1e-12 and np.allclose(ev["t"], ind["t"], atol=1e-12)
    assert gold["n_assoc"] > 3000
    if not (os.path.exists(M.EST) and os.path.exists(M.GT)):
        pytest.skip("the reference's trajectory files are not on this machine (values checked above)")
    assert _sha(M.EST) == gold["source"]["estimate_sha256"] and _sha(M.GT) == gold["source"]["groundtruth_sha256"]
    now = M.compute()
    assert now["n_assoc"] == gold["n_assoc"] and now["n_est"] == gold["n_est"] and now["n_gt"] == gold["n_gt"]
    for k in ("pos_m", "ori_deg", "yaw_rad"):
        assert abs(now["evaluation"][k] - ev[k]) < 1e-12, k
        assert abs(now["independent_svd"][k] - ev[k]) < 1e-9, k
