// ORACLE — test infrastructure only (see la.h header).
#include "propagator.h"

#include <cstdlib>

#include <cstdio>

namespace orc {

Propagator::Propagator(const uvio_hp_options_t &o)
    : sigma_w(o.sigma_w), sigma_a(o.sigma_a), sigma_wb(o.sigma_wb), sigma_ab(o.sigma_ab), gravity(V3(0, 0, o.gravity_mag)) {
  const char *e = std::getenv("ORC_EXPERIMENT_UWB_DT");
  experiment_uwb_dt = e && e[0] == '1';
}

// Propagator.h:65-91
void Propagator::feed_imu(const ImuData &m, double oldest_time) {
  imu_data.push_back(m);
  clean_old_imu_measurements(oldest_time - 0.10);
}
void Propagator::clean_old_imu_measurements(double oldest_time) {
  if (oldest_time < 0) return;
  auto it = imu_data.begin();
  while (it != imu_data.end()) {
    if (it->t < oldest_time)
      it = imu_data.erase(it);
    else
      it++;
  }
}

// Propagator.h:154-164
ImuData Propagator::interpolate(const ImuData &a, const ImuData &b, double t) {
  double lambda = (t - a.t) / (b.t - a.t);
  ImuData d;
  d.t = t;
  for (int k = 0; k < 3; k++) {
    d.am[k] = (1 - lambda) * a.am[k] + lambda * b.am[k];
    d.wm[k] = (1 - lambda) * a.wm[k] + lambda * b.wm[k];
  }
  return d;
}

// Propagator.cpp:269-393
std::vector<ImuData> Propagator::select_imu_readings(const std::vector<ImuData> &imu, double time0, double time1) {
  std::vector<ImuData> prop;
  if (imu.empty()) return prop;
  for (size_t i = 0; i < imu.size() - 1; i++) {
    if (imu[i + 1].t > time0 && imu[i].t < time0) {
      prop.push_back(interpolate(imu[i], imu[i + 1], time0));
      continue;
    }
    if (imu[i].t >= time0 && imu[i + 1].t <= time1) {
      prop.push_back(imu[i]);
      continue;
    }
    if (imu[i + 1].t > time1) {
      if (imu[i].t > time1 && i == 0) {
        break;
      } else if (imu[i].t > time1) {
        prop.push_back(interpolate(imu[i - 1], imu[i], time1));
      } else {
        prop.push_back(imu[i]);
      }
      if (prop.back().t != time1) prop.push_back(interpolate(imu[i], imu[i + 1], time1));
      break;
    }
  }
  if (prop.empty()) return prop;
  if (prop.back().t != time1) prop.push_back(interpolate(imu[imu.size() - 2], imu[imu.size() - 1], time1));
  for (size_t i = 0; i + 1 < prop.size(); i++) {
    if (std::abs(prop[i + 1].t - prop[i].t) < 1e-12) {
      prop.erase(prop.begin() + i);
      i--;
    }
  }
  return prop;
}

std::vector<Ref> Propagator::phi_order(const State &s) const {
  std::vector<Ref> o;
  o.push_back(ref_of(s.imu));
  if (s.opt.do_calib_imu_intrinsics) {
    o.push_back(ref_of(s.dw));
    o.push_back(ref_of(s.da));
    if (s.opt.do_calib_imu_g_sensitivity) o.push_back(ref_of(s.tg));
    if (s.opt.imu_model == 0)
      o.push_back(ref_of(s.q_GYROtoIMU));
    else
      o.push_back(ref_of(s.q_ACCtoIMU));
  }
  return o;
}

void Propagator::accumulate(State &s, const std::vector<ImuData> &prop, Mat &Phi_summed, Mat &Qd_summed) {
  int n = s.imu_intrinsic_size() + 15;
  Phi_summed = Mat::Identity(n);
  Qd_summed = Mat(n, n);
  if (prop.size() > 1) {
    for (size_t i = 0; i < prop.size() - 1; i++) {
      Mat F, Qdi;
      predict_and_compute(s, prop[i], prop[i + 1], F, Qdi);
      Phi_summed = F * Phi_summed;
      Qd_summed = F * Qd_summed * F.T() + Qdi;
      Qd_summed = 0.5 * (Qd_summed + Qd_summed.T());
    }
  }
}

void Propagator::last_w_of(State &s, const std::vector<ImuData> &prop, Mat &last_w) {
  last_w = Mat(3, 1);
  if (!prop.empty()) {
    Mat Dw = s.Dm(s.dw->val), Da = s.Dm(s.da->val), Tg = s.Tg(s.tg->val);
    const ImuData &L = prop.back();
    Mat am = V3(L.am[0], L.am[1], L.am[2]), wm = V3(L.wm[0], L.wm[1], L.wm[2]);
    Mat last_a = s.q_ACCtoIMU->Rot() * Da * (am - s.imu->bias_a());
    last_w = s.q_GYROtoIMU->Rot() * Dw * (wm - s.imu->bias_g() - Tg * last_a);
  }
}

// Propagator.cpp:33-138
bool Propagator::propagate_and_clone(State &s, double timestamp, int *status) {
  *status = 0;
  if (s.timestamp >= timestamp) {
    *status = UVIO_HP_E_ORDER;
    return false;
  }
  if (!have_last_prop_time_offset) {
    last_prop_time_offset = s.calib_dt->val[0];
    have_last_prop_time_offset = true;
  }
  double t_off_new = s.calib_dt->val[0];
  double time0 = s.timestamp + last_prop_time_offset;
  double time1 = timestamp + t_off_new;
  std::vector<ImuData> prop = select_imu_readings(imu_data, time0, time1);
  Mat Phi, Qd;
  accumulate(s, prop, Phi, Qd);
  Mat last_w;
  last_w_of(s, prop, last_w);
  std::vector<Ref> order = phi_order(s);
  if (!StateHelper::EKFPropagation(s, order, order, Phi, Qd)) {
    *status = UVIO_HP_E_NUMERIC;
    return false;
  }
  s.timestamp = timestamp;
  last_prop_time_offset = t_off_new;
  StateHelper::augment_clone(s, last_w);
  return true;
}

// UVioPropagator.cpp:27-115 (quirks kept: time1 ignores the cam-imu offset and
// last_prop_time_offset is not updated)
bool Propagator::propagate_uwb(State &s, double timestamp) {
  if (s.timestamp >= (experiment_uwb_dt ? timestamp - s.calib_dt->val[0] : timestamp)) return false;
  double time0 = s.timestamp + last_prop_time_offset;
  double time1 = timestamp;
  std::vector<ImuData> prop = select_imu_readings(imu_data, time0, time1);
  Mat Phi, Qd;
  accumulate(s, prop, Phi, Qd);
  std::vector<Ref> order = phi_order(s);
  if (!StateHelper::EKFPropagation(s, order, order, Phi, Qd)) return false;
  s.timestamp = timestamp;
  // EXPERIMENT ONLY, off by default (the cfg5 ATE study): keep the state on the camera clock as
  // propagate_and_clone does (the IMU is now at timestamp = camera time + dt), instead of the reference's
  // IMU-clock timestamp that the next propagation then offsets by dt once more
  if (experiment_uwb_dt) {
    s.timestamp = timestamp - s.calib_dt->val[0];
    last_prop_time_offset = s.calib_dt->val[0];
    have_last_prop_time_offset = true;
  }
  return true;
}

// Propagator.cpp:395-480
void Propagator::predict_and_compute(State &s, const ImuData &dm, const ImuData &dp, Mat &F, Mat &Qd) {
  double dt = dp.t - dm.t;
  Mat Dw = s.Dm(s.dw->val), Da = s.Dm(s.da->val), Tg = s.Tg(s.tg->val);
  Mat a_hat1 = V3(dm.am[0], dm.am[1], dm.am[2]) - s.imu->bias_a();
  Mat a_hat2 = V3(dp.am[0], dp.am[1], dp.am[2]) - s.imu->bias_a();
  Mat a_hat_avg = .5 * (a_hat1 + a_hat2);
  Mat a_unc = a_hat_avg;
  Mat R_ACCtoIMU = s.q_ACCtoIMU->Rot();
  a_hat1 = R_ACCtoIMU * Da * a_hat1;
  a_hat2 = R_ACCtoIMU * Da * a_hat2;
  a_hat_avg = R_ACCtoIMU * Da * a_hat_avg;
  Mat w_hat1 = V3(dm.wm[0], dm.wm[1], dm.wm[2]) - s.imu->bias_g() - Tg * a_hat1;
  Mat w_hat2 = V3(dp.wm[0], dp.wm[1], dp.wm[2]) - s.imu->bias_g() - Tg * a_hat2;
  Mat w_hat_avg = .5 * (w_hat1 + w_hat2);
  Mat w_unc = w_hat_avg;
  Mat R_GYROtoIMU = s.q_GYROtoIMU->Rot();
  w_hat1 = R_GYROtoIMU * Dw * w_hat1;
  w_hat2 = R_GYROtoIMU * Dw * w_hat2;
  w_hat_avg = R_GYROtoIMU * Dw * w_hat_avg;

  Mat Xi(3, 18);
  if (s.opt.integration == 1 || s.opt.integration == 2) compute_Xi_sum(dt, w_hat_avg, a_hat_avg, Xi);
  Mat nq, nv, np;
  if (s.opt.integration == 2)
    predict_mean_analytic(s, dt, w_hat_avg, a_hat_avg, nq, nv, np, Xi);
  else if (s.opt.integration == 1)
    predict_mean_rk4(s, dt, w_hat1, a_hat1, w_hat2, a_hat2, nq, nv, np);
  else
    predict_mean_discrete(s, dt, w_hat_avg, a_hat_avg, nq, nv, np);

  int n = s.imu_intrinsic_size() + 15;
  F = Mat(n, n);
  Mat G(n, 12);
  if (s.opt.integration == 1 || s.opt.integration == 2)
    compute_F_and_G_analytic(s, dt, w_hat_avg, a_hat_avg, w_unc, a_unc, nq, nv, np, Xi, F, G);
  else
    compute_F_and_G_discrete(s, dt, w_hat_avg, a_hat_avg, w_unc, a_unc, nq, nv, np, F, G);

  Mat Qc(12, 12);
  for (int k = 0; k < 3; k++) {
    Qc(k, k) = std::pow(sigma_w, 2) / dt;
    Qc(3 + k, 3 + k) = std::pow(sigma_a, 2) / dt;
    Qc(6 + k, 6 + k) = std::pow(sigma_wb, 2) / dt;
    Qc(9 + k, 9 + k) = std::pow(sigma_ab, 2) / dt;
  }
  Qd = G * Qc * G.T();
  Qd = 0.5 * (Qd + Qd.T());

  for (int k = 0; k < 4; k++) s.imu->val[k] = nq[k];
  for (int k = 0; k < 3; k++) {
    s.imu->val[4 + k] = np[k];
    s.imu->val[7 + k] = nv[k];
  }
  s.imu->fej = s.imu->val;
}

void Propagator::predict_mean_discrete(State &s, double dt, const Mat &w_hat, const Mat &a_hat, Mat &new_q, Mat &new_v,
                                       Mat &new_p) {
  double w_norm = norm(w_hat);
  Mat I4 = Mat::Identity(4);
  Mat R_Gtoi = s.imu->Rot();
  Mat bigO;
  if (w_norm > 1e-12)
    bigO = std::cos(0.5 * w_norm * dt) * I4 + (1 / w_norm * std::sin(0.5 * w_norm * dt)) * Omega(w_hat);
  else
    bigO = I4 + (0.5 * dt) * Omega(w_hat);
  new_q = quatnorm(bigO * s.imu->quat());
  new_v = s.imu->vel() + dt * (R_Gtoi.T() * a_hat) - dt * gravity;
  new_p = s.imu->pos() + dt * s.imu->vel() + (0.5 * dt * dt) * (R_Gtoi.T() * a_hat) - (0.5 * dt * dt) * gravity;
}

// Propagator.cpp:507-586
void Propagator::predict_mean_rk4(State &s, double dt, const Mat &w_hat1, const Mat &a_hat1, const Mat &w_hat2,
                                  const Mat &a_hat2, Mat &new_q, Mat &new_v, Mat &new_p) {
  Mat w_hat = w_hat1, a_hat = a_hat1;
  Mat w_alpha = (1.0 / dt) * (w_hat2 - w_hat1);
  Mat a_jerk = (1.0 / dt) * (a_hat2 - a_hat1);
  Mat q_0 = s.imu->quat(), p_0 = s.imu->pos(), v_0 = s.imu->vel();
  Mat dq_0(4, 1);
  dq_0[3] = 1;
  Mat q0_dot = 0.5 * (Omega(w_hat) * dq_0);
  Mat p0_dot = v_0;
  Mat R_Gto0 = quat_2_Rot(quat_multiply(dq_0, q_0));
  Mat v0_dot = R_Gto0.T() * a_hat - gravity;
  Mat k1_q = dt * q0_dot, k1_p = dt * p0_dot, k1_v = dt * v0_dot;

  w_hat = w_hat + (0.5 * dt) * w_alpha;
  a_hat = a_hat + (0.5 * dt) * a_jerk;
  Mat dq_1 = quatnorm(dq_0 + 0.5 * k1_q);
  Mat v_1 = v_0 + 0.5 * k1_v;
  Mat q1_dot = 0.5 * (Omega(w_hat) * dq_1);
  Mat p1_dot = v_1;
  Mat R_Gto1 = quat_2_Rot(quat_multiply(dq_1, q_0));
  Mat v1_dot = R_Gto1.T() * a_hat - gravity;
  Mat k2_q = dt * q1_dot, k2_p = dt * p1_dot, k2_v = dt * v1_dot;

  Mat dq_2 = quatnorm(dq_0 + 0.5 * k2_q);
  Mat v_2 = v_0 + 0.5 * k2_v;
  Mat q2_dot = 0.5 * (Omega(w_hat) * dq_2);
  Mat p2_dot = v_2;
  Mat R_Gto2 = quat_2_Rot(quat_multiply(dq_2, q_0));
  Mat v2_dot = R_Gto2.T() * a_hat - gravity;
  Mat k3_q = dt * q2_dot, k3_p = dt * p2_dot, k3_v = dt * v2_dot;

  w_hat = w_hat + (0.5 * dt) * w_alpha;
  a_hat = a_hat + (0.5 * dt) * a_jerk;
  Mat dq_3 = quatnorm(dq_0 + k3_q);
  Mat v_3 = v_0 + k3_v;
  Mat q3_dot = 0.5 * (Omega(w_hat) * dq_3);
  Mat p3_dot = v_3;
  Mat R_Gto3 = quat_2_Rot(quat_multiply(dq_3, q_0));
  Mat v3_dot = R_Gto3.T() * a_hat - gravity;
  Mat k4_q = dt * q3_dot, k4_p = dt * p3_dot, k4_v = dt * v3_dot;

  Mat dq = quatnorm(dq_0 + (1.0 / 6.0) * k1_q + (1.0 / 3.0) * k2_q + (1.0 / 3.0) * k3_q + (1.0 / 6.0) * k4_q);
  new_q = quat_multiply(dq, q_0);
  new_p = p_0 + (1.0 / 6.0) * k1_p + (1.0 / 3.0) * k2_p + (1.0 / 3.0) * k3_p + (1.0 / 6.0) * k4_p;
  new_v = v_0 + (1.0 / 6.0) * k1_v + (1.0 / 3.0) * k2_v + (1.0 / 3.0) * k3_v + (1.0 / 6.0) * k4_v;
}

// Propagator.cpp:588-665
void Propagator::compute_Xi_sum(double dt, const Mat &w_hat, const Mat &a_hat, Mat &Xi_sum) {
  double w_norm = norm(w_hat);
  double d_th = w_norm * dt;
  Mat k_hat(3, 1);
  if (w_norm > 1e-12) k_hat = (1.0 / w_norm) * w_hat;
  Mat I3 = Mat::Identity(3);
  double d_t2 = std::pow(dt, 2), d_t3 = std::pow(dt, 3);
  double w_norm2 = std::pow(w_norm, 2), w_norm3 = std::pow(w_norm, 3);
  double cos_dth = std::cos(d_th), sin_dth = std::sin(d_th);
  double d_th2 = std::pow(d_th, 2), d_th3 = std::pow(d_th, 3);
  Mat sK = skew_x(k_hat), sK2 = sK * sK, sA = skew_x(a_hat);
  Mat R_ktok1 = exp_so3(-dt * w_hat);
  Mat Jr_ktok1 = Jr_so3(-dt * w_hat);
  double ka = dot(k_hat, a_hat);
  Mat Xi_1, Xi_2, Xi_3, Xi_4;
  bool small_w = (w_norm < 1.0 / 180 * M_PI / 2);
  if (!small_w) {
    Xi_1 = dt * I3 + ((1.0 - cos_dth) / w_norm) * sK + (dt - sin_dth / w_norm) * sK2;
    Xi_2 = (1.0 / 2 * d_t2) * I3 + ((d_th - sin_dth) / w_norm2) * sK + (1.0 / 2 * d_t2 - (1.0 - cos_dth) / w_norm2) * sK2;
    Xi_3 = (1.0 / 2 * d_t2) * sA + ((sin_dth - d_th) / w_norm2) * (sA * sK) +
           ((sin_dth - d_th * cos_dth) / w_norm2) * (sK * sA) + (1.0 / 2 * d_t2 - (1.0 - cos_dth) / w_norm2) * (sA * sK2) +
           (1.0 / 2 * d_t2 + (1.0 - cos_dth - d_th * sin_dth) / w_norm2) * (sK2 * sA + ka * sK) -
           ((3 * sin_dth - 2 * d_th - d_th * cos_dth) / w_norm2 * ka) * sK2;
    Xi_4 = (1.0 / 6 * d_t3) * sA + ((2 * (1.0 - cos_dth) - d_th2) / (2 * w_norm3)) * (sA * sK) +
           ((2 * (1.0 - cos_dth) - d_th * sin_dth) / w_norm3) * (sK * sA) +
           ((sin_dth - d_th) / w_norm3 + d_t3 / 6) * (sA * sK2) +
           ((d_th - 2 * sin_dth + 1.0 / 6 * d_th3 + d_th * cos_dth) / w_norm3) * (sK2 * sA + ka * sK) +
           ((4 * cos_dth - 4 + d_th2 + d_th * sin_dth) / w_norm3 * ka) * sK2;
  } else {
    Xi_1 = dt * (I3 + sin_dth * sK + (1.0 - cos_dth) * sK2);
    Xi_2 = (1.0 / 2 * dt) * Xi_1;
    Xi_3 = (1.0 / 2 * d_t2) *
           (sA + sin_dth * (-(sA * sK) + sK * sA + ka * sK2) + (1.0 - cos_dth) * (sA * sK2 + sK2 * sA + ka * sK));
    Xi_4 = (1.0 / 3 * dt) * Xi_3;
  }
  Xi_sum = Mat(3, 18);
  Xi_sum.set_block(0, 0, R_ktok1);
  Xi_sum.set_block(0, 3, Xi_1);
  Xi_sum.set_block(0, 6, Xi_2);
  Xi_sum.set_block(0, 9, Jr_ktok1);
  Xi_sum.set_block(0, 12, Xi_3);
  Xi_sum.set_block(0, 15, Xi_4);
}

void Propagator::predict_mean_analytic(State &s, double dt, const Mat &w_hat, const Mat &a_hat, Mat &new_q, Mat &new_v,
                                       Mat &new_p, const Mat &Xi) {
  Mat R_Gtok = s.imu->Rot();
  Mat q_ktok1 = rot_2_quat(Xi.block(0, 0, 3, 3));
  Mat Xi_1 = Xi.block(0, 3, 3, 3), Xi_2 = Xi.block(0, 6, 3, 3);
  new_q = quat_multiply(q_ktok1, s.imu->quat());
  new_v = s.imu->vel() + R_Gtok.T() * Xi_1 * a_hat - dt * gravity;
  new_p = s.imu->pos() + dt * s.imu->vel() + R_Gtok.T() * Xi_2 * a_hat - (0.5 * dt * dt) * gravity;
}

static Mat H_Dw(const State &s, const Mat &w) {
  Mat H(3, 6);
  if (s.opt.imu_model == 0) {  // w_1*I, w_2*e_2, w_2*e_3, w_3*e_3
    H(0, 0) = w[0]; H(1, 1) = w[0]; H(2, 2) = w[0];
    H(1, 3) = w[1]; H(2, 4) = w[1]; H(2, 5) = w[2];
  } else {  // w_1*e_1, w_2*e_1, w_2*e_2, w_3*I
    H(0, 0) = w[0]; H(0, 1) = w[1]; H(1, 2) = w[1];
    H(0, 3) = w[2]; H(1, 4) = w[2]; H(2, 5) = w[2];
  }
  return H;
}
static Mat H_Tg(const Mat &a) {
  Mat H(3, 9);
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) H(i, 3 * k + i) = a[k];
  return H;
}

// Propagator.cpp:683-828
void Propagator::compute_F_and_G_analytic(State &s, double dt, const Mat &w_hat, const Mat &a_hat, const Mat &w_unc,
                                          const Mat &a_unc, const Mat &new_q, const Mat &new_v, const Mat &new_p,
                                          const Mat &Xi, Mat &F, Mat &G) {
  int th_id = 0, p_id = 3, v_id = 6, bg_id = 9, ba_id = 12;
  int local_size = 15;
  int Dw_id = -1, Da_id = -1, Tg_id = -1, th_atoI_id = -1, th_wtoI_id = -1;
  if (s.opt.do_calib_imu_intrinsics) {
    Dw_id = local_size; local_size += 6;
    Da_id = local_size; local_size += 6;
    if (s.opt.do_calib_imu_g_sensitivity) { Tg_id = local_size; local_size += 9; }
    if (s.opt.imu_model == 0) { th_wtoI_id = local_size; local_size += 3; }
    else { th_atoI_id = local_size; local_size += 3; }
  }
  Mat R_k = s.imu->Rot(), v_k = s.imu->vel(), p_k = s.imu->pos();
  if (s.opt.do_fej) {
    R_k = s.imu->Rot_fej();
    v_k = s.imu->vel_fej();
    p_k = s.imu->pos_fej();
  }
  Mat dR = quat_2_Rot(new_q) * R_k.T();
  Mat Dw = s.Dm(s.dw->val), Da = s.Dm(s.da->val), Tg = s.Tg(s.tg->val);
  Mat R_atoI = s.q_ACCtoIMU->Rot(), R_wtoI = s.q_GYROtoIMU->Rot();
  Mat a_k = R_atoI * Da * a_unc;
  Mat w_k = R_wtoI * Dw * w_unc;
  Mat Xi_1 = Xi.block(0, 3, 3, 3), Xi_2 = Xi.block(0, 6, 3, 3), Jr = Xi.block(0, 9, 3, 3);
  Mat Xi_3 = Xi.block(0, 12, 3, 3), Xi_4 = Xi.block(0, 15, 3, 3);
  Mat I3 = Mat::Identity(3);
  Mat RkT = R_k.T();

  F.set_block(th_id, th_id, dR);
  F.set_block(p_id, th_id, -(skew_x(new_p - p_k - dt * v_k + (0.5 * dt * dt) * gravity) * RkT));
  F.set_block(v_id, th_id, -(skew_x(new_v - v_k + dt * gravity) * RkT));
  F.set_block(p_id, p_id, I3);
  F.set_block(p_id, v_id, dt * I3);
  F.set_block(v_id, v_id, I3);
  Mat dRJdt = dt * (dR * Jr);
  F.set_block(th_id, bg_id, -(dRJdt * R_wtoI * Dw));
  F.set_block(p_id, bg_id, RkT * Xi_4 * R_wtoI * Dw);
  F.set_block(v_id, bg_id, RkT * Xi_3 * R_wtoI * Dw);
  F.set_block(bg_id, bg_id, I3);
  F.set_block(th_id, ba_id, dRJdt * R_wtoI * Dw * Tg * R_atoI * Da);
  F.set_block(p_id, ba_id, -(RkT * (Xi_2 + Xi_4 * R_wtoI * Dw * Tg) * R_atoI * Da));
  F.set_block(v_id, ba_id, -(RkT * (Xi_1 + Xi_3 * R_wtoI * Dw * Tg) * R_atoI * Da));
  F.set_block(ba_id, ba_id, I3);
  if (Dw_id != -1) {
    Mat Hdw = H_Dw(s, w_unc);
    F.set_block(th_id, Dw_id, dRJdt * R_wtoI * Hdw);
    F.set_block(p_id, Dw_id, -(RkT * Xi_4 * R_wtoI * Hdw));
    F.set_block(v_id, Dw_id, -(RkT * Xi_3 * R_wtoI * Hdw));
    F.set_block(Dw_id, Dw_id, Mat::Identity(6));
  }
  if (Da_id != -1) {
    Mat Hda = H_Dw(s, a_unc);
    F.set_block(th_id, Da_id, -(dRJdt * R_wtoI * Dw * Tg * R_atoI * Hda));
    F.set_block(p_id, Da_id, RkT * (Xi_2 + Xi_4 * R_wtoI * Dw * Tg) * R_atoI * Hda);
    F.set_block(v_id, Da_id, RkT * (Xi_1 + Xi_3 * R_wtoI * Dw * Tg) * R_atoI * Hda);
    F.set_block(Da_id, Da_id, Mat::Identity(6));
  }
  if (Tg_id != -1) {
    Mat Htg = H_Tg(a_k);
    F.set_block(th_id, Tg_id, -(dRJdt * R_wtoI * Dw * Htg));
    F.set_block(p_id, Tg_id, RkT * Xi_4 * R_wtoI * Dw * Htg);
    F.set_block(v_id, Tg_id, RkT * Xi_3 * R_wtoI * Dw * Htg);
    F.set_block(Tg_id, Tg_id, Mat::Identity(9));
  }
  if (th_atoI_id != -1) {
    F.set_block(th_id, th_atoI_id, -(dRJdt * R_wtoI * Dw * Tg * skew_x(a_k)));
    F.set_block(p_id, th_atoI_id, RkT * (Xi_2 + Xi_4 * R_wtoI * Dw * Tg) * skew_x(a_k));
    F.set_block(v_id, th_atoI_id, RkT * (Xi_1 + Xi_3 * R_wtoI * Dw * Tg) * skew_x(a_k));
    F.set_block(th_atoI_id, th_atoI_id, I3);
  }
  if (th_wtoI_id != -1) {
    F.set_block(th_id, th_wtoI_id, dRJdt * skew_x(w_k));
    F.set_block(p_id, th_wtoI_id, -(RkT * Xi_4 * skew_x(w_k)));
    F.set_block(v_id, th_wtoI_id, -(RkT * Xi_3 * skew_x(w_k)));
    F.set_block(th_wtoI_id, th_wtoI_id, I3);
  }
  G.set_block(th_id, 0, -(dRJdt * R_wtoI * Dw));
  G.set_block(p_id, 0, RkT * Xi_4 * R_wtoI * Dw);
  G.set_block(v_id, 0, RkT * Xi_3 * R_wtoI * Dw);
  G.set_block(th_id, 3, dRJdt * R_wtoI * Dw * Tg * R_atoI * Da);
  G.set_block(p_id, 3, -(RkT * (Xi_2 + Xi_4 * R_wtoI * Dw * Tg) * R_atoI * Da));
  G.set_block(v_id, 3, -(RkT * (Xi_1 + Xi_3 * R_wtoI * Dw * Tg) * R_atoI * Da));
  G.set_block(bg_id, 6, dt * I3);
  G.set_block(ba_id, 9, dt * I3);
  (void)w_hat; (void)a_hat;
}

// Propagator.cpp:830-962 (log_so3 used for Jr)
static Mat log_so3(const Mat &R) {
  double R11 = R(0, 0), R12 = R(0, 1), R13 = R(0, 2);
  double R21 = R(1, 0), R22 = R(1, 1), R23 = R(1, 2);
  double R31 = R(2, 0), R32 = R(2, 1), R33 = R(2, 2);
  double tr = R11 + R22 + R33;
  Mat omega;
  if (tr + 1.0 < 1e-10) {
    if (std::abs(R33 + 1.0) > 1e-5)
      omega = (M_PI / std::sqrt(2.0 + 2.0 * R33)) * V3(R13, R23, 1.0 + R33);
    else if (std::abs(R22 + 1.0) > 1e-5)
      omega = (M_PI / std::sqrt(2.0 + 2.0 * R22)) * V3(R12, 1.0 + R22, R32);
    else
      omega = (M_PI / std::sqrt(2.0 + 2.0 * R11)) * V3(1.0 + R11, R21, R31);
  } else {
    double magnitude;
    double tr_3 = tr - 3.0;
    if (tr_3 < -1e-7) {
      double theta = std::acos((tr - 1.0) / 2.0);
      magnitude = theta / (2.0 * std::sin(theta));
    } else {
      magnitude = 0.5 - tr_3 / 12.0;
    }
    omega = magnitude * V3(R32 - R23, R13 - R31, R21 - R12);
  }
  return omega;
}

void Propagator::compute_F_and_G_discrete(State &s, double dt, const Mat &w_hat, const Mat &a_hat, const Mat &w_unc,
                                          const Mat &a_unc, const Mat &new_q, const Mat &new_v, const Mat &new_p, Mat &F,
                                          Mat &G) {
  int th_id = 0, p_id = 3, v_id = 6, bg_id = 9, ba_id = 12;
  int local_size = 15;
  int Dw_id = -1, Da_id = -1, Tg_id = -1, th_atoI_id = -1, th_wtoI_id = -1;
  if (s.opt.do_calib_imu_intrinsics) {
    Dw_id = local_size; local_size += 6;
    Da_id = local_size; local_size += 6;
    if (s.opt.do_calib_imu_g_sensitivity) { Tg_id = local_size; local_size += 9; }
    if (s.opt.imu_model == 0) { th_wtoI_id = local_size; local_size += 3; }
    else { th_atoI_id = local_size; local_size += 3; }
  }
  Mat R_k = s.imu->Rot(), v_k = s.imu->vel(), p_k = s.imu->pos();
  if (s.opt.do_fej) {
    R_k = s.imu->Rot_fej();
    v_k = s.imu->vel_fej();
    p_k = s.imu->pos_fej();
  }
  Mat dR = quat_2_Rot(new_q) * R_k.T();
  Mat Dw = s.Dm(s.dw->val), Da = s.Dm(s.da->val), Tg = s.Tg(s.tg->val);
  Mat R_atoI = s.q_ACCtoIMU->Rot(), R_wtoI = s.q_GYROtoIMU->Rot();
  Mat a_k = R_atoI * Da * a_unc;
  Mat w_k = R_wtoI * Dw * w_unc;
  Mat Jr = Jr_so3(log_so3(dR));
  Mat I3 = Mat::Identity(3);
  Mat RkT = R_k.T();
  Mat dRJdt = dt * (dR * Jr);
  F.set_block(th_id, th_id, dR);
  F.set_block(th_id, bg_id, -(dRJdt * R_wtoI * Dw));
  F.set_block(th_id, ba_id, dRJdt * R_wtoI * Dw * Tg * R_atoI * Da);
  F.set_block(p_id, th_id, -(skew_x(new_p - p_k - dt * v_k + (0.5 * dt * dt) * gravity) * RkT));
  F.set_block(p_id, p_id, I3);
  F.set_block(p_id, v_id, dt * I3);
  F.set_block(p_id, ba_id, -((0.5 * dt * dt) * (RkT * R_atoI * Da)));
  F.set_block(v_id, th_id, -(skew_x(new_v - v_k + dt * gravity) * RkT));
  F.set_block(v_id, v_id, I3);
  F.set_block(v_id, ba_id, -(dt * (RkT * R_atoI * Da)));
  F.set_block(bg_id, bg_id, I3);
  F.set_block(ba_id, ba_id, I3);
  if (Dw_id != -1) {
    Mat Hdw = H_Dw(s, w_unc);
    F.set_block(th_id, Dw_id, dRJdt * R_wtoI * Hdw);
    F.set_block(Dw_id, Dw_id, Mat::Identity(6));
  }
  if (Da_id != -1) {
    Mat Hda = H_Dw(s, a_unc);
    F.set_block(th_id, Da_id, -(dRJdt * R_wtoI * Tg * R_atoI * Hda));
    F.set_block(p_id, Da_id, (0.5 * dt * dt) * (RkT * R_atoI * Hda));
    F.set_block(v_id, Da_id, dt * (RkT * R_atoI * Hda));
    F.set_block(Da_id, Da_id, Mat::Identity(6));
  }
  if (Tg_id != -1) {
    Mat Htg = H_Tg(a_k);
    F.set_block(th_id, Tg_id, -(dRJdt * R_wtoI * Dw * Htg));
    F.set_block(Tg_id, Tg_id, Mat::Identity(9));
  }
  if (th_atoI_id != -1) {
    F.set_block(th_id, th_atoI_id, -(dRJdt * R_wtoI * Dw * Tg * skew_x(a_k)));
    F.set_block(p_id, th_atoI_id, (0.5 * dt * dt) * (RkT * skew_x(a_k)));
    F.set_block(v_id, th_atoI_id, dt * (RkT * skew_x(a_k)));
    F.set_block(th_atoI_id, th_atoI_id, I3);
  }
  if (th_wtoI_id != -1) {
    F.set_block(th_id, th_wtoI_id, dRJdt * skew_x(w_k));
    F.set_block(th_wtoI_id, th_wtoI_id, I3);
  }
  G.set_block(th_id, 0, -(dRJdt * R_wtoI * Dw));
  G.set_block(th_id, 3, dRJdt * R_wtoI * Dw * Tg * R_atoI * Da);
  G.set_block(v_id, 3, -(dt * (RkT * R_atoI * Da)));
  G.set_block(p_id, 3, -((0.5 * dt * dt) * (RkT * R_atoI * Da)));
  G.set_block(bg_id, 6, dt * I3);
  G.set_block(ba_id, 9, dt * I3);
  (void)w_hat; (void)a_hat;
}

}  // namespace orc
