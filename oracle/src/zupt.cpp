// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_msckf/src/update/UpdaterZeroVelocity.{h,cpp} (feed_imu :77-90, clean_old_imu_measurements
// :96-107, try_update :65-329 with the defaults integrated_accel_constraint = false, model_time_varying_bias
// = true, override_with_disparity_check = true, explicitly_enforce_zero_motion = false),
// ov_core/src/feat/FeatureHelper.h:60-108 (compute_disparity between two times) and
// FeatureDatabase.cpp:245-263 (cleanup_measurements_exact).
#include "zupt.h"

#include <algorithm>
#include <cmath>

namespace orc {

UpdaterZUPT::UpdaterZUPT(const uvio_hp_options_t &o)
    : chi2_mult(o.zupt_chi2_multipler), max_velocity(o.zupt_max_velocity), noise_multiplier(o.zupt_noise_multiplier),
      max_disparity(o.zupt_max_disparity), sigma_w(o.sigma_w), sigma_a(o.sigma_a), sigma_wb(o.sigma_wb),
      sigma_ab(o.sigma_ab), gravity(V3(0, 0, o.gravity_mag)) {
  for (int i = 1; i < 1000; i++) chi2_table[i] = chi2_quantile95(i);
}

void UpdaterZUPT::feed_imu(const ImuData &m, double oldest_time) {
  imu_data.push_back(m);
  clean_old_imu_measurements(oldest_time - 0.10);
}

void UpdaterZUPT::clean_old_imu_measurements(double oldest_time) {
  if (oldest_time < 0) return;
  auto it = imu_data.begin();
  while (it != imu_data.end()) {
    if (it->t < oldest_time)
      it = imu_data.erase(it);
    else
      it++;
  }
}

// FeatureHelper::compute_disparity(db, time0, time1, ...) (FeatureHelper.h:60-108)
static void compute_disparity(FeatureDatabase &db, double time0, double time1, double &disp_mean, double &disp_var,
                              int &total_feats) {
  std::vector<FeatP> feats0 = db.features_containing(time0, false, true);
  std::vector<double> disparities;
  for (auto &feat : feats0) {
    for (auto &campairs : feat->timestamps) {
      size_t camid = campairs.first;
      const auto &ts = feat->timestamps.at(camid);
      auto it0 = std::find(ts.begin(), ts.end(), time0);
      auto it1 = std::find(ts.begin(), ts.end(), time1);
      if (it0 == ts.end() || it1 == ts.end()) continue;
      auto idx0 = std::distance(ts.begin(), it0);
      auto idx1 = std::distance(ts.begin(), it1);
      // (uv1 - uv0).norm() of Eigen::Vector2f: float arithmetic
      const auto &uv0 = feat->uvs.at(camid).at(idx0), &uv1 = feat->uvs.at(camid).at(idx1);
      const float dx = uv1.first - uv0.first, dy = uv1.second - uv0.second;
      disparities.push_back((double)std::sqrt(dx * dx + dy * dy));
    }
  }
  if (disparities.size() < 2) {
    disp_mean = -1;
    disp_var = -1;
    total_feats = 0;
  }
  disp_mean = 0;
  for (double d : disparities) disp_mean += d;
  disp_mean /= (double)disparities.size();
  disp_var = 0;
  for (double d : disparities) disp_var += std::pow(d - disp_mean, 2);
  disp_var = std::sqrt(disp_var / (double)(disparities.size() - 1));
  total_feats = (int)disparities.size();
}

// FeatureDatabase::cleanup_measurements_exact (FeatureDatabase.cpp:245-263)
static void cleanup_measurements_exact(FeatureDatabase &db, double timestamp) {
  for (auto it = db.features_idlookup.begin(); it != db.features_idlookup.end();) {
    Feature &f = *it->second;
    int ct = 0;
    for (auto &pair : f.timestamps) {
      auto &ts = f.timestamps[pair.first];
      auto &uv = f.uvs[pair.first];
      auto &un = f.uvs_norm[pair.first];
      size_t w = 0;
      for (size_t i = 0; i < ts.size(); i++)
        if (ts[i] != timestamp) {
          ts[w] = ts[i];
          uv[w] = uv[i];
          un[w] = un[i];
          w++;
        }
      ts.resize(w);
      uv.resize(w);
      un.resize(w);
      ct += (int)w;
    }
    if (ct < 1)
      db.features_idlookup.erase(it++);
    else
      it++;
  }
}

int UpdaterZUPT::try_update(State &s, FeatureDatabase &db, double timestamp) {
  last_accepted = false;
  if (imu_data.empty()) {
    last_zupt_state_timestamp = 0.0;
    return 0;
  }
  if (s.timestamp == timestamp) {
    last_zupt_state_timestamp = 0.0;
    return 0;
  }
  if (!have_last_prop_time_offset) {
    last_prop_time_offset = s.calib_dt->val[0];
    have_last_prop_time_offset = true;
  }
  const double t_off_new = s.calib_dt->val[0];
  const double time0 = s.timestamp + last_prop_time_offset;
  const double time1 = timestamp + t_off_new;
  std::vector<ImuData> imu_recent = Propagator::select_imu_readings(imu_data, time0, time1);
  last_prop_time_offset = t_off_new;
  if (imu_recent.size() < 2) {
    last_zupt_state_timestamp = 0.0;
    return 0;
  }
  // H_order [q_GtoI, bg, ba] (9 columns); 6 rows per IMU interval: [w_true = 0, a_true = 0]
  std::vector<Ref> Hx_order = {Ref{s.imu.get(), 0, 3}, Ref{s.imu.get(), 9, 3}, Ref{s.imu.get(), 12, 3}};
  const int m_size = 6 * ((int)imu_recent.size() - 1);
  Mat H(m_size, 9), res(m_size, 1);
  Mat Dw = s.Dm(s.dw->val), Da = s.Dm(s.da->val), Tg = s.Tg(s.tg->val);
  Mat R_ACCtoIMU = quat_2_Rot(s.q_ACCtoIMU->val.block(0, 0, 4, 1));
  Mat R_GYROtoIMU = quat_2_Rot(s.q_GYROtoIMU->val.block(0, 0, 4, 1));
  double dt_summed = 0;
  for (size_t i = 0; i + 1 < imu_recent.size(); i++) {
    const double dt = imu_recent[i + 1].t - imu_recent[i].t;
    Mat am = V3(imu_recent[i].am[0], imu_recent[i].am[1], imu_recent[i].am[2]);
    Mat wm = V3(imu_recent[i].wm[0], imu_recent[i].wm[1], imu_recent[i].wm[2]);
    Mat a_hat = R_ACCtoIMU * (Da * (am - s.imu->bias_a()));
    Mat w_hat = R_GYROtoIMU * (Dw * (wm - s.imu->bias_g() - Tg * a_hat));
    const double w_omega = std::sqrt(dt) / sigma_w;
    const double w_accel = std::sqrt(dt) / sigma_a;
    Mat r1 = (-w_omega) * w_hat;
    Mat r2 = (-w_accel) * (a_hat - s.imu->Rot() * gravity);
    for (int k = 0; k < 3; k++) {
      res[6 * (int)i + k] = r1[k];
      res[6 * (int)i + 3 + k] = r2[k];
    }
    Mat R_GtoI_jacob = s.opt.do_fej ? s.imu->Rot_fej() : s.imu->Rot();
    Mat Sg = skew_x(R_GtoI_jacob * gravity);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        H(6 * (int)i + a, 3 + b) = (a == b) ? -w_omega : 0.0;
        H(6 * (int)i + 3 + a, 0 + b) = -w_accel * Sg(a, b);
        H(6 * (int)i + 3 + a, 6 + b) = (a == b) ? -w_accel : 0.0;
      }
    dt_summed += dt;
  }
  UpdaterHelper::measurement_compress_inplace(H, res);
  if (H.r < 1) return 0;
  const double Rscale = noise_multiplier;
  Mat Q_bias = Mat::Identity(6);
  for (int k = 0; k < 3; k++) {
    Q_bias(k, k) *= dt_summed * sigma_wb * sigma_wb;
    Q_bias(3 + k, 3 + k) *= dt_summed * sigma_ab * sigma_ab;
  }
  Mat P_marg = StateHelper::get_marginal_covariance(s, Hx_order);
  P_marg.add_block(3, 3, Q_bias);
  Mat S = H * P_marg * H.T() + Rscale * Mat::Identity(H.r);
  Mat x = res;
  if (!llt_solve(S, x)) return 0;
  const double chi2 = dot(res, x);
  const double chi2_check = chi2_table.at(std::min(res.r, 999));
  double disp_avg = 0, disp_var = 0;
  int num_features = 0;
  compute_disparity(db, s.timestamp, timestamp, disp_avg, disp_var, num_features);
  const bool disparity_passed = (disp_avg < max_disparity && num_features > 20);
  last_chi2 = chi2;
  last_disparity = disp_avg;
  if (!disparity_passed && (chi2 > chi2_mult * chi2_check || norm(s.imu->vel()) > max_velocity)) {
    last_zupt_state_timestamp = 0.0;
    last_zupt_count = 0;
    return 0;
  }
  if (last_zupt_count >= 2) cleanup_measurements_exact(db, last_zupt_state_timestamp);
  std::vector<Ref> Phi_order = {Ref{s.imu.get(), 9, 3}, Ref{s.imu.get(), 12, 3}};
  if (!StateHelper::EKFPropagation(s, Phi_order, Phi_order, Mat::Identity(6), Q_bias)) return UVIO_HP_E_NUMERIC;
  if (!StateHelper::EKFUpdate(s, Hx_order, H, res, Rscale)) return UVIO_HP_E_NUMERIC;
  s.timestamp = timestamp;
  last_zupt_state_timestamp = timestamp;
  last_zupt_count++;
  last_accepted = true;
  return 1;
}

}  // namespace orc
