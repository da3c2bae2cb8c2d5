// ORACLE — test infrastructure only (see la.h header).
#include "init.h"

#include <cmath>

namespace orc {

// InertialInitializer.cpp:49-71 (the age test reads the new message's time, as in the reference)
void InertialInitializer::feed_imu(const ImuData &m, double oldest_time) {
  imu_data.push_back(m);
  if (oldest_time != -1) {
    auto it0 = imu_data.begin();
    while (it0 != imu_data.end()) {
      if (m.t < oldest_time)
        it0 = imu_data.erase(it0);
      else
        it0++;
    }
  }
}

// FeatureHelper.h:123-181
static void compute_disparity(FeatureDatabase &db, double &disp_mean, double &disp_var, int &total_feats,
                              double newest_time = -1, double oldest_time = -1) {
  std::vector<double> disparities;
  for (auto &feat : db.features_idlookup) {
    for (auto &campairs : feat.second->timestamps) {
      if (campairs.second.size() < 2) continue;
      size_t camid = campairs.first;
      bool found0 = false, found1 = false;
      float u0 = 0, v0 = 0, u1 = 0, v1 = 0;
      for (size_t idx = 0; idx < feat.second->timestamps.at(camid).size(); idx++) {
        double time = feat.second->timestamps.at(camid).at(idx);
        if ((oldest_time == -1 || time > oldest_time) && !found0) {
          u0 = feat.second->uvs.at(camid).at(idx).first;
          v0 = feat.second->uvs.at(camid).at(idx).second;
          found0 = true;
          continue;
        }
        if ((newest_time == -1 || time < newest_time) && found0) {
          u1 = feat.second->uvs.at(camid).at(idx).first;
          v1 = feat.second->uvs.at(camid).at(idx).second;
          found1 = true;
          continue;
        }
      }
      if (!found0 || !found1) continue;
      float du = u1 - u0, dv = v1 - v0;
      disparities.push_back(std::sqrt(du * du + dv * dv));
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

// InertialInitializer.cpp:73-147
bool InertialInitializer::initialize(FeatureDatabase &db, double *timestamp, Mat &covariance, Mat &imu_state,
                                     bool wait_for_jerk) {
  double newest_cam_time = -1;
  for (auto const &feat : db.features_idlookup)
    for (auto const &camtimepair : feat.second->timestamps)
      for (auto const &time : camtimepair.second) newest_cam_time = std::max(newest_cam_time, time);
  double oldest_time = newest_cam_time - o.init_window_time - 0.10;
  if (newest_cam_time < 0 || oldest_time < 0) return false;
  db.cleanup_measurements(oldest_time);
  auto it_imu = imu_data.begin();
  while (it_imu != imu_data.end() && it_imu->t < oldest_time + o.calib_camimu_dt) it_imu = imu_data.erase(it_imu);
  bool moving_1to0 = false, moving_2to1 = false;
  if (o.init_max_disparity > 0) {
    double newest_time_allowed = newest_cam_time - 0.5 * o.init_window_time;
    int num_features0 = 0, num_features1 = 0;
    double avg_disp0, avg_disp1, var_disp0, var_disp1;
    compute_disparity(db, avg_disp0, var_disp0, num_features0, newest_time_allowed);
    compute_disparity(db, avg_disp1, var_disp1, num_features1, newest_cam_time, newest_time_allowed);
    int feat_thresh = 15;
    if (num_features0 < feat_thresh || num_features1 < feat_thresh) return false;
    moving_1to0 = (avg_disp0 > o.init_max_disparity);
    moving_2to1 = (avg_disp1 > o.init_max_disparity);
  }
  bool has_jerk = (!moving_1to0 && moving_2to1);
  bool is_still = (!moving_1to0 && !moving_2to1);
  if (((has_jerk && wait_for_jerk) || (is_still && !wait_for_jerk)) && o.init_imu_thresh > 0.0)
    return static_initialize(timestamp, covariance, imu_state, wait_for_jerk);
  return false;  // the dynamic initializer (init_dyn_use && !is_still) is not restated
}

// StaticInitializer.cpp:37-165
bool InertialInitializer::static_initialize(double *timestamp, Mat &covariance, Mat &imu_state, bool wait_for_jerk) {
  if (imu_data.size() < 2) return false;
  double newesttime = imu_data.back().t;
  double oldesttime = imu_data.front().t;
  const double w = o.init_window_time;
  if (newesttime - oldesttime < w) return false;
  std::vector<ImuData> window_1to0, window_2to1;
  for (const ImuData &data : imu_data) {
    if (data.t > newesttime - 0.5 * w && data.t <= newesttime - 0.0 * w) window_1to0.push_back(data);
    if (data.t > newesttime - 1.0 * w && data.t <= newesttime - 0.5 * w) window_2to1.push_back(data);
  }
  if (window_1to0.size() < 2 || window_2to1.size() < 2) return false;
  auto am = [](const ImuData &d) { return V3(d.am[0], d.am[1], d.am[2]); };
  auto wm = [](const ImuData &d) { return V3(d.wm[0], d.wm[1], d.wm[2]); };
  Mat a_avg_1to0(3, 1);
  for (const ImuData &data : window_1to0) a_avg_1to0 = a_avg_1to0 + am(data);
  for (int k = 0; k < 3; k++) a_avg_1to0[k] /= (int)window_1to0.size();
  double a_var_1to0 = 0;
  for (const ImuData &data : window_1to0) a_var_1to0 += dot(am(data) - a_avg_1to0, am(data) - a_avg_1to0);
  a_var_1to0 = std::sqrt(a_var_1to0 / ((int)window_1to0.size() - 1));
  Mat a_avg_2to1(3, 1), w_avg_2to1(3, 1);
  for (const ImuData &data : window_2to1) {
    a_avg_2to1 = a_avg_2to1 + am(data);
    w_avg_2to1 = w_avg_2to1 + wm(data);
  }
  for (int k = 0; k < 3; k++) {
    a_avg_2to1[k] = a_avg_2to1[k] / (double)window_2to1.size();
    w_avg_2to1[k] = w_avg_2to1[k] / (double)window_2to1.size();
  }
  double a_var_2to1 = 0;
  for (const ImuData &data : window_2to1) a_var_2to1 += dot(am(data) - a_avg_2to1, am(data) - a_avg_2to1);
  a_var_2to1 = std::sqrt(a_var_2to1 / ((int)window_2to1.size() - 1));
  const double thr = o.init_imu_thresh;
  if (a_var_1to0 < thr && wait_for_jerk) return false;
  if (a_var_2to1 > thr && wait_for_jerk) return false;
  if ((a_var_1to0 > thr || a_var_2to1 > thr) && !wait_for_jerk) return false;
  // gram_schmidt (helper.h:160-169)
  Mat z_axis = (1.0 / norm(a_avg_2to1)) * a_avg_2to1;
  Mat e_1 = V3(1.0, 0.0, 0.0);
  Mat x_axis = e_1 - z_axis * z_axis.T() * e_1;
  x_axis = (1.0 / norm(x_axis)) * x_axis;
  Mat y_axis = skew_x(z_axis) * x_axis;
  y_axis = (1.0 / norm(y_axis)) * y_axis;
  Mat Ro(3, 3);
  for (int k = 0; k < 3; k++) {
    Ro(k, 0) = x_axis[k];
    Ro(k, 1) = y_axis[k];
    Ro(k, 2) = z_axis[k];
  }
  Mat q_GtoI = rot_2_quat(Ro);
  Mat gravity_inG = V3(0.0, 0.0, o.gravity_mag);
  Mat bg = w_avg_2to1;
  Mat ba = a_avg_2to1 - quat_2_Rot(q_GtoI) * gravity_inG;
  *timestamp = window_2to1.back().t;
  imu_state = Mat(16, 1);
  for (int k = 0; k < 4; k++) imu_state[k] = q_GtoI[k];
  for (int k = 0; k < 3; k++) {
    imu_state[10 + k] = bg[k];
    imu_state[13 + k] = ba[k];
  }
  covariance = std::pow(0.02, 2) * Mat::Identity(15);
  for (int k = 0; k < 3; k++) {
    covariance(k, k) = std::pow(0.02, 2);
    covariance(3 + k, 3 + k) = std::pow(0.05, 2);
    covariance(6 + k, 6 + k) = std::pow(0.01, 2);
  }
  return true;
}

}  // namespace orc
