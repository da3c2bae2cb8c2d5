// Start-up from rest: VioManager::try_to_initialize (VioManagerHelper.cpp:78-190) with
// InertialInitializer::initialize (InertialInitializer.cpp:73-147), FeatureHelper::compute_disparity
// (FeatureHelper.h:123-181) and StaticInitializer::initialize (StaticInitializer.cpp:37-165).
//
// Host-only and run once per camera frame until it succeeds: a few hundred IMU samples and one pass
// over the feature database, nothing the device would speed up.  The reference runs it on a detached
// thread when use_multi_threading_subs is set; here it runs inline (the reference's single-threaded
// branch, VioManagerHelper.cpp:182-183), so no camera times queue up while it runs.  As in the reference,
// a successful attempt returns false: the frame that initialized ends there (UVioManager.cpp:168-175) and
// the next camera frame, finding thread_init_success, propagates and updates (VioManagerHelper.cpp:91-93).
// The dynamic initializer (DynamicInitializer.cpp, a Ceres MLE) is outside the hot path (SURVEY.md §8
// f3 names the static one): where the reference would call it (init_dyn_use and a moving platform,
// InertialInitializer.cpp:135-139) the frame fails with UVIO_HP_E_CONFIG and says so.
#include <cmath>

#include "engine.h"

namespace uvhp {

// FeatureDatabase::cleanup_measurements (FeatureDatabase.cpp:224-243): drop every measurement at or
// before t, then the features left without any
void Engine::db_cleanup_measurements(double t) {
  for (auto it = db_.begin(); it != db_.end();) {
    it->second->clean_older_measurements(t);
    if (it->second->count() < 1)
      it = db_erase(it);
    else
      it++;
  }
}

// FeatureHelper::compute_disparity (FeatureHelper.h:123-181) over the raw pixel coordinates of every
// feature and camera: per track the first measurement newer than oldest_time and the last one older than
// newest_time after it (-1 disables a bound).  Returns the number of disparities; the mean in *mean.
static int compute_disparity(const DbMap &db, double *mean, double newest_time,
                             double oldest_time) {
  std::vector<double> disp;
  for (const auto &kv : db) {
    for (const CamTrack &tr : kv.second->tracks) {
      if (tr.m.size() < 2) continue;
      bool found0 = false, found1 = false;
      float u0 = 0.f, v0 = 0.f, u1 = 0.f, v1 = 0.f;
      for (const FeatMeas &x : tr.m) {
        if ((oldest_time == -1 || x.t > oldest_time) && !found0) {
          u0 = x.u, v0 = x.v;
          found0 = true;
          continue;
        }
        if ((newest_time == -1 || x.t < newest_time) && found0) {
          u1 = x.u, v1 = x.v;
          found1 = true;
        }
      }
      if (!found0 || !found1) continue;
      const float du = u1 - u0, dv = v1 - v0;
      disp.push_back((double)std::sqrt(du * du + dv * dv));  // Eigen::Vector2f::norm, in float
    }
  }
  double m = 0;
  for (double d : disp) m += d;
  *mean = disp.empty() ? 0.0 : m / (double)disp.size();
  return (int)disp.size();
}

// StaticInitializer::initialize (StaticInitializer.cpp:37-165) on the initializer's IMU buffer.
// true: imu_ holds the static estimate; *t_init the state time; cov the 15x15 covariance of imu_.
bool Engine::static_initialize(bool wait_for_jerk, double *t_init, std::vector<double> &cov) {
  const std::vector<ImuSample> &imu = init_imu_;
  if (imu.size() < 2) return false;
  const double newest = imu.back().t, oldest = imu.front().t;
  const double w = o_.init_window_time;
  if (newest - oldest < w) return false;
  std::vector<const ImuSample *> w10, w21;  // (newest - w/2, newest], (newest - w, newest - w/2]
  for (const ImuSample &s : imu) {
    if (s.t > newest - 0.5 * w && s.t <= newest - 0.0 * w) w10.push_back(&s);
    if (s.t > newest - 1.0 * w && s.t <= newest - 0.5 * w) w21.push_back(&s);
  }
  if (w10.size() < 2 || w21.size() < 2) return false;
  auto mean_std = [](const std::vector<const ImuSample *> &win, double avg[3], double wavg[3]) {
    for (int k = 0; k < 3; k++) avg[k] = wavg[k] = 0.0;
    for (const ImuSample *s : win)
      for (int k = 0; k < 3; k++) avg[k] += s->am[k], wavg[k] += s->wm[k];
    for (int k = 0; k < 3; k++) avg[k] /= (double)win.size(), wavg[k] /= (double)win.size();
    double var = 0;
    for (const ImuSample *s : win) {
      const double d0 = s->am[0] - avg[0], d1 = s->am[1] - avg[1], d2 = s->am[2] - avg[2];
      var += d0 * d0 + d1 * d1 + d2 * d2;
    }
    return std::sqrt(var / (double)((int)win.size() - 1));
  };
  double a10[3], w10avg[3], a21[3], w21avg[3];
  const double var10 = mean_std(w10, a10, w10avg);
  const double var21 = mean_std(w21, a21, w21avg);
  const double thr = o_.init_imu_thresh;
  if (var10 < thr && wait_for_jerk) return false;   // no excitation yet
  if (var21 > thr && wait_for_jerk) return false;   // the older window was not at rest
  if ((var10 > thr || var21 > thr) && !wait_for_jerk) return false;  // moving
  // InitializerHelper::gram_schmidt (helper.h:138-170, the "original method" it ends with): z along the
  // mean specific force, x = e1 - z z^T e1, y = z x x; R_GtoI = [x y z]
  const double nz = std::sqrt(a21[0] * a21[0] + a21[1] * a21[1] + a21[2] * a21[2]);
  const double z[3] = {a21[0] / nz, a21[1] / nz, a21[2] / nz};
  double x[3] = {1.0 - z[0] * z[0], 0.0 - z[1] * z[0], 0.0 - z[2] * z[0]};
  const double nx = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  for (int k = 0; k < 3; k++) x[k] /= nx;
  double y[3] = {-z[2] * x[1] + z[1] * x[2], z[2] * x[0] - z[0] * x[2], -z[1] * x[0] + z[0] * x[1]};
  const double ny = std::sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
  for (int k = 0; k < 3; k++) y[k] /= ny;
  const double Ro[9] = {x[0], y[0], z[0], x[1], y[1], z[1], x[2], y[2], z[2]};
  double q[4], R[9];
  rot_2_quat(Ro, q);
  quat_2_Rot(q, R);
  // biases: gyro = mean rate, accel = mean specific force - R_GtoI g (StaticInitializer.cpp:127-131)
  double xs[16] = {0};
  for (int k = 0; k < 4; k++) xs[k] = q[k];
  for (int k = 0; k < 3; k++) {
    xs[10 + k] = w21avg[k];
    xs[13 + k] = a21[k] - R[3 * k + 2] * o_.gravity_mag;
  }
  for (int k = 0; k < 16; k++) imu_->val[k] = imu_->fej[k] = xs[k];
  *t_init = w21.back()->t;
  cov.assign(15 * 15, 0.0);
  for (int k = 0; k < 15; k++) cov[k * 15 + k] = 0.02 * 0.02;
  for (int k = 0; k < 3; k++) {
    cov[k * 15 + k] = 0.02 * 0.02;              // q
    cov[(3 + k) * 15 + 3 + k] = 0.05 * 0.05;    // p
    cov[(6 + k) * 15 + 6 + k] = 0.01 * 0.01;    // v (static)
  }
  return true;
}

// VioManager::try_to_initialize (VioManagerHelper.cpp:78-190) -> InertialInitializer::initialize
bool Engine::try_to_initialize() {
  // the newest camera time of the database and the window before it
  double newest_cam = -1;
  for (const auto &kv : db_)
    for (const CamTrack &tr : kv.second->tracks)
      for (const FeatMeas &x : tr.m) newest_cam = std::max(newest_cam, x.t);
  const double w = o_.init_window_time;
  const double oldest = newest_cam - w - 0.10;
  if (newest_cam < 0 || oldest < 0) return false;
  db_cleanup_measurements(oldest);
  {
    std::lock_guard<std::mutex> lk(imu_mtx_);
    auto it = init_imu_.begin();
    while (it != init_imu_.end() && it->t < oldest + o_.calib_camimu_dt) it++;
    init_imu_.erase(init_imu_.begin(), it);
  }
  bool moving_10 = false, moving_21 = false;
  if (o_.init_max_disparity > 0) {
    // InertialInitializer.cpp:102-125: the older half of the window, then the newer half
    const double newest_allowed = newest_cam - 0.5 * w;
    double d0 = 0, d1 = 0;
    const int n0 = compute_disparity(db_, &d0, newest_allowed, -1);
    const int n1 = compute_disparity(db_, &d1, newest_cam, newest_allowed);
    if (n0 < 15 || n1 < 15) return false;
    moving_10 = d0 > o_.init_max_disparity;
    moving_21 = d1 > o_.init_max_disparity;
  }
  const bool wait_for_jerk = !o_.try_zupt;  // VioManagerHelper.cpp:106
  const bool has_jerk = !moving_10 && moving_21, is_still = !moving_10 && !moving_21;
  if (!(((has_jerk && wait_for_jerk) || (is_still && !wait_for_jerk)) && o_.init_imu_thresh > 0.0)) {
    if (o_.init_dyn_use && !is_still)
      throw HpError(UVIO_HP_E_CONFIG,
                    "try_to_initialize: the platform is moving and init_dyn_use is set, so the reference would run "
                    "its dynamic initializer (InertialInitializer.cpp:135-139), which is not built; start from rest "
                    "or call initialize_with_gt");
    return false;
  }
  double t_init = 0;
  std::vector<double> cov;
  bool ok;
  {
    std::lock_guard<std::mutex> lk(imu_mtx_);
    ok = static_initialize(wait_for_jerk, &t_init, cov);
  }
  if (!ok) return false;
  // VioManagerHelper.cpp:111-166
  set_initial_covariance(cov, {imu_});
  timestamp_ = t_init;
  startup_time_ = t_init;
  db_cleanup_measurements(timestamp_);
  if (tracker_) tracker_->set_num_features((int)std::floor((double)o_.num_pts / (double)o_.num_cameras));
  const double *v = imu_->val + 7;
  if (std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) > o_.zupt_max_velocity) has_moved_since_zupt_ = true;
  // thread_init_success = true, but try_to_initialize returns false (VioManagerHelper.cpp:164, 187): the
  // frame that initialized ends here (UVioManager.cpp:168-175); the next camera frame reports success
  init_success_ = true;
  {
    std::lock_guard<std::mutex> lk(imu_mtx_);
    init_imu_.clear();
    init_imu_.shrink_to_fit();
  }
  return false;
}

}  // namespace uvhp
