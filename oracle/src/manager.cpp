// ORACLE — test infrastructure only (see la.h header).
#include "manager.h"

#include <cmath>

#include <algorithm>

namespace orc {

using clk = std::chrono::steady_clock;
static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

Manager::Manager(const uvio_hp_options_t &opt)
    : o(opt), state(opt), prop(opt), msckf(opt), slam(opt), uwb(opt), initializer(opt), currid(4 * (size_t)opt.max_aruco_features + 1) {
  msckf.dbg = &fdbg;
  slam.dbg = &fdbg;
  tracker.num_features = (int)std::floor((double)opt.init_max_features / (double)opt.num_cameras);
  tracker.threshold = opt.fast_threshold;
  tracker.grid_x = opt.grid_x;
  tracker.grid_y = opt.grid_y;
  tracker.min_px_dist = opt.min_px_dist;
  tracker.histogram_method = opt.histogram_method;
  tracker.use_stereo = opt.use_stereo != 0;
  tracker.currid = 4 * (size_t)opt.max_aruco_features + 1;
  tracker.cams = &state.cams;
  if (o.try_zupt) zupt.reset(new UpdaterZUPT(opt));
  // UVioManager ctor (UVioManager.cpp:33-58)
  if (o.use_uwb) {
    if (o.do_calib_uwb_extrinsics) {
      std::vector<Ref> H_order = {imu_q_ref(state)};
      Mat H_R(3, 3), H_L = Mat::Identity(3), R = o.prior_uwb_imu_cov * Mat::Identity(3), res(3, 1);
      StateHelper::initialize_invertible(state, state.calib_UWBtoIMU, H_order, H_R, H_L, R, res);
      for (int k = 0; k < 3; k++) state.calib_UWBtoIMU->val[k] = state.calib_UWBtoIMU->fej[k] = o.p_IinU[k];
    }
    if (o.n_anchors > 0) {
      std::vector<uvio_hp_anchor_t> a(o.anchors, o.anchors + o.n_anchors);
      init_anchors(a);
    }
  }
}

// VioManagerHelper.cpp:40-76
void Manager::initialize_with_gt(const double x[17]) {
  for (int k = 0; k < 16; k++) state.imu->val[k] = state.imu->fej[k] = x[1 + k];
  Mat Cov = std::pow(0.02, 2) * Mat::Identity(15);
  for (int k = 0; k < 3; k++) {
    Cov(k, k) = std::pow(0.017, 2);
    Cov(3 + k, 3 + k) = std::pow(0.05, 2);
    Cov(6 + k, 6 + k) = std::pow(0.01, 2);
  }
  StateHelper::set_initial_covariance(state, Cov, {ref_of(state.imu)});
  state.timestamp = x[0];
  startup_time = x[0];
  is_initialized = true;
  db.cleanup_measurements(state.timestamp);
}

// VioManager.cpp:166-189
void Manager::feed_imu(double t, const double wm[3], const double am[3]) {
  double oldest_time = state.margtimestep();
  if (oldest_time > state.timestamp) oldest_time = -1;
  if (!is_initialized) oldest_time = t - o.init_window_time + state.calib_dt->val[0] - 0.10;
  ImuData d;
  d.t = t;
  for (int k = 0; k < 3; k++) {
    d.wm[k] = wm[k];
    d.am[k] = am[k];
  }
  prop.feed_imu(d, oldest_time);
  if (!is_initialized) initializer.feed_imu(d, oldest_time);
  if (is_initialized && zupt && (!o.zupt_only_at_beginning || !has_moved_since_zupt)) zupt->feed_imu(d, oldest_time);
}

// UVioManager.cpp:61-79
int Manager::feed_uwb(double t, const std::vector<std::pair<size_t, double>> &ranges) {
  if (!(is_initialized && anchors_initialized && distance > o.min_dist_to_use_uwb)) return 0;
  if (state.timestamp >= t) return 0;
  UwbMsg m;
  m.t = t;
  for (auto &r : ranges) m.ranges[r.first] = r.second;
  past_uwb.insert({t, m});
  return 0;
}

// UVioManager.cpp:81-113, 207-266
int Manager::init_anchors(const std::vector<uvio_hp_anchor_t> &anchors) {
  if (anchors.empty()) return 0;
  for (const auto &a : anchors) {
    if (state.anchors.find(a.id) != state.anchors.end()) continue;
    auto v = std::make_shared<Var>(K_ANCHOR, 5, 5);
    v->anchor_id = a.id;
    v->fixed = a.fix != 0;
    double x[5] = {a.p_AinG[0], a.p_AinG[1], a.p_AinG[2], a.const_bias, a.dist_bias};
    for (int k = 0; k < 5; k++) v->val[k] = v->fej[k] = x[k];
    state.anchors.insert({(size_t)a.id, v});
    if (!a.fix) {
      std::vector<Ref> H_order = {imu_q_ref(state)};
      Mat H_R(5, 3), H_L = Mat::Identity(5), R = Mat::Identity(5), res(5, 1);
      StateHelper::initialize_invertible(state, v, H_order, H_R, H_L, R, res);
      Mat cov(5, 5);
      for (int k = 0; k < 5; k++) cov(k, k) = a.cov_diag[k];
      StateHelper::set_initial_covariance(state, cov, {ref_of(v)});
    }
  }
  anchors_initialized = true;
  return 0;
}

// UVioManager.cpp:308-344
int Manager::do_uwb_propagate_update(const UwbMsg &m) {
  bool valid = false;
  for (auto &r : m.ranges)
    if (state.anchors.find(r.first) != state.anchors.end()) {
      valid = true;
      break;
    }
  if (!valid) return 0;
  if (!prop.propagate_uwb(state, m.t)) return 0;
  if (state.timestamp != (prop.experiment_uwb_dt ? m.t - state.calib_dt->val[0] : m.t)) return 0;
  for (auto &r : m.ranges) {
    if (state.anchors.find(r.first) != state.anchors.end()) {
      int rc = uwb.update_single(state, m.t, r.first, r.second);
      if (rc < 0) return rc;
    }
  }
  return 0;
}

// VioManager.cpp:191-254 + TrackSIM.cpp:30-79 (+ the UVIO UWB loop of UVioManager.cpp:178-188)
int Manager::feed_simulation(double t, const std::vector<int> &camids,
                             const std::vector<std::vector<std::pair<size_t, std::pair<float, float>>>> &feats) {
  auto rT1 = clk::now();
  for (size_t i = 0; i < camids.size(); i++) {
    int cam_id = camids[i];
    const Camera &cam = state.cams.at(cam_id);
    for (const auto &f : feats[i]) {
      size_t id = f.first + currid;
      float un, vn;
      cam.undistort_f(f.second.first, f.second.second, un, vn);
      db.update_feature(id, t, cam_id, f.second.first, f.second.second, un, vn);
    }
  }
  for (size_t i = 0; i < camids.size(); i++) sim_last[camids[i]] = feats[i];
  return after_tracking(t, camids, rT1);
}

// VioManagerHelper.cpp:78-190 (the thread's body, run inline: use_multi_threading_subs off)
bool Manager::try_to_initialize() {
  double timestamp = 0;
  Mat covariance, imu_state;
  bool wait_for_jerk = (zupt == nullptr);
  if (!initializer.initialize(db, &timestamp, covariance, imu_state, wait_for_jerk)) return false;
  for (int k = 0; k < 16; k++) state.imu->val[k] = state.imu->fej[k] = imu_state[k];
  StateHelper::set_initial_covariance(state, covariance, {ref_of(state.imu)});
  state.timestamp = timestamp;
  startup_time = timestamp;
  db.cleanup_measurements(state.timestamp);
  tracker.num_features = (int)std::floor((double)o.num_pts / (double)o.num_cameras);
  if (norm(state.imu->vel()) > o.zupt_max_velocity) has_moved_since_zupt = true;
  // VioManagerHelper.cpp:164, 187: success is recorded, yet the call returns false; the next camera frame
  // returns true through thread_init_success (:91-93)
  thread_init_success = true;
  return false;
}

int Manager::after_tracking(double t, const std::vector<int> &camids, clk::time_point rT1, bool try_init) {
  auto rT2 = clk::now();
  timing = uvio_hp_timing_t{};
  timing.tracking = secs(rT1, rT2);
  fdbg.feats.clear();
  // VioManager.cpp:308-317 (camera frames only; a simulated frame needs an initialized filter, :236-240)
  // UVioManager.cpp:152 / VioManager.cpp:294: the zero-velocity check comes first and reads is_initialized_vio
  // as it was before this frame's initialization check
  const bool was_initialized = is_initialized;
  if (!is_initialized) {
    if (!try_init) return UVIO_HP_E_STATE;
    if (!thread_init_success) {
      try_to_initialize();
      return UVIO_HP_E_STATE;
    }
    is_initialized = true;
  }
  // UVioManager.cpp:147-162 / VioManager.cpp:291-307: zero-velocity update; on success the frame ends here
  if (was_initialized && zupt && (!o.zupt_only_at_beginning || !has_moved_since_zupt)) {
    if (state.timestamp != t) {
      int z = zupt->try_update(state, db, t);
      if (z < 0) return z;
      did_zupt_update = z == 1;
    }
    if (did_zupt_update) {
      const double c = t + state.calib_dt->val[0] - 0.10;
      prop.clean_old_imu_measurements(c);
      zupt->clean_old_imu_measurements(c);
      timing.zupt = 1;
      timing.timestamp = t;
      timing.n_clones = (int)state.clones.size();
      timing.cov_dim = state.Cov.r;
      timing.total = secs(rT1, clk::now());
      return 0;
    }
  }
  if (!past_uwb.empty()) {
    for (auto it = past_uwb.begin(); it != past_uwb.lower_bound(t); it++) {
      // (experiment, see Propagator::propagate_uwb: compare on the camera clock)
      const double tu = prop.experiment_uwb_dt ? it->first - state.calib_dt->val[0] : it->first;
      if (tu < t && tu > state.timestamp) {
        int rc = do_uwb_propagate_update(it->second);
        if (rc < 0) return rc;
      }
    }
    past_uwb.erase(past_uwb.begin(), past_uwb.upper_bound(t));
  }
  int rc = do_feature_propagate_update(t, camids);
  timing.total = secs(rT1, clk::now());
  return rc;
}

// VioManager.cpp:255-321 (track_image_and_update; downsampling in capi.cpp, no ArUco)
int Manager::feed_camera(double t, const std::vector<int> &camids, const std::vector<GrayImg> &imgs,
                         const std::vector<GrayImg> &masks) {
  auto rT1 = clk::now();
  tracker.feed(t, camids, imgs, masks, db);
  return after_tracking(t, camids, rT1, true);
}

// VioManager.cpp:323-651
int Manager::do_feature_propagate_update(double t, const std::vector<int> &camids) {
  auto rT2 = clk::now();
  if (state.timestamp > t) return UVIO_HP_E_ORDER;
  if (state.timestamp != t) {
    int st = 0;
    if (!prop.propagate_and_clone(state, t, &st)) return st;
  }
  auto rT3 = clk::now();
  timing.timestamp = t;
  timing.propagation = secs(rT2, rT3);
  timing.n_clones = (int)state.clones.size();
  timing.cov_dim = state.Cov.r;
  if ((int)state.clones.size() < std::min(state.opt.max_clone_size, 5)) return 0;
  if (state.timestamp != t) return 0;
  has_moved_since_zupt = true;

  std::vector<FeatP> feats_lost, feats_marg, feats_slam;
  feats_lost = db.features_not_containing_newer(state.timestamp, false, true);
  if ((int)state.clones.size() > state.opt.max_clone_size || (int)state.clones.size() > 5)
    feats_marg = db.features_containing(state.margtimestep(), false, true);
  auto it1 = feats_lost.begin();
  while (it1 != feats_lost.end()) {
    bool found = false;
    for (const auto &p : (*it1)->uvs)
      if (std::find(camids.begin(), camids.end(), (int)p.first) != camids.end()) {
        found = true;
        break;
      }
    if (found)
      it1++;
    else
      it1 = feats_lost.erase(it1);
  }
  it1 = feats_lost.begin();
  while (it1 != feats_lost.end()) {
    if (std::find(feats_marg.begin(), feats_marg.end(), *it1) != feats_marg.end())
      it1 = feats_lost.erase(it1);
    else
      it1++;
  }
  std::vector<FeatP> feats_maxtracks;
  auto it2 = feats_marg.begin();
  while (it2 != feats_marg.end()) {
    bool reached_max = false;
    for (const auto &cams : (*it2)->timestamps)
      if ((int)cams.second.size() > state.opt.max_clone_size) {
        reached_max = true;
        break;
      }
    if (reached_max) {
      feats_maxtracks.push_back(*it2);
      it2 = feats_marg.erase(it2);
    } else {
      it2++;
    }
  }
  int curr_aruco_tags = 0;
  for (auto &l : state.features_SLAM)
    if ((int)l.second->featid <= 4 * state.opt.max_aruco_features) curr_aruco_tags++;
  if (state.opt.max_slam_features > 0 && t - startup_time >= state.opt.dt_slam_delay &&
      (int)state.features_SLAM.size() < state.opt.max_slam_features + curr_aruco_tags) {
    int amount_to_add = (state.opt.max_slam_features + curr_aruco_tags) - (int)state.features_SLAM.size();
    int valid_amount = (amount_to_add > (int)feats_maxtracks.size()) ? (int)feats_maxtracks.size() : amount_to_add;
    if (valid_amount > 0) {
      feats_slam.insert(feats_slam.end(), feats_maxtracks.end() - valid_amount, feats_maxtracks.end());
      feats_maxtracks.erase(feats_maxtracks.end() - valid_amount, feats_maxtracks.end());
    }
  }
  for (auto &landmark : state.features_SLAM) {
    FeatP feat2 = db.get_feature(landmark.second->featid);
    if (feat2 != nullptr) feats_slam.push_back(feat2);
    bool current_unique_cam = std::find(camids.begin(), camids.end(), landmark.second->unique_cam) != camids.end();
    if (feat2 == nullptr && current_unique_cam) landmark.second->should_marg = true;
    if (landmark.second->fail_count > 1) landmark.second->should_marg = true;
  }
  StateHelper::marginalize_slam(state);
  std::vector<FeatP> feats_slam_DELAYED, feats_slam_UPDATE;
  for (auto &f : feats_slam) {
    if (state.features_SLAM.find(f->featid) != state.features_SLAM.end())
      feats_slam_UPDATE.push_back(f);
    else
      feats_slam_DELAYED.push_back(f);
  }
  std::vector<FeatP> featsup_MSCKF = feats_lost;
  featsup_MSCKF.insert(featsup_MSCKF.end(), feats_marg.begin(), feats_marg.end());
  featsup_MSCKF.insert(featsup_MSCKF.end(), feats_maxtracks.begin(), feats_maxtracks.end());
  auto compare_feat = [](const FeatP &a, const FeatP &b) -> bool {
    size_t asize = 0, bsize = 0;
    for (const auto &p : a->timestamps) asize += p.second.size();
    for (const auto &p : b->timestamps) bsize += p.second.size();
    return asize < bsize;
  };
  std::sort(featsup_MSCKF.begin(), featsup_MSCKF.end(), compare_feat);
  if ((int)featsup_MSCKF.size() > state.opt.max_msckf_in_update)
    featsup_MSCKF.erase(featsup_MSCKF.begin(), featsup_MSCKF.end() - state.opt.max_msckf_in_update);
  timing.n_msckf = (int)featsup_MSCKF.size();
  last_msckf = UpdateStats{};
  int rc = msckf.update(state, featsup_MSCKF, &last_msckf);
  if (rc < 0) return rc;
  timing.msckf_rows = last_msckf.rows_stacked;
  timing.msckf_cols = last_msckf.cols;
  auto rT4 = clk::now();
  std::vector<FeatP> feats_slam_UPDATE_TEMP;
  while (!feats_slam_UPDATE.empty()) {
    size_t k = std::min((size_t)state.opt.max_slam_in_update, feats_slam_UPDATE.size());
    std::vector<FeatP> tmp(feats_slam_UPDATE.begin(), feats_slam_UPDATE.begin() + k);
    feats_slam_UPDATE.erase(feats_slam_UPDATE.begin(), feats_slam_UPDATE.begin() + k);
    rc = slam.update(state, tmp);
    if (rc < 0) return rc;
    feats_slam_UPDATE_TEMP.insert(feats_slam_UPDATE_TEMP.end(), tmp.begin(), tmp.end());
  }
  auto rT5 = clk::now();
  timing.n_slam_delayed = (int)feats_slam_DELAYED.size();
  rc = slam.delayed_init(state, feats_slam_DELAYED);
  if (rc < 0) return rc;
  auto rT6 = clk::now();
  if (!camids.empty() && camids[0] == 0) retriangulate_active_tracks(t, camids);
  for (auto &f : featsup_MSCKF) f->to_delete = true;
  db.cleanup();
  rc = slam.change_anchors(state);
  if (rc < 0) return rc;
  timing.n_anchor_change = rc;
  if ((int)state.clones.size() > state.opt.max_clone_size) db.cleanup_measurements(state.margtimestep());
  StateHelper::marginalize_old_clone(state);
  auto rT7 = clk::now();
  timing.msckf_update = secs(rT3, rT4);
  timing.slam_update = secs(rT4, rT5);
  timing.slam_delayed = secs(rT5, rT6);
  timing.marg = secs(rT6, rT7);
  timing.n_slam = (int)state.features_SLAM.size();
  if (timelastupdate != -1 && state.clones.find(timelastupdate) != state.clones.end()) {
    Mat dx = state.imu->pos() - state.clones.at(timelastupdate)->pos();
    distance += norm(dx);
  }
  timelastupdate = t;
  return 0;
}

// VioManager::retriangulate_active_tracks (VioManagerHelper.cpp:190-388)
void Manager::retriangulate_active_tracks(double t, const std::vector<int> &camids) {
  active_tracks_time = t;
  active_tracks_posinG.clear();
  active_tracks_uvd.clear();
  std::map<size_t, Mat> A_new, b_new;
  std::map<size_t, int> count_new;
  std::unordered_map<size_t, Mat> posinG_new;
  std::map<size_t, std::pair<float, float>> feat_uvs_in_cam0;
  // TrackBase::get_last_obs / get_last_ids: TrackKLT's points of the last feed, or TrackSIM's
  auto last_obs = [&](int cam, std::vector<std::pair<size_t, std::pair<float, float>>> &out) {
    out.clear();
    if (!sim_last.empty()) {
      auto it = sim_last.find(cam);
      if (it != sim_last.end())
        for (auto &f : it->second) out.push_back({f.first + currid, f.second});
      return;
    }
    auto it = tracker.pts_last.find((size_t)cam);
    if (it == tracker.pts_last.end()) return;
    const auto &ids = tracker.ids_last[(size_t)cam];
    for (size_t i = 0; i < it->second.size(); i++) out.push_back({ids[i], {it->second[i].x, it->second[i].y}});
  };
  const VarP &clone = state.clones.at(active_tracks_time);
  std::vector<std::pair<size_t, std::pair<float, float>>> obs;
  for (int cam_id : camids) {
    Mat R_GtoI = clone->Rot(), p_IinG = clone->pos();
    const VarP &calib = state.calib_IMUtoCAM.at(cam_id);
    Mat R_ItoC = calib->Rot(), p_IinC = calib->pos();
    Mat R_GtoCi = R_ItoC * R_GtoI;
    Mat p_CiinG = p_IinG - R_GtoCi.T() * p_IinC;
    last_obs(cam_id, obs);
    for (auto &ob : obs) {
      size_t featid = ob.first;
      if (cam_id == 0) feat_uvs_in_cam0[featid] = ob.second;
      if (state.features_SLAM.find(featid) != state.features_SLAM.end()) continue;
      float un, vn;
      state.cams.at(cam_id).undistort_f(ob.second.first, ob.second.second, un, vn);
      Mat b_i = V3(un, vn, 1);
      b_i = R_GtoCi.T() * b_i;
      b_i = (1.0 / norm(b_i)) * b_i;
      Mat Bperp = skew_x(b_i);
      Mat Ai = Bperp.T() * Bperp;
      Mat bi = Ai * p_CiinG;
      if (linsys_A.find(featid) == linsys_A.end()) {
        // std::map::insert: a second camera's observation of a new track does not replace the first's
        A_new.insert({featid, Ai});
        b_new.insert({featid, bi});
        count_new.insert({featid, 1});
      } else {
        A_new[featid] = Ai + linsys_A[featid];
        b_new[featid] = bi + linsys_b[featid];
        count_new[featid] = 1 + linsys_count[featid];
      }
      if (count_new.at(featid) > 3) {
        Mat A = A_new[featid], b = b_new[featid];
        Mat p_FinG = colpiv_qr_solve(A, b);
        Mat p_FinCi = R_GtoCi * (p_FinG - p_CiinG);
        double sv[3];
        singular_values3(A, sv);
        double condA = sv[0] / sv[2];
        if (std::abs(condA) <= o.fi_max_cond_number && p_FinCi[2] >= o.fi_min_dist && p_FinCi[2] <= o.fi_max_dist &&
            !std::isnan(norm(p_FinCi)))
          posinG_new[featid] = p_FinG;
      }
    }
  }
  linsys_A = A_new;
  linsys_b = b_new;
  linsys_count = count_new;
  active_tracks_posinG = posinG_new;
  if (active_tracks_posinG.empty() && state.features_SLAM.empty()) return;
  for (const auto &feat : state.features_SLAM) {
    Mat p_FinG = feat.second->get_xyz(false);
    if (is_relative(feat.second->rep)) {
      const VarP &cal = state.calib_IMUtoCAM.at(feat.second->anchor_cam);
      const VarP &anc = state.clones.at(feat.second->anchor_time);
      p_FinG = anc->Rot().T() * (cal->Rot().T() * (feat.second->get_xyz(false) - cal->pos())) + anc->pos();
    }
    active_tracks_posinG[feat.second->featid] = p_FinG;
  }
  const VarP &cal0 = state.calib_IMUtoCAM.at(0);
  Mat R_ItoC = cal0->Rot(), p_IinC = cal0->pos();
  Mat R_GtoIi = clone->Rot(), p_IiinG = clone->pos();
  const Camera &cam0 = state.cams.at(0);
  for (const auto &feat : active_tracks_posinG) {
    auto uv = feat_uvs_in_cam0.find(feat.first);
    if (uv == feat_uvs_in_cam0.end()) continue;
    Mat p_FinIi = R_GtoIi * (feat.second - p_IiinG);
    Mat p_FinCi = R_ItoC * p_FinIi + p_IinC;
    double depth = p_FinCi[2];
    double u = (double)uv->second.first, v = (double)uv->second.second;
    if (depth < 0.1) continue;
    if (u < 0 || (int)u >= cam0.w || v < 0 || (int)v >= cam0.h) continue;
    active_tracks_uvd[feat.first] = V3(u, v, depth);
  }
}

}  // namespace orc
