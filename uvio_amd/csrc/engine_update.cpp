// Engine: per-frame manager logic (VioManager.cpp:166-651, UVioManager.cpp:61-344), feature database
// (FeatureDatabase.cpp:59-263) and the update orchestration (UpdaterMSCKF.cpp:58-295,
// UpdaterSLAM.cpp:61-647, UpdaterUWB.cpp:53-90) over the device kernels.
#include <exception>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_set>

#include "engine.h"

namespace uvhp {

using clk = std::chrono::steady_clock;
static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// ---- chi-squared 0.95 quantile (boost::math::quantile(chi_squared(dof), 0.95), UpdaterMSCKF.cpp:52-55) ----
static double gamma_p(double a, double x) {
  if (x <= 0) return 0.0;
  double gln = std::lgamma(a);
  if (x < a + 1.0) {
    double ap = a, sum = 1.0 / a, del = sum;
    for (int n = 0; n < 100000; n++) {
      ap += 1;
      del *= x / ap;
      sum += del;
      if (std::fabs(del) < std::fabs(sum) * 1e-17) break;
    }
    return sum * std::exp(-x + a * std::log(x) - gln);
  }
  double b = x + 1.0 - a, c = 1e300, d = 1.0 / b, h = d;
  for (int i = 1; i < 100000; i++) {
    double an = -i * (i - a);
    b += 2.0;
    d = an * d + b;
    if (std::fabs(d) < 1e-300) d = 1e-300;
    c = b + an / c;
    if (std::fabs(c) < 1e-300) c = 1e-300;
    d = 1.0 / d;
    double del = d * c;
    h *= del;
    if (std::fabs(del - 1.0) < 1e-17) break;
  }
  return 1.0 - std::exp(-x + a * std::log(x) - gln) * h;
}
double chi2_quantile95(int dof) {
  double a = 0.5 * dof, lo = 0, hi = std::max(10.0, 4.0 * dof + 50);
  for (int it = 0; it < 200; it++) {
    double mid = 0.5 * (lo + hi);
    if (gamma_p(a, 0.5 * mid) < 0.95)
      lo = mid;
    else
      hi = mid;
    if (hi - lo < 1e-14 * std::max(1.0, hi)) break;
  }
  return 0.5 * (lo + hi);
}

// ---------------------------------------------------------------------------------------------------
// VioManagerHelper.cpp:40-76
void Engine::initialize_with_gt(const double x[17]) {
  for (int k = 0; k < 16; k++) imu_->val[k] = imu_->fej[k] = x[1 + k];
  std::vector<double> cov(15 * 15, 0.0);
  for (int k = 0; k < 15; k++) cov[k * 15 + k] = 0.02 * 0.02;
  for (int k = 0; k < 3; k++) {
    cov[k * 15 + k] = 0.017 * 0.017;
    cov[(3 + k) * 15 + 3 + k] = 0.05 * 0.05;
    cov[(6 + k) * 15 + 6 + k] = 0.01 * 0.01;
  }
  set_initial_covariance(cov, {imu_});
  timestamp_ = x[0];
  startup_time_ = x[0];
  is_initialized_ = true;
  db_cleanup_measurements(timestamp_);
  std::lock_guard<std::mutex> lk(imu_mtx_);
  init_imu_.clear();
}

// VioManager.cpp:166-189 + Propagator::feed_imu (Propagator.h:65-91)
void Engine::feed_imu(double t, const double wm[3], const double am[3]) {
  double oldest = margtimestep();
  if (oldest > timestamp_) oldest = -1;
  if (!is_initialized_) oldest = t - o_.init_window_time + calib_dt_->val[0] - 0.10;
  ImuSample s;
  s.t = t;
  for (int k = 0; k < 3; k++) s.wm[k] = wm[k], s.am[k] = am[k];
  std::lock_guard<std::mutex> lk(imu_mtx_);
  imu_data_.push_back(s);
  // InertialInitializer::feed_imu (InertialInitializer.cpp:49-71): its age test reads the new message's
  // time, so the buffer is emptied only by a message older than oldest (never, in time order); the
  // window is trimmed in InertialInitializer::initialize
  if (!is_initialized_ && !init_success_) {
    init_imu_.push_back(s);
    if (oldest != -1 && t < oldest) init_imu_.clear();
  }
  double cut = oldest - 0.10;
  // UpdaterZeroVelocity::feed_imu (VioManager.cpp:186-188; UpdaterZeroVelocity.h:77-107)
  if (is_initialized_ && o_.try_zupt && (!o_.zupt_only_at_beginning || !has_moved_since_zupt_)) {
    zupt_imu_.push_back(s);
    if (cut >= 0)
      zupt_imu_.erase(std::remove_if(zupt_imu_.begin(), zupt_imu_.end(), [&](const ImuSample &a) { return a.t < cut; }),
                      zupt_imu_.end());
  }
  if (cut >= 0) {
    auto it = imu_data_.begin();
    while (it != imu_data_.end() && it->t < cut) it++;
    // measurements arrive in time order: erase the prefix (same result as the reference's scan)
    bool sorted = true;
    for (auto jt = it; jt != imu_data_.end(); ++jt)
      if (jt->t < cut) sorted = false;
    if (sorted)
      imu_data_.erase(imu_data_.begin(), it);
    else
      imu_data_.erase(std::remove_if(imu_data_.begin(), imu_data_.end(), [&](const ImuSample &a) { return a.t < cut; }),
                      imu_data_.end());
  }
}

// FeatureDatabase::update_feature (FeatureDatabase.cpp:59-85)
void Engine::db_update(size_t id, double t, size_t cam, float u, float v, float un, float vn) {
  auto it = db_.find(id);
  Feature *f;  // no shared_ptr copy (two atomic reference-count updates per observation)
  if (it != db_.end()) {
    f = it->second.get();
  } else {
    FeatP nf = new_feature(id);
    f = nf.get();
    db_insert(id, std::move(nf));
  }
  f->track(cam).m.push_back(FeatMeas{u, v, un, vn, t});
}

// UVioManager.cpp:61-79
int Engine::feed_uwb(double t, int n, const uint64_t *ids, const double *ranges) {
  stage_ = "feed_uwb";
  if (!(is_initialized_ && anchors_initialized_ && distance_ > o_.min_dist_to_use_uwb)) return 0;
  if (timestamp_ >= t) return 0;
  auto &m = past_uwb_[t];
  for (int i = 0; i < n; i++) m[(size_t)ids[i]] = ranges[i];
  return 0;
}

// UVioManager.cpp:81-113 / 207-266
int Engine::init_anchors(int n, const uvio_hp_anchor_t *a) {
  if (n <= 0) return 0;
  for (int i = 0; i < n; i++) {
    if (anchors_.find(a[i].id) != anchors_.end()) continue;
    VarP v = std::make_shared<Var>(V_ANCHOR, 5, 5);
    v->anchor_id = a[i].id;
    v->fixed = a[i].fix != 0;
    double x[5] = {a[i].p_AinG[0], a[i].p_AinG[1], a[i].p_AinG[2], a[i].const_bias, a[i].dist_bias};
    for (int k = 0; k < 5; k++) v->val[k] = v->fej[k] = x[k];
    anchors_.insert({(size_t)a[i].id, v});
    if (!a[i].fix) {
      std::vector<double> HR(15, 0.0), HL(25, 0.0), R(25, 0.0), res(5, 0.0);
      for (int k = 0; k < 5; k++) HL[6 * k] = 1.0, R[6 * k] = 1.0;
      initialize_invertible_host(v, {{imu_->id, 3}}, HR, HL, R, res);
      std::vector<double> cov(25, 0.0);
      for (int k = 0; k < 5; k++) cov[6 * k] = a[i].cov_diag[k];
      set_initial_covariance(cov, {v});
    }
  }
  anchors_initialized_ = true;
  return 0;
}

// ---------------------------------------------------------------------------------------------------
// VioManager.cpp:191-254 + TrackSIM.cpp:30-79 (+ the UVIO range loop of UVioManager.cpp:178-188)
int Engine::feed_simulation(double t, int ncam, const int *cam_ids, const int *counts, const uint64_t *ids,
                            const float *uv) {
  stage_ = "feed_simulation";
  auto rT1 = clk::now();
  early_prop_s_ = 0.0;
  frame_begin();
  retri_flush();  // the previous frame's retriangulation reads frame_obs_, which this feed refills
  std::vector<int> camids, cam_of;
  for (int i = 0; i < ncam; i++) {
    int cid = cam_ids[i];
    if (cid < 0 || cid >= o_.num_cameras || counts[i] < 0) return UVIO_HP_E_ARG;
    camids.push_back(cid);
    cam_of.insert(cam_of.end(), counts[i], cid);
  }
  // FeatureDatabase::update_feature for every observation, in order, in three passes with the same
  // result: (a) undistort every observation, record it for the retriangulation and look up the known
  // features (independent per observation, read-only on db_, one pool job), (b) insert the new ids into db_
  // sequentially in observation order (db_'s iteration order depends on it), (c) append each observation
  // to its feature; features are split across workers by pointer, and every worker walks the observations
  // in order, so each feature's appends keep the sequential order.
  const size_t nobs = cam_of.size();
  std::vector<float> uvn(2 * nobs);
  std::vector<Feature *> fp(nobs, nullptr);
  frame_obs_.resize(nobs);
  {
    HPROF("feed.undistort_lookup");
    pool_.parallel_for(nobs, 2048, [&](size_t b, size_t e) {
      for (size_t k = b; k < e; k++) {
        const size_t id = (size_t)ids[k] + currid_;
        cam_undistort_f(cams_[cam_of[k]], uv[2 * k], uv[2 * k + 1], uvn[2 * k], uvn[2 * k + 1]);
        DRetriObs &o = frame_obs_[k];
        o.featid = (unsigned long long)id;
        o.u = uv[2 * k];
        o.v = uv[2 * k + 1];
        o.un = uvn[2 * k];
        o.vn = uvn[2 * k + 1];
        o.cam = cam_of[k];
        o.pad = 0;
        auto it = db_.find(id);
        if (it != db_.end()) fp[k] = it->second.get();
      }
    });
  }
  // (b) and (c) as one pool job: its first task inserts the new ids in observation order while the other
  // tasks append the observations of the features db_ already held (they touch neither db_ nor a new
  // feature); then the new features' observations are appended.  Every feature's observations are all in
  // one of the two groups, so its appends keep the sequential order.
  {
    HPROF("feed.db");
    // 4 buckets per thread: the known features' buckets share the threads with the insert task and are
    // taken dynamically (one bucket per thread left one thread with two while the others waited)
    const uint32_t nw = 4 * (uint32_t)pool_.threads();
    std::vector<uint32_t> known, fresh;
    known.reserve(nobs);
    for (size_t k = 0; k < nobs; k++) (fp[k] ? known : fresh).push_back((uint32_t)k);
    // bucket a list of observations by owning worker (a counting sort that keeps observation order inside a
    // bucket); a worker appends its bucket with the feature objects prefetched a few entries ahead -- the
    // appends are cache-miss bound (feature, its track array, the measurement storage)
    struct Buckets {
      std::vector<uint32_t> start, order;
    };
    auto bucket = [&](const std::vector<uint32_t> &obs, Buckets &bk) {
      bk.start.assign(nw + 1, 0);
      bk.order.resize(obs.size());
      std::vector<uint16_t> owner(obs.size());
      for (size_t i = 0; i < obs.size(); i++) {
        const uint64_t h = (uint64_t)((uintptr_t)fp[obs[i]] >> 6) * 0x9E3779B97F4A7C15ull;
        owner[i] = (uint16_t)(((h >> 32) * nw) >> 32);
        bk.start[owner[i] + 1]++;
      }
      for (uint32_t w = 0; w < nw; w++) bk.start[w + 1] += bk.start[w];
      std::vector<uint32_t> pos(bk.start.begin(), bk.start.end() - 1);
      for (size_t i = 0; i < obs.size(); i++) bk.order[pos[owner[i]]++] = obs[i];
    };
    auto append = [&](const Buckets &bk, uint32_t w) {
      const uint32_t i0 = bk.start[w], i1 = bk.start[w + 1];
      for (uint32_t i = i0; i < i1; i++) {
        // two-stage software prefetch: the feature object's first three lines (its tracks) 32 ahead, then
        // the append slot of the observation's camera track 16 ahead
        if (i + 32 < i1) {
          const char *p = (const char *)fp[bk.order[i + 32]];
          __builtin_prefetch(p, 1);
          __builtin_prefetch(p + 64, 1);
          __builtin_prefetch(p + 128, 1);
        }
        if (i + 16 < i1) {
          const size_t k2 = bk.order[i + 16];
          for (const CamTrack &c : fp[k2]->tracks)
            if ((int)c.cam == cam_of[k2]) __builtin_prefetch(c.m.v.data() + c.m.v.size(), 1);
        }
        const size_t k = bk.order[i];
        fp[k]->track((size_t)cam_of[k]).m.push_back(FeatMeas{uv[2 * k], uv[2 * k + 1], uvn[2 * k], uvn[2 * k + 1], t});
      }
    };
    Buckets bk_known, bk_fresh;
    {
      HPROF("feed.db.bucket");
      bucket(known, bk_known);
    }
    const size_t db0 = db_.size();
    auto tj0 = clk::now();
    pool_.parallel_for((size_t)nw + 1, 1, [&](size_t b, size_t e) {
      for (size_t w = b; w < e; w++) {
        if (w > 0) {
          append(bk_known, (uint32_t)w - 1);
          continue;
        }
        HPROF("feed.insert");  // on whichever thread takes task 0; no other task touches the profile
        for (uint32_t k : fresh) {
          const size_t id = (size_t)ids[k] + currid_;
          auto it = db_.find(id);  // a new id seen by an earlier camera of this frame
          if (it == db_.end()) it = db_insert(id, new_feature(id));
          fp[k] = it->second.get();
        }
      }
    });
    if (hprof_.on) {
      auto &a = hprof_.acc["feed.db.job"];
      a.first += secs(tj0, clk::now());
      a.second++;
    }
    stock_target_ = std::min<size_t>(3 * (db_.size() - db0) / 2 + 16, 16384);
    hprof_.count("feed.new_features", (double)(db_.size() - db0));
    hprof_.count("feed.obs", (double)nobs);
    hprof_.count("feed.db_size", (double)db_.size());
    if (!fresh.empty()) {
      HPROF("feed.db.fresh");
      bucket(fresh, bk_fresh);
      pool_.parallel_for((size_t)nw, 1, [&](size_t b, size_t e) {
        for (size_t w = b; w < e; w++) append(bk_fresh, (uint32_t)w);
      });
    }
  }
  return after_tracking(t, camids, rT1);
}

// VioManager::feed_measurement_camera -> TrackKLT::feed_new_camera (TrackKLT.cpp:34-94), then the
// same propagate / update sequence as the simulated feed
int Engine::feed_camera(double t, int ncam, const int *cam_ids, const uint8_t *const *imgs, const int *strides,
                        const uint8_t *const *masks, bool device_imgs) {
  auto rT1 = clk::now();
  frame_begin();
  std::vector<int> camids;
  for (int i = 0; i < ncam; i++) {
    int cid = cam_ids[i];
    if (cid < 0 || cid >= o_.num_cameras || !imgs[i]) return UVIO_HP_E_ARG;
    camids.push_back(cid);
  }
  if (!tracker_) {
    tracker_.reset(new Tracker(o_, cams_, d_.stream, &kprof_));
    tracker_->set_host_prof(&hprof_);
  }
  // Propagator::propagate_and_clone reads nothing the tracker produces.  When nothing can run between the
  // tracking and the propagation (no zero-velocity check, no UWB range before t), the host computes it
  // while the frame's LK + RANSAC are on the device and enqueues its launches behind them: the same
  // launches in the same stream order, the host's share hidden under the tracker's wait.
  // An exception of the early propagation is held until the tracker has finished its frame (results
  // consumed, buffers flipped) and rethrown then; its host time is booked as propagation, not tracking.
  bool early = false;
  int early_rc = 0;
  std::exception_ptr early_exc;
  std::function<void()> in_flight;
  early_prop_s_ = 0.0;
  if (propagation_can_precede_tracking(t))
    in_flight = [&, t]() {
      HPROF("prop");
      early = true;
      auto p0 = clk::now();
      try {
        early_rc = propagate_and_clone(t);
      } catch (...) {
        early_exc = std::current_exception();
      }
      early_prop_s_ = secs(p0, clk::now());
    };
  {
    HPROF("track.feed");
    tracker_->feed(
        t, ncam, cam_ids, imgs, strides, masks, device_imgs,
        [this](size_t id, double tt, int cam, float u, float v, float un, float vn) {
          db_update(id, tt, (size_t)cam, u, v, un, vn);
        },
        std::move(in_flight));
  }
  if (early_exc) std::rethrow_exception(early_exc);
  if (early && early_rc) return early_rc;
  struct FrameFlag {
    bool &f;
    explicit FrameFlag(bool &x) : f(x) { f = true; }
    ~FrameFlag() { f = false; }
  } in_camera_frame(camera_frame_);
  return after_tracking(t, camids, rT1, tracker_->device_syncs, tracker_->sync_wait, true);
}

// the conditions under which after_tracking's first state change is propagate_and_clone(t)
bool Engine::propagation_can_precede_tracking(double t) const {
  if (!is_initialized_ || timestamp_ >= t) return false;
  if (o_.try_zupt && (!o_.zupt_only_at_beginning || !has_moved_since_zupt_)) return false;
  for (auto it = past_uwb_.begin(); it != past_uwb_.end() && it->first < t; it++)
    if (it->first > timestamp_) return false;
  return true;
}

int Engine::after_tracking(double t, const std::vector<int> &camids, clk::time_point rT1, int track_syncs,
                           double track_wait, bool try_init) {
  HPROF("after_tracking");
  auto rT2 = clk::now();
  timing_ = uvio_hp_timing_t{};
  frame_feats_.clear();
  timing_.tracking = secs(rT1, rT2) - early_prop_s_;
  timing_.device_syncs = track_syncs;
  timing_.sync_wait = track_wait;
  // VioManager.cpp:308-317: a camera frame before initialization tries the initializer (the simulated
  // feed requires an initialized filter, VioManager.cpp:236-240)
  // The initializer runs single-threaded (use_multi_threading_subs off): on success it sets the state and
  // returns false, so that frame ends uninitialized and the next camera frame finds thread_init_success
  // (VioManagerHelper.cpp:91-93, 187).  The zero-velocity check of that next frame is skipped: it precedes
  // the initialization check and reads is_initialized_vio (VioManager.cpp:294, UVioManager.cpp:152).
  const bool was_initialized = is_initialized_;
  if (!is_initialized_) {
    if (!try_init || !init_success_) {
      if (try_init) try_to_initialize();
      return UVIO_HP_E_STATE;
    }
    is_initialized_ = true;
  }
  // zero-velocity update (UVioManager.cpp:147-162, VioManager.cpp:291-307): on success the frame ends here
  if (was_initialized && o_.try_zupt && (!o_.zupt_only_at_beginning || !has_moved_since_zupt_)) {
    if (timestamp_ != t) did_zupt_update_ = zupt_try_update(t) == 1;
    if (did_zupt_update_) {
      // Propagator / UpdaterZeroVelocity::clean_old_imu_measurements(t + dt - 0.10)
      const double cut = t + calib_dt_->val[0] - 0.10;
      std::lock_guard<std::mutex> lk(imu_mtx_);
      if (cut >= 0) {
        auto old = [&](const ImuSample &a) { return a.t < cut; };
        imu_data_.erase(std::remove_if(imu_data_.begin(), imu_data_.end(), old), imu_data_.end());
        zupt_imu_.erase(std::remove_if(zupt_imu_.begin(), zupt_imu_.end(), old), zupt_imu_.end());
      }
      timing_.zupt = 1;
      timing_.timestamp = t;
      timing_.n_clones = (int)clones_.size();
      timing_.cov_dim = N_;
      timing_.total = secs(rT1, clk::now());
      return 0;
    }
  }
  if (!past_uwb_.empty()) {
    HPROF("uwb");
    for (auto it = past_uwb_.begin(); it != past_uwb_.lower_bound(t); it++) {
      if (it->first < t && it->first > timestamp_) {
        bool valid = false;
        for (auto &r : it->second)
          if (anchors_.count(r.first)) valid = true;
        if (!valid) continue;
        {
          HPROF("uwb.prop");
          if (propagate_uwb(it->first) != 0) continue;
        }
        HPROF("uwb.chain");
        std::vector<std::pair<size_t, double>> rs;
        for (auto &r : it->second)
          if (anchors_.count(r.first)) rs.emplace_back(r.first, r.second);
        uwb_update_message(rs);
      }
    }
    past_uwb_.erase(past_uwb_.begin(), past_uwb_.upper_bound(t));
  }
  int rc = do_feature_propagate_update(t, camids, rT2);
  timing_.total = secs(rT1, clk::now());
  // VioManager.cpp:631-644: one row per frame that ran the whole update, times in the reference's columns
  // (the UWB ranges processed before the propagation land in "propagation", as in UVioManager.cpp:147-188)
  if (rc == 0 && timing_csv_ && timing_.n_clones >= std::min(o_.max_clone_size, 5)) {
    std::fprintf(timing_csv_, "%.15f,%.5f,%.5f,%.5f,", timestamp_ + calib_dt_->val[0], timing_.tracking,
                 timing_.propagation, timing_.msckf_update);
    if (o_.max_slam_features > 0) std::fprintf(timing_csv_, "%.5f,%.5f,", timing_.slam_update, timing_.slam_delayed);
    std::fprintf(timing_csv_, "%.5f,%.5f\n", timing_.marg, timing_.total);
    std::fflush(timing_csv_);
  }
  return rc;
}

// VioManager.cpp:323-651 (rT2: the end of tracking, UVioManager.cpp:147)
int Engine::do_feature_propagate_update(double t, const std::vector<int> &camids, clk::time_point rT2) {
  stage_ = "feature selection";
  if (timestamp_ > t) return UVIO_HP_E_ORDER;
  if (timestamp_ != t) {
    HPROF("prop");
    int rc = propagate_and_clone(t);
    if (rc) return rc;
  }
  // the device queue is in order: propagation runs on while the host builds the update batches
  // (record_timing >= 2 waits here so the stage timings are attributable)
  if (o_.record_timing >= 2) dev_sync();
  auto rT3 = clk::now();
  timing_.timestamp = t;
  timing_.propagation = secs(rT2, rT3) + early_prop_s_;  // + the propagation run during the tracking wait
  early_prop_s_ = 0.0;
  timing_.n_clones = (int)clones_.size();
  timing_.cov_dim = N_;
  if ((int)clones_.size() < std::min(o_.max_clone_size, 5)) return 0;
  if (timestamp_ != t) return 0;
  has_moved_since_zupt_ = true;

  std::vector<FeatP> feats_lost, feats_marg, feats_slam;
  auto t_sel = clk::now();
  // FeatureDatabase::features_not_containing_newer(t, false, true) and features_containing(margtimestep), then
  // VioManager.cpp:377-392's filter of the lost list (a track in one of this frame's cameras, not in the marg
  // list): per-feature flags on the pool, lists built in db_ order
  {
    const bool do_marg = (int)clones_.size() > o_.max_clone_size || (int)clones_.size() > 5;
    const double mt = do_marg ? margtimestep() : 0.0, ts = timestamp_;
    // pointers to the map's values (no shared_ptr copies: a reference-count round trip per feature
    // costs more than the scan at cfg4's database sizes); nothing inserts into db_ during the scan
    std::vector<const FeatP *> all;  // the map's values in db_ order
    std::vector<const Feature *> fs;  // the features themselves (the scan reads no map node)
    all.reserve(db_.size());
    fs.reserve(db_.size());
    {
      HPROF("select.walk");
      for (auto &kv : db_) {
        all.push_back(&kv.second);
        fs.push_back(kv.second.get());
      }
    }
    HPROF("select.flags");
    // each chunk's lost / marg lists built by the thread that flagged it (the reference-count increments
    // then hit lines that thread has just read), joined in chunk order = db_ order
    constexpr size_t kChunk = 1024;
    const size_t nchunk = (all.size() + kChunk - 1) / kChunk;
    std::vector<std::vector<FeatP>> lost_c(nchunk), marg_c(nchunk);
    pool_.parallel_for(all.size(), kChunk, [&](size_t b, size_t e) {
      std::vector<FeatP> &lo = lost_c[b / kChunk], &ma = marg_c[b / kChunk];
      for (size_t i = b; i < e; i++) {
        if (i + 8 < e) __builtin_prefetch(fs[i + 8]);
        const Feature &f = *fs[i];
        if (f.to_delete) continue;
        bool newer = false, has = false;
        for (auto &p : f.tracks) {
          newer = (!p.m.empty() && p.m.last_t() >= ts);
          if (newer) break;
        }
        if (do_marg)
          for (auto &p : f.tracks) {
            has = p.m.contains(mt);  // binary search on an in-order track
            if (has) break;
          }
        bool lost = !newer && !has;
        if (lost) {
          bool found = false;
          for (auto &p : f.tracks)
            if (std::find(camids.begin(), camids.end(), (int)p.cam) != camids.end()) {
              found = true;
              break;
            }
          lost = found;
        }
        if (lost) lo.push_back(*all[i]);
        if (has) ma.push_back(*all[i]);
      }
    });
    HPROF("select.lists");
    size_t nl = 0, nm = 0;
    for (size_t c = 0; c < nchunk; c++) nl += lost_c[c].size(), nm += marg_c[c].size();
    feats_lost.reserve(nl);
    feats_marg.reserve(nm);
    for (size_t c = 0; c < nchunk; c++) {
      std::move(lost_c[c].begin(), lost_c[c].end(), std::back_inserter(feats_lost));
      std::move(marg_c[c].begin(), marg_c[c].end(), std::back_inserter(feats_marg));
    }
    hprof_.count("select.db_size", (double)all.size());
    hprof_.count("select.lost", (double)feats_lost.size());
    hprof_.count("select.marg", (double)feats_marg.size());
  }
  std::vector<FeatP> feats_maxtracks;
  {
    HPROF("select.maxtracks");
    std::vector<FeatP> keep;
    for (auto &f : feats_marg) {
      bool reached = false;
      for (auto &p : f->tracks)
        if ((int)p.m.size() > o_.max_clone_size) {
          reached = true;
          break;
        }
      (reached ? feats_maxtracks : keep).push_back(std::move(f));  // (moves: no reference-count traffic)
    }
    feats_marg = std::move(keep);
  }
  int curr_aruco = 0;
  for (auto &l : slam_)
    if ((int)l.second->featid <= 4 * o_.max_aruco_features) curr_aruco++;
  if (o_.max_slam_features > 0 && t - startup_time_ >= o_.dt_slam_delay &&
      (int)slam_.size() < o_.max_slam_features + curr_aruco) {
    int amount = (o_.max_slam_features + curr_aruco) - (int)slam_.size();
    int valid = std::min(amount, (int)feats_maxtracks.size());
    if (valid > 0) {
      feats_slam.insert(feats_slam.end(), std::make_move_iterator(feats_maxtracks.end() - valid),
                        std::make_move_iterator(feats_maxtracks.end()));
      feats_maxtracks.erase(feats_maxtracks.end() - valid, feats_maxtracks.end());
    }
  }
  for (auto &lm : slam_) {
    auto it = db_.find(lm.second->featid);
    FeatP f2 = (it == db_.end()) ? nullptr : it->second;
    if (f2) feats_slam.push_back(f2);
    bool cur = std::find(camids.begin(), camids.end(), lm.second->unique_cam) != camids.end();
    if (!f2 && cur) lm.second->should_marg = true;
    if (lm.second->fail_count > 1) lm.second->should_marg = true;
  }
  {
    HPROF("select.marg_slam");
    marginalize_slam();
  }
  std::vector<FeatP> slam_delayed, slam_upd;
  for (auto &f : feats_slam) {
    if (slam_.find(f->featid) != slam_.end())
      slam_upd.push_back(f);
    else
      slam_delayed.push_back(f);
  }
  std::vector<FeatP> up = std::move(feats_lost);
  up.insert(up.end(), std::make_move_iterator(feats_marg.begin()), std::make_move_iterator(feats_marg.end()));
  up.insert(up.end(), std::make_move_iterator(feats_maxtracks.begin()), std::make_move_iterator(feats_maxtracks.end()));
  // VioManager.cpp:518 std::sort by measurement count (compare_feat), on the counts computed once: std::sort's
  // permutation depends only on the comparison outcomes, which are the same
  {
    HPROF("select.sort");
    std::vector<std::pair<int, FeatP>> keyed(up.size());
    for (size_t i = 0; i < up.size(); i++) keyed[i] = {up[i]->count(), std::move(up[i])};
    std::sort(keyed.begin(), keyed.end(),
              [](const std::pair<int, FeatP> &a, const std::pair<int, FeatP> &b) { return a.first < b.first; });
    for (size_t i = 0; i < up.size(); i++) up[i] = std::move(keyed[i].second);
  }
  if ((int)up.size() > o_.max_msckf_in_update) up.erase(up.begin(), up.end() - o_.max_msckf_in_update);
  // every feature the updaters may flag to_delete (the MSCKF list, SLAM updates, delayed inits); a
  // frame that returns early keeps its entries for the next frame's cleanup
  pending_delete_.insert(pending_delete_.end(), up.begin(), up.end());
  pending_delete_.insert(pending_delete_.end(), feats_slam.begin(), feats_slam.end());
  timing_.n_msckf = (int)up.size();
  if (hprof_.on) {
    auto &a = hprof_.acc["select"];
    a.first += secs(t_sel, clk::now());
    a.second++;
  }
  timing_.n_slam_delayed = (int)slam_delayed.size();
  int rc = 0;
  auto rT4 = clk::now(), rT5 = rT4, rT6 = rT4;
  // FeatureDatabase::cleanup_measurements(margtimestep) of every feature the updaters do not read runs while
  // the device executes the chain: one feature's trimming is independent of the others', nothing between
  // the updates and the cleanup reads the trimmed (older than the marginalized clone) measurements of an
  // unread feature, and erasing a node keeps the other nodes' iteration order.  The held features (every
  // one handed to an updater, pending_delete_) are trimmed at the reference's point, after the chain.
  const bool do_clean = (int)clones_.size() > o_.max_clone_size;
  const double mt_clean = do_clean ? margtimestep() : 0.0;
  bool cleaned_early = false;
  std::vector<FeatP> held;
  // on every exit (a returned error or an exception included): no overlap job left behind, no feature held
  struct HeldGuard {
    Engine &e;
    std::vector<FeatP> &h;
    ~HeldGuard() {
      e.chain_overlap_ = nullptr;
      for (auto &f : h) f->held = false;
    }
  } held_guard{*this, held};
  // the chain also carries the feature-sharded MSCKF update: over RCCL its all-reduce is enqueued; the host
  // all-reduce (a callback, for ranks that share a GPU) waits for this rank's Gram in the middle of the enqueueing
  if (!no_chain_) {
    if (do_clean) {
      held = pending_delete_;
      for (auto &f : held) f->held = true;
      chain_overlap_ = [this, mt_clean, &cleaned_early]() {
        cleanup_measurements(mt_clean, true);
        cleaned_early = true;
      };
    }
    // the three updaters as one device chain with one host wait (engine_chain.cpp)
    rc = update_frame(up, slam_upd, slam_delayed);
    chain_overlap_ = nullptr;
    if (rc) return rc;
    rT6 = clk::now();
    timing_.msckf_update = chain_times_[0];
    timing_.slam_update = chain_times_[1];
    timing_.slam_delayed = chain_times_[2];
  } else {
    rc = msckf_update(up);
    if (rc) return rc;
    rT4 = clk::now();
    while (!slam_upd.empty()) {
      size_t k = std::min((size_t)std::max(o_.max_slam_in_update, 1), slam_upd.size());
      std::vector<FeatP> tmp(slam_upd.begin(), slam_upd.begin() + k);
      slam_upd.erase(slam_upd.begin(), slam_upd.begin() + k);
      rc = slam_update(tmp);
      if (rc) return rc;
    }
    rT5 = clk::now();
    rc = slam_delayed_init(slam_delayed);
    if (rc) return rc;
    rT6 = clk::now();
    timing_.msckf_update = secs(rT3, rT4);
    timing_.slam_update = secs(rT4, rT5);
    timing_.slam_delayed = secs(rT5, rT6);
  }
  HPROF("marg.total");
  {
    HPROF("marg.retri");
    retriangulate_active_tracks(t, camids);
  }
  for (auto &f : up) f->to_delete = true;
  // FeatureDatabase::cleanup: only features handed to an updater can carry to_delete, so they are
  // erased by key (erasing a node keeps the others' iteration order, as the reference's scan does)
  for (auto &f : pending_delete_) {
    if (!f->to_delete) continue;
    auto it = db_.find(f->featid);
    if (it != db_.end() && it->second == f) db_erase(it);
  }
  pending_delete_.clear();
  {
    HPROF("marg.anchors");
    rc = slam_change_anchors();
  }
  if (rc) return rc;
  if (do_clean) {
    HPROF("marg.cleanmeas");
    if (!cleaned_early) {
      cleanup_measurements(mt_clean, false);
    } else {
      for (auto &f : held) {  // the chain's features still in the database
        auto it = db_.find(f->featid);
        if (it == db_.end() || it->second != f) continue;
        f->clean_older_measurements(mt_clean);
        if (f->count() < 1) db_erase(it);
      }
    }
  }
  marginalize_old_clone();
  if (o_.record_timing >= 2) dev_sync();
  auto rT7 = clk::now();
  timing_.marg = secs(rT6, rT7);
  timing_.n_slam = (int)slam_.size();
  timing_.cov_dim = N_;
  if (kprof_.on) kprof_.harvest(false);
  if (timelastupdate_ != -1 && clones_.find(timelastupdate_) != clones_.end()) {
    const double *a = imu_->val + 4, *b = clones_.at(timelastupdate_)->val + 4;
    double d[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
    distance_ += norm3(d);
  }
  timelastupdate_ = t;
  return 0;
}

// FeatureDatabase::cleanup_measurements (FeatureDatabase.cpp:226-243): per-feature trimming on the pool, then
// the emptied features are erased (erasing by key keeps the others' iteration order)
void Engine::cleanup_measurements(double t, bool skip_held) {
  const std::vector<Feature *> all(dense_);  // (a copy: the erasures below reorder dense_)
  std::vector<uint8_t> empty(all.size(), 0);
  pool_.parallel_for(all.size(), 1024, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; i++) {
      if (i + 8 < e) __builtin_prefetch(all[i + 8], 1);
      if (skip_held && all[i]->held) continue;
      all[i]->clean_older_measurements(t);
      empty[i] = all[i]->count() < 1;
    }
  });
  for (size_t i = 0; i < all.size(); i++)
    if (empty[i]) db_erase(db_.find(all[i]->featid));
}

// StateHelper::marginalize_slam (StateHelper.cpp:631-645)
// (the landmarks of one call leave the covariance in one launch, marginalize_many)
void Engine::marginalize_slam() {
  stage_ = "marginalize_slam";
  std::vector<VarP> ms;
  for (auto it = slam_.begin(); it != slam_.end();) {
    if (it->second->should_marg && (int)it->first > 4 * o_.max_aruco_features) {
      ms.push_back(it->second);
      it = slam_.erase(it);
    } else {
      it++;
    }
  }
  marginalize_many(ms);
}

// StateHelper::marginalize_old_clone (StateHelper.cpp:618-629)
void Engine::marginalize_old_clone() {
  stage_ = "marginalize_old_clone";
  if ((int)clones_.size() > o_.max_clone_size) {
    double mt = margtimestep();
    marginalize(clones_.at(mt));
    clones_.erase(mt);
  }
}

// ---------------------------------------------------------------------------------------------------
// Batch tables: clone slots (time order), cameras, canonical columns (calib blocks, clones, landmarks)
void Engine::build_clone_cam_tables(Batch &b, bool include_landmarks) {
  b.clones.clear();
  b.cams.clear();
  b.hidx.clear();
  b.slot_of_time.clear();
  int canon = 0;
  for (int c = 0; c < o_.num_cameras; c++) {
    DCam dc{};
    const VarP &pose = calib_pose_.at(c);
    quat_2_Rot(pose->val, dc.R_ItoC);
    for (int k = 0; k < 3; k++) dc.p_IinC[k] = pose->val[4 + k];
    dc.cam = cams_[c];
    dc.pid_ext = o_.do_calib_camera_pose ? pose->id : -1;
    dc.pid_intr = o_.do_calib_camera_intrinsics ? calib_intr_.at(c)->id : -1;
    dc.canon_ext = dc.canon_intr = -1;
    if (o_.do_calib_camera_pose) {
      dc.canon_ext = canon;
      for (int k = 0; k < 6; k++) b.hidx.push_back(pose->id + k);
      canon += 6;
    }
    if (o_.do_calib_camera_intrinsics) {
      dc.canon_intr = canon;
      for (int k = 0; k < 8; k++) b.hidx.push_back(calib_intr_.at(c)->id + k);
      canon += 8;
    }
    b.cams.push_back(dc);
  }
  for (auto &c : clones_) {
    DClone d{};
    quat_2_Rot(c.second->val, d.R);
    quat_2_Rot(c.second->fej, d.Rf);
    for (int k = 0; k < 3; k++) d.p[k] = c.second->val[4 + k], d.pf[k] = c.second->fej[4 + k];
    d.pid = c.second->id;
    d.canon = canon;
    for (int k = 0; k < 6; k++) b.hidx.push_back(c.second->id + k);
    canon += 6;
    b.slot_of_time.push(c.first);  // slot = index in time order
    b.clones.push_back(d);
  }
  (void)include_landmarks;
  b.n_canon = canon;
}

// Builds the per-feature measurement / variable tables in the reference iteration order
// (get_feature_jacobian_full's x_order, UpdaterHelper.cpp:200-262) and appends them to the batch.
void add_feature(Engine *, const FeatP &f, int mode, int rep, const uvio_hp_options_t &o, const std::vector<DCam> &cams,
                        const SlotTable &slot_of_time, const std::vector<DClone> &clones, std::vector<DFeat> &feats,
                        std::vector<DMeas> &meas, std::vector<DVar> &vars, int &rows, const Var *landmark,
                        int landmark_canon) {
  DFeat F{};
  F.meas_off = (int)meas.size();
  F.var_off = (int)vars.size();
  F.rep = rep;
  F.mode = mode;
  // anchor (FeatureInitializer.cpp:35-45): camera with most measurements (first max in map order),
  // anchor time = its last measurement
  size_t anchor_cam = 0, most = 0;
  for (auto &p : f->tracks)
    if (p.m.size() > most) {
      anchor_cam = p.cam;
      most = p.m.size();
    }
  const CamTrack *at = f->find(anchor_cam);
  if (!at || at->m.empty()) throw HpError(UVIO_HP_E_STATE, "feature without measurements in a batch");
  double anchor_time = at->m.back().t;
  if (landmark) {
    anchor_cam = (size_t)landmark->anchor_cam;
    anchor_time = landmark->anchor_time;
  }
  F.anchor_cam = (int)anchor_cam;
  const bool rel = (rep == 2 || rep == 3 || rep == 4 || rep == 5);
  // a global landmark's anchor clone may have been marginalized (change_anchors only re-anchors relative
  // representations, UpdaterSLAM.cpp:481-500) and get_feature_jacobian_full never reads it for a global
  // representation (UpdaterHelper.cpp:226-262): slot 0 is a placeholder the kernel does not use
  const int anc = slot_of_time.find(anchor_time);
  if (anc < 0 && (rel || !landmark)) throw HpError(UVIO_HP_E_STATE, "feature anchor clone is not in the window");
  F.anchor_slot = (anc < 0) ? 0 : anc;
  int loc = 0;
  std::vector<int> clone_loc(clones.size(), -1);  // slot -> local col
  int ext_loc[UVIO_HP_MAX_CAMS], intr_loc[UVIO_HP_MAX_CAMS];
  for (int k = 0; k < UVIO_HP_MAX_CAMS; k++) ext_loc[k] = intr_loc[k] = -1;
  for (auto &p : f->tracks) {
    int c = (int)p.cam;
    if (o.do_calib_camera_pose) {
      vars.push_back(DVar{cams[c].pid_ext, cams[c].canon_ext, 6, loc});
      ext_loc[c] = loc;
      loc += 6;
    }
    if (o.do_calib_camera_intrinsics) {
      vars.push_back(DVar{cams[c].pid_intr, cams[c].canon_intr, 8, loc});
      intr_loc[c] = loc;
      loc += 8;
    }
    for (size_t m = 0; m < p.m.size(); m++) {
      int s = slot_of_time.at(p.m[m].t);
      if (clone_loc[s] < 0) {
        clone_loc[s] = loc;
        vars.push_back(DVar{clones[s].pid, clones[s].canon, 6, loc});
        loc += 6;
      }
    }
  }
  if (rel) {
    if (clone_loc[F.anchor_slot] < 0) {
      clone_loc[F.anchor_slot] = loc;
      vars.push_back(DVar{clones[F.anchor_slot].pid, clones[F.anchor_slot].canon, 6, loc});
      loc += 6;
    }
    if (o.do_calib_camera_pose && ext_loc[F.anchor_cam] < 0) {
      ext_loc[F.anchor_cam] = loc;
      vars.push_back(DVar{cams[F.anchor_cam].pid_ext, cams[F.anchor_cam].canon_ext, 6, loc});
      loc += 6;
    }
    F.lc_anchor_clone = clone_loc[F.anchor_slot];
    F.lc_anchor_ext = ext_loc[F.anchor_cam];
  }
  if (landmark) {
    F.lm_pid = landmark->id;
    F.lm_loc = loc;
    vars.push_back(DVar{landmark->id, landmark_canon, landmark->size, loc});
    loc += landmark->size;
    double p[3], pf[3];
    landmark->xyz(false, p);
    landmark->xyz(true, pf);
    for (int k = 0; k < 3; k++) F.p_in[k] = p[k], F.p_in_fej[k] = pf[k];
  }
  F.nf = loc;
  F.nvar = (int)vars.size() - F.var_off;
  for (auto &p : f->tracks) {
    int c = (int)p.cam;
    for (size_t m = 0; m < p.m.size(); m++) {
      const FeatMeas &fm = p.m[m];
      DMeas d{};
      d.u = fm.u;
      d.v = fm.v;
      d.un = fm.un;
      d.vn = fm.vn;
      d.cam = c;
      d.slot = slot_of_time.at(fm.t);
      d.lc_clone = clone_loc[d.slot];
      d.lc_ext = ext_loc[c];
      d.lc_intr = intr_loc[c];
      meas.push_back(d);
    }
  }
  F.nmeas = (int)meas.size() - F.meas_off;
  F.row_off = rows;
  rows += (mode == 0) ? 2 * F.nmeas - 3 : 2 * F.nmeas;
  feats.push_back(F);
}

void Engine::add_feature_to_batch(Batch &b, const FeatP &f, int mode, int rep) {
  if (b.meas_dev) throw HpError(UVIO_HP_E_INTERNAL, "add_feature_to_batch: measurements already staged");
  add_feature(this, f, mode, rep, o_, b.cams, b.slot_of_time, b.clones, b.feats, b.meas, b.vars, b.rows, nullptr, -1);
}

// fv[lo, hi) appended in order.  Large batches (configs 4-5: 800-1500 features x 26-31 clones) are built
// in contiguous chunks on the pool (add_feature only reads the batch's clone / camera tables), then the
// chunks are stitched in order with their offsets shifted: the same tables as the sequential loop.
void Engine::add_features_to_batch(Batch &b, const std::vector<FeatP> &fv, size_t lo, size_t hi, int mode, int rep) {
  const size_t nf = hi - lo;
  if (nf < 256 || pool_.threads() == 1) {
    for (size_t i = lo; i < hi; i++) add_feature_to_batch(b, fv[i], mode, rep);
    return;
  }
  struct Part {
    std::vector<DFeat> feats;
    std::vector<DMeas> meas;
    std::vector<DVar> vars;
    int rows = 0;
  };
  const size_t nparts = std::min(nf / 64, (size_t)pool_.threads() * 4);
  std::vector<Part> parts(nparts);
  pool_.parallel_for(nparts, 1, [&](size_t p0, size_t p1) {
    for (size_t p = p0; p < p1; p++) {
      Part &P = parts[p];
      const size_t a = lo + nf * p / nparts, e = lo + nf * (p + 1) / nparts;
      for (size_t i = a; i < e; i++)
        add_feature(this, fv[i], mode, rep, o_, b.cams, b.slot_of_time, b.clones, P.feats, P.meas, P.vars, P.rows,
                    nullptr, -1);
    }
  });
  // the parts' measurement / variable tables go straight into the upload staging, copied in parallel
  // (no merged host copy); the batch must not hold host tables already
  if (!b.meas.empty() || !b.vars.empty() || b.meas_dev)
    throw HpError(UVIO_HP_E_INTERNAL, "add_features_to_batch: batch already holds measurements");
  std::vector<size_t> mo(nparts + 1, 0), vo(nparts + 1, 0);
  for (size_t p = 0; p < nparts; p++) {
    mo[p + 1] = mo[p] + parts[p].meas.size();
    vo[p + 1] = vo[p] + parts[p].vars.size();
  }
  // ONE reservation for both tables, filled before anything else is staged: a second reservation could
  // flush and recycle the ring while the first one is still unfilled
  const size_t mbytes = (sizeof(DMeas) * mo[nparts] + 255) / 256 * 256;
  void *hm = nullptr;
  char *dm = (char *)stage_reserve(mbytes + sizeof(DVar) * vo[nparts], &hm);
  void *hv = (char *)hm + mbytes;
  b.meas_dev = (const DMeas *)dm;
  b.vars_dev = (const DVar *)(dm + mbytes);
  b.stg_epoch = d_.stg_epoch;
  b.n_meas_dev = mo[nparts];
  b.n_vars_dev = vo[nparts];
  pool_.parallel_for(nparts, 1, [&](size_t p0, size_t p1) {
    for (size_t p = p0; p < p1; p++) {
      if (!parts[p].meas.empty())
        std::memcpy((DMeas *)hm + mo[p], parts[p].meas.data(), sizeof(DMeas) * parts[p].meas.size());
      if (!parts[p].vars.empty())
        std::memcpy((DVar *)hv + vo[p], parts[p].vars.data(), sizeof(DVar) * parts[p].vars.size());
    }
  });
  for (size_t p = 0; p < nparts; p++) {
    const int ro = b.rows;
    for (DFeat F : parts[p].feats) {
      F.meas_off += (int)mo[p];
      F.var_off += (int)vo[p];
      F.row_off += ro;
      b.feats.push_back(F);
    }
    b.rows += parts[p].rows;
  }
}

DBatchParams Engine::batch_params(const Batch &b, double sigma_pix_sq, double chi2_mult) const {
  DBatchParams bp{};
  bp.nfeat = (int)b.feats.size();
  bp.n_canon = b.n_canon;
  bp.ldh = d_.ldh;
  bp.ldp = d_.ldp;
  bp.sigma_pix_sq = sigma_pix_sq;
  bp.chi2_mult = chi2_mult;
  bp.do_fej = o_.do_fej;
  bp.calib_ext = o_.do_calib_camera_pose;
  bp.calib_intr = o_.do_calib_camera_intrinsics;
  bp.fi_max_runs = o_.fi_max_runs;
  bp.fi_refine = o_.fi_refine_features;
  bp.fi_tri1d = o_.fi_triangulate_1d;
  bp.fi_init_lamda = o_.fi_init_lamda;
  bp.fi_max_lamda = o_.fi_max_lamda;
  bp.fi_min_dx = o_.fi_min_dx;
  bp.fi_min_dcost = o_.fi_min_dcost;
  bp.fi_lam_mult = o_.fi_lam_mult;
  bp.fi_min_dist = o_.fi_min_dist;
  bp.fi_max_dist = o_.fi_max_dist;
  bp.fi_max_baseline = o_.fi_max_baseline;
  bp.fi_max_cond = o_.fi_max_cond_number;
  return bp;
}

// Upload a batch, run the per-feature kernel and (optionally) compression; results in outs.
// Returns the number of stacked rows written to H_all.
int Engine::run_batch(Batch &b, int mode, double sigma_pix_sq, double chi2_mult, bool wait, std::vector<DFeatOut> &outs,
                      bool chi2) {
  int nf = (int)b.feats.size();
  if (nf == 0) return 0;
  b.chi2 = chi2;
  if (nf > d_.max_feat || (int)b.n_meas() > d_.max_meas_total || (int)b.n_vars() > d_.max_vars_total ||
      b.rows > d_.max_rows || b.n_canon + 1 > d_.max_ncol)
    throw HpError(UVIO_HP_E_CAPACITY, "update batch exceeds device capacity");
  int max_meas = 0, max_nf = 0;
  for (auto &F : b.feats) {
    max_meas = std::max(max_meas, F.nmeas);
    max_nf = std::max(max_nf, F.nf);
  }
  if (max_meas > kMaxMeasPerFeat) throw HpError(UVIO_HP_E_CAPACITY, "too many measurements per feature");
  size_t lds = feature_lds_bytes(max_meas, max_nf);
  if (lds + 4096 > 160 * 1024) throw HpError(UVIO_HP_E_CAPACITY, "feature LDS footprint too large");
  // the batch tables go up packed in one copy
  const DFeat *t_feats = stage(b.feats.data(), b.feats.size());
  const DMeas *t_meas = b.meas_dev ? b.meas_dev : stage(b.meas.data(), b.meas.size());
  const DVar *t_vars = b.vars_dev ? b.vars_dev : stage(b.vars.data(), b.vars.size());
  const DClone *t_clones = stage(b.clones.data(), b.clones.size());
  const DCam *t_cams = stage(b.cams.data(), b.cams.size());
  const int *t_hidx = stage(b.hidx.data(), b.hidx.size());
  stage_flush();
  // the measurement / variable reservation must still be intact: after a ring restart in between, the
  // tables staged since then start at offset 0 and must end before the reservation (a ring smaller than
  // one launch group, UVIO_HP_STAGE_BYTES, would let them overwrite it on the device)
  if (b.meas_dev && b.stg_epoch != d_.stg_epoch && d_.stg_used > (size_t)((const char *)b.meas_dev - d_.stg_d))
    throw HpError(UVIO_HP_E_CAPACITY, "upload staging ring restarted inside one launch group (UVIO_HP_STAGE_BYTES too small)");
  b.hidx_dev = t_hidx;
  DBatchParams bp = batch_params(b, sigma_pix_sq, chi2_mult);
  const char *mdump = (mode == 0) ? std::getenv("UVIO_HP_MEAS_DUMP") : nullptr;  // debug only
  if (mdump) HP_HIP(hipMalloc(&bp.dbg, sizeof(double) * 8 * b.n_meas()));
  const char *tsdump = std::getenv("UVIO_HP_FEAT_TS");  // debug only: per-feature phase cycle counts
  if (tsdump) {  // 8 k_feature phases + 4 k_chi2 phases per feature
    HP_HIP(hipMalloc(&bp.dbg_ts, sizeof(long long) * 16 * nf));
    HP_HIP(hipMemset(bp.dbg_ts, 0, sizeof(long long) * 16 * nf));
  }
  // the feature group's event pair only while kernel timing is on: a timing event between the upload and
  // k_feature costs a dispatch gap on every batch
  b.evtimed = o_.record_timing && kprof_.on;
  if (b.evtimed) HP_HIP(hipEventRecord(d_.ev0, d_.stream));
  {
    KScope ks(&kprof_, KC_FEATURE);
    launch_feature_linearize(d_.stream, bp, t_feats, t_meas, t_vars, t_clones, t_cams, d_.P, d_.chi2, d_.H, d_.fout,
                             max_meas, max_nf);
  }
  if (chi2) {
    int max_rows_f = 0;
    for (auto &F : b.feats) {
      int rows_out = (mode == 0) ? 2 * F.nmeas - 3 : 2 * F.nmeas;
      max_rows_f = std::max(max_rows_f, rows_out - (mode >= 2 ? 3 : 0));
    }
    KScope ks(&kprof_, KC_CHI2);
    // d_.R (the information-form Gram buffer, 2 max_ncol ldh doubles) holds the gathered P_can until the
    // T GEMM has read it; the Gram reduce writes it only later on the same stream
    launch_chi2_batch(d_.stream, bp, t_feats, d_.P, t_hidx, d_.H, b.rows, d_.Tall, d_.chi2, d_.fout,
                      max_rows_f, d_.acc, d_.R, &d_.chi2S, &d_.chi2S_cap);
  }
  if (b.evtimed) HP_HIP(hipEventRecord(d_.ev1, d_.stream));
  d_.fout_pending = nf;  // copied with the next readback (read_dx) or before the next wait (dev_sync)
  if (!wait && !tsdump && !mdump) return b.rows;  // the caller's next sync completes the batch (finish_batch)
  dev_sync();
  finish_batch(b, mode, outs);
  if (tsdump) {
    std::vector<long long> h(16 * (size_t)nf);
    HP_HIP(hipMemcpy(h.data(), bp.dbg_ts, sizeof(long long) * h.size(), hipMemcpyDeviceToHost));
    HP_HIP(hipFree(bp.dbg_ts));
    FILE *fp = std::fopen(tsdump, "ab");
    for (int i = 0; i < nf; i++) {
      long long rec[16] = {mode, nf, b.feats[i].nmeas, b.feats[i].nf};
      for (int k = 0; k < 12; k++) rec[4 + k] = h[16 * (size_t)i + k];
      std::fwrite(rec, sizeof(long long), 16, fp);
    }
    std::fclose(fp);
  }
  if (mdump) {
    std::vector<double> h(8 * b.n_meas());
    HP_HIP(hipMemcpy(h.data(), bp.dbg, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
    HP_HIP(hipFree(bp.dbg));
    FILE *fp = std::fopen(mdump, "ab");
    for (int i = 0; i < nf; i++) {
      if (outs[i].status != 0) continue;
      for (int k = 0; k < b.feats[i].nmeas; k++) {
        double fid = (double)i;
        std::fwrite(&fid, sizeof(double), 1, fp);
        std::fwrite(h.data() + 8 * (size_t)(b.feats[i].meas_off + k), sizeof(double), 8, fp);
      }
    }
    std::fclose(fp);
  }
  return b.rows;
}

// per-feature results of a batch whose readback has completed (after a device sync), plus the feature
// group's event timing
void Engine::finish_batch(Batch &b, int mode, std::vector<DFeatOut> &outs) {
  const int nf = (int)b.feats.size();
  outs.assign(d_.fout_host + b.fout_off, d_.fout_host + b.fout_off + nf);
  if (b.finished) return;
  b.finished = true;
  if (b.evtimed) {
    float ms = 0.f;
    HP_HIP(hipEventElapsedTime(&ms, d_.ev0, d_.ev1));
    timing_.k_feat_launches += 1;
    timing_.k_feat_s += 1e-3 * ms;
    // algorithmic FP64 FLOPs (SURVEY.md §8(d) F_feat) of the features that reached the projection
    for (int i = 0; i < nf && mode != 2; i++) {  // mode 2 triangulates only
      if (outs[i].status == 1 || outs[i].status == 2) continue;
      double rows = 2.0 * b.feats[i].nmeas, nfc = b.feats[i].nf;
      double r = (mode == 1) ? rows : rows - 3.0;
      double refl = (mode == 1) ? 0.0 : 12.0 * rows * (nfc + 4.0);
      const double chi2 = b.chi2 ? 2.0 * r * nfc * nfc + 2.0 * r * r * nfc + r * r * r / 3.0 : 0.0;
      timing_.k_feat_flops += refl + chi2;
    }
  }
  if (kprof_.on) {
    // the same F_feat split by class: reflections -> k_feature, the chi2 terms -> the chi2 group; bytes =
    // the rows each writes (k_feature) / reads with their T rows (chi2) plus the P block gathered
    double fl = 0, fb = 0, cl = 0, cb = 0;
    for (int i = 0; i < nf; i++) {
      const double rows = 2.0 * b.feats[i].nmeas, nfc = b.feats[i].nf;
      fb += 8.0 * (rows * (nfc + 1) + 4.0 * b.feats[i].nmeas);
      if (mode == 2 || outs[i].status == 1 || outs[i].status == 2) continue;
      const double r = (mode == 1) ? rows : rows - 3.0;
      if (mode != 1) fl += 12.0 * rows * (nfc + 4.0);
      if (b.chi2) {
        cl += 2.0 * r * nfc * nfc + 2.0 * r * r * nfc + r * r * r / 3.0;
        cb += 8.0 * (2.0 * r * (nfc + 1) + nfc * nfc);
      }
    }
    kprof_.credit(KC_FEATURE, fl, fb);
    if (b.chi2) kprof_.credit(KC_CHI2, cl, cb);
  }
}

// the Gram [H r]^T [H r] of the m stacked rows in H_all (upper triangle: m ncol (ncol + 1) FLOPs, H read once)
void Engine::gram(int m, int ncol, int *nch) {
  {
    KScope ks(&kprof_, KC_GRAM);
    launch_gram(d_.stream, d_.H, m, ncol, d_.ldh, d_.partials, nch);
  }
  kprof_.credit(KC_GRAM, (double)m * ncol * (ncol + 1), 8.0 * ((double)m * ncol + (double)*nch * ncol * ncol));
}

// UpdaterMSCKF::update (UpdaterMSCKF.cpp:58-295)
int Engine::msckf_update(std::vector<FeatP> &fv) {
  stage_ = "UpdaterMSCKF::update";
  last_msckf_.clear();
  if (fv.empty()) return 0;
  HPROF("msckf.total");
  std::vector<double> clonetimes;
  for (auto &c : clones_) clonetimes.push_back(c.first);
  std::vector<uint8_t> few(fv.size());
  pool_.parallel_for(fv.size(), 64, [&](size_t b0, size_t e0) {
    for (size_t i = b0; i < e0; i++) {
      fv[i]->clean_old_measurements(clonetimes);
      few[i] = fv[i]->count() < 2;
    }
  });
  std::vector<FeatP> keep;
  for (size_t i = 0; i < fv.size(); i++) {
    if (few[i])
      fv[i]->to_delete = true;
    else
      keep.push_back(fv[i]);
  }
  fv = keep;
  if (fv.empty()) return 0;
  if (o_.feat_rep_msckf != 0 && o_.feat_rep_msckf != 4)
    throw HpError(UVIO_HP_E_CONFIG, "feat_rep_msckf: only GLOBAL_3D / ANCHORED_MSCKF_INVERSE_DEPTH are implemented");
  if (shard_.enabled && (int)fv.size() >= shard_.min_features) return msckf_update_sharded(fv);
  Batch b;
  {
    HPROF("msckf.build");
    build_clone_cam_tables(b, false);
    add_features_to_batch(b, fv, 0, fv.size(), 0, o_.feat_rep_msckf);
  }
  // compressed (information-form) update ahead: its P_II factor and V start now, beside the feature group
  PrefactorJoin pj(this);
  if (b.rows > b.n_canon || b.rows > kMaxEkfRows) info_prefactor(b.hidx);
  // The update is enqueued right behind the feature group: rejected features already have zero rows in
  // H_all and the device skips the P update when no feature was accepted (d_.acc), so the host reads the
  // per-feature results with the update's dx instead of waiting for them in between.
  std::vector<DFeatOut> outs;
  const double s2 = o_.msckf_sigma_pix * o_.msckf_sigma_pix;
  int m;
  {
    HPROF("msckf.run_batch");
    m = run_batch(b, 0, s2, o_.msckf_chi2_multipler, false, outs);
  }
  const int n = b.n_canon, ncol = n + 1;
  auto results = [&]() {
    HPROF("msckf.results");
    finish_batch(b, 0, outs);
    int acc = 0, acc_rows = 0;
    for (size_t i = 0; i < outs.size(); i++) {
      last_msckf_.push_back(FeatDebug{fv[i]->featid, {outs[i].p_FinG[0], outs[i].p_FinG[1], outs[i].p_FinG[2]},
                                      outs[i].status == 2 ? 1 : outs[i].status, outs[i].chi2});
      frame_feats_.push_back({0, last_msckf_.back()});
      fv[i]->to_delete = true;
      for (int k = 0; k < 3; k++) fv[i]->p_FinG[k] = outs[i].p_FinG[k], fv[i]->p_FinA[k] = outs[i].p_FinA[k];
      if (outs[i].status == 0) acc++, acc_rows += outs[i].rows;
    }
    timing_.msckf_rows = acc_rows;
    timing_.msckf_cols = b.n_canon;
    if (const char *dump = std::getenv("UVIO_HP_DUMP")) {  // debug: projected rows per feature
      int nc = b.n_canon + 1;
      std::vector<double> Hh((size_t)std::max(m, 1) * nc);
      if (m > 0)
        HP_HIP(hipMemcpy2D(Hh.data(), sizeof(double) * nc, d_.H, sizeof(double) * d_.ldh, sizeof(double) * nc, m,
                           hipMemcpyDeviceToHost));
      FILE *fp = std::fopen(dump, "ab");
      for (size_t i = 0; i < outs.size(); i++) {
        if (outs[i].status != 0) continue;
        std::vector<double> hdr = {(double)fv[i]->featid, (double)outs[i].rows, (double)b.n_canon};
        for (int j = 0; j < b.n_canon; j++) hdr.push_back(b.hidx[j]);
        std::fwrite(hdr.data(), sizeof(double), hdr.size(), fp);
        std::fwrite(Hh.data() + (size_t)b.feats[i].row_off * nc, sizeof(double), (size_t)outs[i].rows * nc, fp);
      }
      std::fclose(fp);
    }
    return acc > 0;
  };
  if (m < 1) {
    dev_sync();
    results();
    return 0;
  }
  if (m > n || m > kMaxEkfRows) {
    // measurement compression (UpdaterHelper.cpp:456-487) + EKFUpdate on the compressed system, carried
    // out in information form on G = [H r]^T [H r] (see launch_ekf_info)
    int nch = 0;
    gram(m, ncol, &nch);
    ekf_update_info(nch, n, b.hidx, s2, results, d_.acc);
  } else {
    ekf_update_rows(d_.H, d_.ldh, m, n, b.hidx, d_.H + n, d_.ldh, s2, b.hidx_dev, results, d_.acc, d_.Tall);
  }
  return 0;
}

// UpdaterSLAM::update (UpdaterSLAM.cpp:253-479)
int Engine::slam_update(std::vector<FeatP> &fv) {
  stage_ = "UpdaterSLAM::update";
  if (fv.empty()) return 0;
  std::vector<double> clonetimes;
  for (auto &c : clones_) clonetimes.push_back(c.first);
  std::vector<FeatP> keep;
  for (auto &f : fv) {
    f->clean_old_measurements(clonetimes);
    int ct = f->count();
    if (ct < 1)
      f->to_delete = true;
    else
      keep.push_back(f);
  }
  fv = keep;
  if (fv.empty()) return 0;
  Batch b;
  build_clone_cam_tables(b, true);
  // landmark columns appended to the canonical set
  std::vector<int> lm_canon;
  for (auto &f : fv) {
    const VarP &lm = slam_.at(f->featid);
    lm_canon.push_back(b.n_canon);
    for (int k = 0; k < lm->size; k++) b.hidx.push_back(lm->id + k);
    b.n_canon += lm->size;
  }
  for (size_t i = 0; i < fv.size(); i++) {
    const VarP &lm = slam_.at(fv[i]->featid);
    if (lm->rep != 0 && lm->rep != 2 && lm->rep != 4)
      throw HpError(UVIO_HP_E_CONFIG, "feat_rep_slam: representation not implemented");
    add_feature(this, fv[i], 1, lm->rep, o_, b.cams, b.slot_of_time, b.clones, b.feats, b.meas, b.vars, b.rows,
                lm.get(), lm_canon[i]);
  }
  // enqueued behind the feature group as in msckf_update (rejected rows are zero, d_.acc gates P)
  PrefactorJoin pj(this);
  if (b.rows > b.n_canon || b.rows > kMaxEkfRows) info_prefactor(b.hidx);
  std::vector<DFeatOut> outs;
  const double s2 = o_.slam_sigma_pix * o_.slam_sigma_pix;
  const int m = run_batch(b, 1, s2, o_.slam_chi2_multipler, false, outs);
  const int n = b.n_canon, ncol = n + 1;
  last_upd_.clear();
  auto results = [&]() {
    finish_batch(b, 1, outs);
    int acc = 0;
    for (size_t i = 0; i < outs.size(); i++) {
      last_upd_.push_back(FeatDebug{fv[i]->featid, {0.0, 0.0, 0.0}, outs[i].status == 2 ? 1 : outs[i].status, outs[i].chi2});
      frame_feats_.push_back({1, last_upd_.back()});
      fv[i]->to_delete = true;
      if (outs[i].status == 3) slam_.at(fv[i]->featid)->fail_count++;
      if (outs[i].status == 0) acc++;
    }
    return acc > 0;
  };
  if (m < 1) {
    dev_sync();
    results();
    return 0;
  }
  if (m > n || m > kMaxEkfRows) {
    int nch = 0;
    gram(m, ncol, &nch);
    ekf_update_info(nch, n, b.hidx, s2, results, d_.acc);
  } else {
    ekf_update_rows(d_.H, d_.ldh, m, n, b.hidx, d_.H + n, d_.ldh, s2, b.hidx_dev, results, d_.acc, d_.Tall);
  }
  return 0;
}

// UpdaterSLAM::delayed_init (UpdaterSLAM.cpp:61-251) + StateHelper::initialize (StateHelper.cpp:393-482).
// Triangulation of the whole batch runs first (as in the reference); each accepted landmark then
// initializes and updates the state before the next one is linearized.
int Engine::slam_delayed_init(std::vector<FeatP> &fv) {
  stage_ = "UpdaterSLAM::delayed_init";
  if (fv.empty()) return 0;
  std::vector<double> clonetimes;
  for (auto &c : clones_) clonetimes.push_back(c.first);
  std::vector<FeatP> keep;
  for (auto &f : fv) {
    f->clean_old_measurements(clonetimes);
    if (f->count() < 2)
      f->to_delete = true;
    else
      keep.push_back(f);
  }
  fv = keep;
  if (fv.empty()) return 0;
  int rep = o_.feat_rep_slam;
  if (rep != 0 && rep != 2 && rep != 4) throw HpError(UVIO_HP_E_CONFIG, "feat_rep_slam: representation not implemented");
  double s2 = o_.slam_sigma_pix * o_.slam_sigma_pix;
  last_upd_.clear();
  // 1) triangulate + refine all features against the pre-update state (UpdaterSLAM.cpp:119-141)
  HPROF("di.total");
  std::vector<DFeatOut> tri;
  {
    HPROF("di.tri");
    Batch b;
    build_clone_cam_tables(b, false);
    for (auto &f : fv)
      add_feature(this, f, 2, rep, o_, b.cams, b.slot_of_time, b.clones, b.feats, b.meas, b.vars, b.rows, nullptr, -1);
    // triangulation only: the rows and chi2 come from the per-feature mode-3 linearization below
    run_batch(b, 2, s2, o_.slam_chi2_multipler, true, tri, false);
  }
  std::vector<size_t> cand;
  for (size_t i = 0; i < fv.size(); i++) {
    FeatP &f = fv[i];
    if (tri[i].status == 1 || tri[i].status == 2) {
      f->to_delete = true;
      last_upd_.push_back(FeatDebug{f->featid, {0.0, 0.0, 0.0}, tri[i].status, 0.0});
      frame_feats_.push_back({2, FeatDebug{f->featid, {0.0, 0.0, 0.0}, 1, 0.0}});
      continue;
    }
    // anchor (host rule, identical to the kernel's) and triangulated position
    size_t anchor_cam = 0, most = 0;
    for (auto &p : f->tracks)
      if (p.m.size() > most) anchor_cam = p.cam, most = p.m.size();
    f->anchor_cam_id = (int)anchor_cam;
    f->anchor_clone_timestamp = f->find(anchor_cam)->m.back().t;
    for (int k = 0; k < 3; k++) f->p_FinA[k] = tri[i].p_FinA[k], f->p_FinG[k] = tri[i].p_FinG[k];
    cand.push_back(i);
  }
  // 2) per candidate, in order: linearize at the current state, initialize_invertible, the EKF update of the
  // remaining rows behind StateHelper::initialize's chi2 test -- as device chains of up to chain_k candidates
  for (size_t c0 = 0; c0 < cand.size(); c0 += (size_t)d_.chain_k) {
    std::vector<size_t> part(cand.begin() + c0, cand.begin() + std::min(cand.size(), c0 + (size_t)d_.chain_k));
    HPROF("di.chain");
    int rc = slam_delayed_chain(fv, part, rep, s2);
    if (rc) return rc;
  }
  return 0;
}

// The delayed initializations of one frame (StateHelper::initialize per candidate, StateHelper.cpp:393-482)
// as one device chain with one host wait.  Candidate j is linearized (mode 3: at the batch triangulation,
// the current clone / camera values), its landmark is appended by initialize_invertible in a FIXED slot
// N0 + 3 j, its remaining rows update the state behind the chi2 test of their own factor (the S of
// StateHelper::initialize's test, StateHelper.cpp:451-470, is the S the update factors), and k_chain_apply
// then either moves the device clone / camera tables by the update's dx (the next candidate linearizes at
// the updated state, as the reference's loop does) or clears the slot of a rejected candidate: a zero slot
// has zero rows in every later M and K, so it changes nothing until the host marginalizes it afterwards
// (StateHelper::marginalize, the same exact copy-compaction as any other variable).  The host then replays
// the candidates in order from one readback: landmark values (H_finit^-1 times the init residual), the
// updates' dx on its mean, the landmark set.
int Engine::slam_delayed_chain(std::vector<FeatP> &fv, const std::vector<size_t> &idx, int rep, double s2) {
  const int K = (int)idx.size();
  if (K == 0) return 0;
  const int N0 = N_;
  if (N0 + 3 * K > d_.ldp) throw HpError(UVIO_HP_E_CAPACITY, "covariance capacity exceeded");
  Batch b;
  {
    HPROF("di.prep");
    build_clone_cam_tables(b, false);
    for (size_t i : idx)
      add_feature(this, fv[i], 3, rep, o_, b.cams, b.slot_of_time, b.clones, b.feats, b.meas, b.vars, b.rows, nullptr, -1);
  }
  if ((int)b.feats.size() > d_.max_feat || (int)b.n_meas() > d_.max_meas_total || (int)b.n_vars() > d_.max_vars_total ||
      b.rows > d_.max_rows || b.n_canon + 1 > d_.max_ncol)
    throw HpError(UVIO_HP_E_CAPACITY, "delayed-initialization chain exceeds device capacity");
  for (int j = 0; j < K; j++) {  // mode 3 linearizes at the batch triangulation (p_in = p_FinA, p_in_fej = p_FinG)
    const FeatP &f = fv[idx[j]];
    for (int k = 0; k < 3; k++) b.feats[j].p_in[k] = f->p_FinA[k], b.feats[j].p_in_fej[k] = f->p_FinG[k];
    if (b.feats[j].nmeas > kMaxMeasPerFeat) throw HpError(UVIO_HP_E_CAPACITY, "too many measurements per feature");
  }
  // the pose values behind the clone / camera tables (k_chain_apply updates them in place)
  std::vector<DPoseVal> cv(b.clones.size()), camv(b.cams.size());
  {
    size_t s = 0;
    for (auto &c : clones_) {
      for (int k = 0; k < 4; k++) cv[s].q[k] = c.second->val[k];
      for (int k = 0; k < 3; k++) cv[s].p[k] = c.second->val[4 + k];
      cv[s].pid = c.second->id;
      s++;
    }
    for (size_t c = 0; c < camv.size(); c++) {
      const VarP &pose = calib_pose_.at((int)c);
      for (int k = 0; k < 4; k++) camv[c].q[k] = pose->val[k];
      for (int k = 0; k < 3; k++) camv[c].p[k] = pose->val[4 + k];
      camv[c].pid = pose->id;
    }
  }
  const DFeat *t_feats = stage(b.feats.data(), b.feats.size());
  const DMeas *t_meas = stage(b.meas.data(), b.meas.size());
  const DVar *t_vars = stage(b.vars.data(), b.vars.size());
  DClone *t_clones = const_cast<DClone *>(stage(b.clones.data(), b.clones.size()));
  DCam *t_cams = const_cast<DCam *>(stage(b.cams.data(), b.cams.size()));
  DPoseVal *t_cv = const_cast<DPoseVal *>(stage(cv.data(), cv.size()));
  DPoseVal *t_camv = const_cast<DPoseVal *>(stage(camv.data(), camv.size()));
  const int *t_hidx = stage(b.hidx.data(), b.hidx.size());
  stage_flush();
  DBatchParams bp = batch_params(b, s2, o_.slam_chi2_multipler);
  bp.nfeat = 1;
  bp.gate_out = d_.acc;  // the candidate's linearization status: gates initialize_invertible and its update
  const int n = b.n_canon;
  const size_t st = d_.chain_stride;
  {
    HPROF("di.enqueue");
    for (int j = 0; j < K; j++) {
      const DFeat &F = b.feats[j];
      const int Ni = N0 + 3 * j, nup = 2 * F.nmeas - 3;
      {
        KScope ks(&kprof_, KC_FEATURE);
        launch_feature_linearize(d_.stream, bp, t_feats + j, t_meas, t_vars, t_clones, t_cams, d_.P, d_.chi2, d_.H,
                                 d_.fout + j, F.nmeas, F.nf);
      }
      EkfScratch sc = d_.ekf;
      sc.dx = d_.region_dev(j);
      double *Hrow = d_.H + (size_t)F.row_off * d_.ldh;
      // initialize_invertible with rows 0..2 (H_Linv from the feature's H_finit); its residual column lands in
      // the candidate's region behind the chi2 gate's [chi2, accepted]
      launch_init_invertible(d_.stream, d_.P, d_.ldp, Ni, Hrow, d_.ldh, n, t_hidx, nullptr, s2, sc, d_.fout + j, d_.acc,
                             sc.dx + Ni + 5);
      if (nup > 0) {
        sc.chi2_gate = d_.acc;
        sc.chi2_thr = o_.slam_chi2_multipler * chi2_table_[std::min(2 * F.nmeas, 999)];
        sc.gate = nullptr;
        KScope ks(&kprof_, KC_EKF);
        launch_ekf_update(d_.stream, d_.P, d_.ldp, Ni + 3, Hrow + 3 * (size_t)d_.ldh, d_.ldh, nup, n, t_hidx,
                          Hrow + 3 * (size_t)d_.ldh + n, d_.ldh, s2, sc);
      }
      if (nup > 0) kprof_.credit(KC_EKF, ekf_flops(Ni + 3, n, nup), ekf_bytes(Ni + 3, n, nup));
      launch_chain_apply(d_.stream, d_.fout + j, d_.acc, nup > 0 ? sc.neg : nullptr, nup > 0 ? sc.dx : nullptr,
                         t_clones, t_cv, (int)b.clones.size(), t_cams, t_camv, (int)b.cams.size(),
                         o_.do_calib_camera_pose, o_.do_calib_camera_intrinsics, nullptr, 0, d_.P, d_.ldp, Ni + 3, Ni,
                         sc.dx + Ni + 8);
    }
    ++p_epoch_;
    chain_results_copy(K, K);
    d_.fout_pending = 0;
  }
  dev_sync();
  // replay on the host mean, candidate by candidate
  HPROF("di.replay");
  N_ = N0 + 3 * K;
  std::vector<int> dead;
  for (int j = 0; j < K; j++) {
    FeatP &f = fv[idx[j]];
    const DFeat &F = b.feats[j];
    const DFeatOut &o1 = d_.fout_host[j];
    const int Ni = N0 + 3 * j, nup = 2 * F.nmeas - 3;
    const double *base = d_.region_host(j);
    if (base[Ni + 9] > 0.5) throw HpError(UVIO_HP_E_NUMERIC, "EKFUpdate: negative covariance diagonal");
    const bool accepted = base[Ni + 8] > 0.5;
    f->to_delete = true;
    last_upd_.push_back(FeatDebug{f->featid, {f->p_FinG[0], f->p_FinG[1], f->p_FinG[2]}, accepted ? 0 : 3,
                                  nup > 0 ? base[Ni + 3] : 0.0});
    frame_feats_.push_back({2, last_upd_.back()});
    if (!accepted) {
      dead.push_back(Ni);
      continue;
    }
    VarP lm = std::make_shared<Var>(V_LANDMARK, 3, 3);
    lm->featid = f->featid;
    lm->rep = rep;
    lm->unique_cam = f->anchor_cam_id;
    lm->anchor_cam = f->anchor_cam_id;
    lm->anchor_time = f->anchor_clone_timestamp;
    const bool relr = (rep == 2 || rep == 4);
    lm->set_xyz(relr ? f->p_FinA : f->p_FinG, false);
    lm->set_xyz(relr ? f->p_FinA : f->p_FinG, true);
    lm->id = Ni;
    vars_.push_back(lm);
    double HLinv[9], dl[3];
    inv3_cofactor(o1.HfR, HLinv);  // the device's formula: identical H_Linv
    const double *resinit = base + Ni + 5;
    for (int a = 0; a < 3; a++)
      dl[a] = HLinv[3 * a] * resinit[0] + HLinv[3 * a + 1] * resinit[1] + HLinv[3 * a + 2] * resinit[2];
    lm->update(dl);
    if (nup > 0) apply_dx(base);
    slam_.insert({f->featid, lm});
  }
  // the rejected candidates' (zeroed) slots leave the covariance, last first
  for (size_t k = dead.size(); k-- > 0;) {
    VarP ph = std::make_shared<Var>(V_LANDMARK, 3, 3);
    ph->id = dead[k];
    vars_.push_back(ph);
    marginalize(ph);
  }
  return 0;
}

// UpdaterSLAM::change_anchors / perform_anchor_change (UpdaterSLAM.cpp:481-647)
int Engine::slam_change_anchors() {
  stage_ = "UpdaterSLAM::change_anchors";
  if ((int)clones_.size() <= o_.max_clone_size) return 0;
  double mt = margtimestep();
  // The landmarks' propagations are batched into one EKFPropagation with a block-row Phi: each
  // landmark's rows reference only its own inputs (old/new anchor clone, calibration, itself), so the
  // sequential per-landmark propagations of the reference compose to exactly this single one.
  std::vector<int> b_rows, b_iold;
  std::vector<std::vector<std::pair<int, double>>> b_phi;  // per batched row: (cov id, value)
  auto flush = [&]() {
    if (b_rows.empty()) return;
    std::unordered_map<int, int> col;
    for (size_t k = 0; k < b_iold.size(); k++) col[b_iold[k]] = (int)k;
    const int pr = (int)b_rows.size(), q = (int)b_iold.size();
    std::vector<double> Phi((size_t)pr * q, 0.0), Q((size_t)pr * pr, 0.0);
    for (int x = 0; x < pr; x++)
      for (auto &e : b_phi[x]) Phi[(size_t)x * q + col.at(e.first)] += e.second;
    cov_propagate(0, pr, b_iold, Phi, Q, &b_rows);
    b_rows.clear();
    b_iold.clear();
    b_phi.clear();
  };
  for (auto &kv : slam_) {
    VarP lm = kv.second;
    if (lm->rep == 0 || lm->rep == 1) continue;
    if (lm->anchor_time != mt) continue;
    // old / new anchor camera poses
    auto cam_pose = [&](int cam, const VarP &clone, bool fej, double *R_GtoC, double *p_CinG) {
      double Ric[9], Rgi[9], t[3];
      quat_2_Rot(calib_pose_.at(cam)->val, Ric);
      quat_2_Rot(fej ? clone->fej : clone->val, Rgi);
      m3_mul(Ric, Rgi, R_GtoC);
      m3t_vec(R_GtoC, calib_pose_.at(cam)->val + 4, t);
      const double *p = (fej ? clone->fej : clone->val) + 4;
      for (int k = 0; k < 3; k++) p_CinG[k] = p[k] - t[k];
    };
    VarP iold = clones_.at(lm->anchor_time), inew = clones_.at(timestamp_);
    int cam = lm->anchor_cam;
    double p_old[3], p_old_fej[3];
    lm->xyz(false, p_old);
    lm->xyz(true, p_old_fej);
    auto transfer = [&](bool fej, const double *pin, double *pout) {
      double Ro[9], po[3], Rn[9], pn[3], Ron[9], d[3], t[3];
      cam_pose(cam, iold, fej, Ro, po);
      cam_pose(cam, inew, fej, Rn, pn);
      m3_mul_bt(Rn, Ro, Ron);
      for (int k = 0; k < 3; k++) d[k] = po[k] - pn[k];
      m3_vec(Rn, d, t);
      double a[3];
      m3_vec(Ron, pin, a);
      for (int k = 0; k < 3; k++) pout[k] = a[k] + t[k];
    };
    double p_new[3], p_new_fej[3];
    transfer(false, p_old, p_new);
    transfer(true, p_old_fej, p_new_fej);
    // representation Jacobians (get_feature_jacobian_representation, UpdaterHelper.cpp:90-168)
    auto rep_jac = [&](const VarP &anchor, const double *pFA_in, double *Hf, double *Hanc, double *Hcal) {
      double Ric[9], Rgi[9], pIinC[3], pIinG[3], pFA[3];
      quat_2_Rot(calib_pose_.at(cam)->val, Ric);
      for (int k = 0; k < 3; k++) pIinC[k] = calib_pose_.at(cam)->val[4 + k];
      quat_2_Rot(anchor->val, Rgi);
      for (int k = 0; k < 3; k++) pIinG[k] = anchor->val[4 + k], pFA[k] = pFA_in[k];
      if (o_.do_fej) {
        double d0[3] = {pFA[0] - pIinC[0], pFA[1] - pIinC[1], pFA[2] - pIinC[2]}, t1[3], t2[3], best[3];
        m3t_vec(Ric, d0, t1);
        m3t_vec(Rgi, t1, t2);
        for (int k = 0; k < 3; k++) best[k] = t2[k] + pIinG[k];
        quat_2_Rot(anchor->fej, Rgi);
        for (int k = 0; k < 3; k++) pIinG[k] = anchor->fej[4 + k];
        double d1[3] = {best[0] - pIinG[0], best[1] - pIinG[1], best[2] - pIinG[2]}, u[3];
        m3_vec(Rgi, d1, u);
        m3_vec(Ric, u, t1);
        for (int k = 0; k < 3; k++) pFA[k] = t1[k] + pIinC[k];
      }
      double RIT[9], RCT[9], RCG[9], Sk[9], Tm[9];
      m3_transpose(Rgi, RIT);
      m3_transpose(Ric, RCT);
      m3_mul(RIT, RCT, RCG);
      double dd[3] = {pFA[0] - pIinC[0], pFA[1] - pIinC[1], pFA[2] - pIinC[2]}, w[3];
      m3t_vec(Ric, dd, w);
      skew(w, Sk);
      m3_mul(RIT, Sk, Tm);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          Hanc[6 * i + j] = -Tm[3 * i + j];
          Hanc[6 * i + 3 + j] = (i == j);
        }
      skew(dd, Sk);
      m3_mul(RCG, Sk, Tm);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          Hcal[6 * i + j] = -Tm[3 * i + j];
          Hcal[6 * i + 3 + j] = -RCG[3 * i + j];
        }
      if (lm->rep == 2) {
        std::memcpy(Hf, RCG, sizeof(double) * 9);
      } else {
        double alpha = pFA[0] / pFA[2], beta = pFA[1] / pFA[2], rho = 1 / pFA[2];
        double d[9] = {1.0 / rho, 0, -(1.0 / (rho * rho)) * alpha, 0, 1.0 / rho, -(1.0 / (rho * rho)) * beta, 0, 0,
                       -(1.0 / (rho * rho))};
        m3_mul(RCG, d, Hf);
      }
    };
    double Hf_old[9], Ha_old[18], Hc_old[18], Hf_new[9], Ha_new[18], Hc_new[18];
    double pA_old[3], pA_new_tmp[3];
    lm->xyz(false, pA_old);
    rep_jac(iold, pA_old, Hf_old, Ha_old, Hc_old);
    // new representation at the new anchor: the reference passes new_feat with p_FinA = transferred value
    std::memcpy(pA_new_tmp, p_new, sizeof(p_new));
    rep_jac(inew, pA_new_tmp, Hf_new, Ha_new, Hc_new);
    // Phi order: x_order_old (anchor clone, calib), x_order_new (new clone, calib dup), landmark
    std::vector<std::pair<int, int>> order;  // (cov id, size)
    std::vector<int> col_anchor_old, col_cal, col_anchor_new;
    int cur = 0;
    order.push_back({iold->id, 6});
    int c_old = cur;
    cur += 6;
    int c_cal = -1;
    if (o_.do_calib_camera_pose) {
      order.push_back({calib_pose_.at(cam)->id, 6});
      c_cal = cur;
      cur += 6;
    }
    int c_new = cur;
    order.push_back({inew->id, 6});
    cur += 6;
    int c_lm = cur;
    order.push_back({lm->id, 3});
    cur += 3;
    double Hinv[9];
    {
      double *A = Hf_new;
      double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) + A[2] * (A[3] * A[7] - A[4] * A[6]);
      Hinv[0] = (A[4] * A[8] - A[5] * A[7]) / det;
      Hinv[1] = (A[2] * A[7] - A[1] * A[8]) / det;
      Hinv[2] = (A[1] * A[5] - A[2] * A[4]) / det;
      Hinv[3] = (A[5] * A[6] - A[3] * A[8]) / det;
      Hinv[4] = (A[0] * A[8] - A[2] * A[6]) / det;
      Hinv[5] = (A[2] * A[3] - A[0] * A[5]) / det;
      Hinv[6] = (A[3] * A[7] - A[4] * A[6]) / det;
      Hinv[7] = (A[1] * A[6] - A[0] * A[7]) / det;
      Hinv[8] = (A[0] * A[4] - A[1] * A[3]) / det;
    }
    std::vector<double> Phi((size_t)3 * cur, 0.0), Q(9, 0.0);
    auto addblk = [&](int col, const double *H36, double sgn) {
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 6; j++) {
          double s = 0;
          for (int k = 0; k < 3; k++) s += Hinv[3 * i + k] * H36[6 * k + j];
          Phi[(size_t)i * cur + col + j] += sgn * s;
        }
    };
    addblk(c_old, Ha_old, 1.0);
    if (c_cal >= 0) addblk(c_cal, Hc_old, 1.0);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += Hinv[3 * i + k] * Hf_old[3 * k + j];
        Phi[(size_t)i * cur + c_lm + j] = s;
      }
    addblk(c_new, Ha_new, -1.0);
    if (c_cal >= 0) addblk(c_cal, Hc_new, -1.0);
    std::vector<int> iold_ids;
    for (auto &o : order)
      for (int k = 0; k < o.second; k++) iold_ids.push_back(o.first + k);
    if (b_rows.size() + 3 > 63 || b_iold.size() + iold_ids.size() > 256) flush();
    for (int id : iold_ids)
      if (std::find(b_iold.begin(), b_iold.end(), id) == b_iold.end()) b_iold.push_back(id);
    for (int i = 0; i < 3; i++) {
      b_rows.push_back(lm->id + i);
      std::vector<std::pair<int, double>> rowv;
      for (int c = 0; c < cur; c++)
        if (Phi[(size_t)i * cur + c] != 0.0) rowv.push_back({iold_ids[c], Phi[(size_t)i * cur + c]});
      b_phi.push_back(rowv);
    }
    lm->anchor_time = timestamp_;
    timing_.n_anchor_change++;
    lm->set_xyz(p_new, false);
    lm->set_xyz(p_new_fej, true);
  }
  flush();
  return 0;
}

// UpdaterUWB::update_single (UpdaterUWB.cpp:53-90) + UVioUpdaterHelper::get_uwb_jacobian_single
// (UVioUpdaterHelper.cpp:147-241) for one range: a message of one range
int Engine::uwb_update_single(size_t anchor_id, double range) {
  if (anchors_.find(anchor_id) == anchors_.end()) return 0;
  return uwb_update_message({{anchor_id, range}});
}

// The ranges of one message as ONE device chain (UVioManager.cpp:178-188 runs update_single per range, each
// linearized at the state the previous one left): the linearization state (IMU pose, p_IinU, the message's
// anchors) goes up once; per range k_uwb_row moves it by the previous range's dx when that was accepted (Var::update's
// formulas) and forms the row, k_uwb_M forms M = P[:, I] h, k_uwb_update gates chi2 = res^2 / S on the device and
// updates P and dx when accepted.  One readback returns every range's [accepted, negative diagonals, chi2, S | dx];
// the host then applies the accepted dx's to its mean in order (the same values the device state moved by), so
// each row is linearized exactly where the per-range path linearized it -- with two host waits per range (S for
// the gate, then dx) instead of one per message.
int Engine::uwb_update_message(const std::vector<std::pair<size_t, double>> &ranges) {
  stage_ = "UpdaterUWB::update_single";
  int applied = 0;
  for (size_t c0 = 0; c0 < ranges.size(); c0 += kUwbMaxRanges) {
    const int nr = (int)std::min(ranges.size() - c0, (size_t)kUwbMaxRanges);
    DUwbState st{};
    std::memcpy(st.q, imu_->val, sizeof(double) * 4);
    std::memcpy(st.p, imu_->val + 4, sizeof(double) * 3);
    std::memcpy(st.pU, p_IinU_->val, sizeof(double) * 3);
    st.id_imu = imu_->id;
    st.id_cal = o_.do_calib_uwb_extrinsics ? p_IinU_->id : -1;
    st.nr = nr;
    std::vector<int> hidx;
    std::vector<int> off(nr), ncol(nr);
    for (int j = 0; j < nr; j++) {
      const VarP &an = anchors_.at(ranges[c0 + j].first);
      std::memcpy(st.anc[j], an->val, sizeof(double) * 5);
      st.range[j] = ranges[c0 + j].second;
      st.id_anc[j] = an->fixed ? -1 : an->id;
      off[j] = (int)hidx.size();
      for (int k = 0; k < 6; k++) hidx.push_back(imu_->id + k);
      if (o_.do_calib_uwb_extrinsics)
        for (int k = 0; k < 3; k++) hidx.push_back(p_IinU_->id + k);
      if (!an->fixed)
        for (int k = 0; k < 5; k++) hidx.push_back(an->id + k);
      ncol[j] = (int)hidx.size() - off[j];
    }
    DUwbState *dst = stage(&st, 1);
    const int *dh = stage(hidx.data(), hidx.size());
    stage_flush();
    const double s2 = o_.uwb_sigma_range * o_.uwb_sigma_range;
    const double thr = o_.uwb_chi2_multipler * chi2_table_[1];
    for (int j = 0; j < nr; j++) {
      double *reg = d_.uwb_reg + (size_t)j * d_.uwb_stride, *h = d_.uwb_h + 16 * j;
      launch_uwb_row(d_.stream, dst, j, j ? reg - d_.uwb_stride : nullptr, h, reg);
      launch_uwb_M(d_.stream, d_.P, d_.ldp, N_, h, dh + off[j], ncol[j], d_.ekf.M);
      launch_uwb_update(d_.stream, d_.P, d_.ldp, N_, d_.ekf.M, h, dh + off[j], ncol[j], s2, thr, reg);
    }
    ++p_epoch_;
    const size_t n = (size_t)(nr - 1) * d_.uwb_stride + 4 + N_;
    HP_HIP(hipMemcpyAsync(d_.uwb_host, d_.uwb_reg, sizeof(double) * n, hipMemcpyDeviceToHost, d_.stream));
    dev_sync();
    for (int j = 0; j < nr; j++) {
      const double *reg = d_.uwb_host + (size_t)j * d_.uwb_stride;
      if (reg[0] == 0.0) continue;
      if (*reinterpret_cast<const int *>(reg + 1) > 0)
        throw HpError(UVIO_HP_E_NUMERIC, "UWB EKFUpdate: negative covariance diagonal");
      apply_dx(reg + 4);
      applied++;
    }
  }
  return applied;
}

}  // namespace uvhp
