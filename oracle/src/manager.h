// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_msckf/src/core/VioManager.cpp:166-651 (feed_measurement_imu,
// feed_measurement_simulation, feed_measurement_camera / track_image_and_update,
// do_feature_propagate_update), VioManagerHelper.cpp:40-76
// (initialize_with_gt), ov_core/src/track/TrackSIM.cpp:30-79 and
// uvio/src/core/UVioManager.cpp:26-344 (UWB buffering, anchors, do_uwb_propagate_update).
// UpdaterZeroVelocity (zupt.h) and retriangulate_active_tracks (VioManagerHelper.cpp:190-388: the active
// tracks' running linear triangulation systems, their positions and depths; they change neither the state
// nor the feature database) are restated too.
#pragma once
#include <chrono>
#include <map>
#include <memory>

#include "init.h"
#include "propagator.h"
#include "tracker.h"
#include "updater.h"
#include "zupt.h"

namespace orc {

struct UwbMsg {
  double t;
  std::unordered_map<size_t, double> ranges;
};

struct Manager {
  uvio_hp_options_t o;
  State state;
  Propagator prop;
  UpdaterMSCKF msckf;
  UpdaterSLAM slam;
  UpdaterUWB uwb;
  FeatureDatabase db;
  InertialInitializer initializer;  // VioManager.cpp:150-153 (static initializer, init.h)
  TrackKLT tracker;
  size_t currid;
  bool is_initialized = false;
  bool thread_init_success = false;  // VioManager.h:226
  double startup_time = -1;
  double distance = 0;
  double timelastupdate = -1;
  bool anchors_initialized = false;
  std::map<double, UwbMsg> past_uwb;
  uvio_hp_timing_t timing{};
  UpdateStats last_msckf{};
  FrameDebug fdbg;  // this frame's per-feature results + lock-step steering (updater.h)
  // UpdaterZeroVelocity (VioManager.cpp:160, 186-188, 294-307, 360)
  std::unique_ptr<UpdaterZUPT> zupt;
  bool did_zupt_update = false, has_moved_since_zupt = false;
  // TrackSIM's get_last_obs / get_last_ids of the last simulated frame (TrackSIM.cpp:72-77)
  std::map<int, std::vector<std::pair<size_t, std::pair<float, float>>>> sim_last;
  // retriangulate_active_tracks (VioManagerHelper.cpp:190-388) state and outputs
  std::map<size_t, Mat> linsys_A, linsys_b;
  std::map<size_t, int> linsys_count;
  double active_tracks_time = -1;
  std::unordered_map<size_t, Mat> active_tracks_posinG, active_tracks_uvd;

  explicit Manager(const uvio_hp_options_t &opt);
  void initialize_with_gt(const double x[17]);
  void feed_imu(double t, const double wm[3], const double am[3]);
  int feed_simulation(double t, const std::vector<int> &camids,
                      const std::vector<std::vector<std::pair<size_t, std::pair<float, float>>>> &feats);
  int feed_uwb(double t, const std::vector<std::pair<size_t, double>> &ranges);
  // VioManager::feed_measurement_camera -> track_image_and_update (VioManager.cpp:255-321) with TrackKLT
  int feed_camera(double t, const std::vector<int> &camids, const std::vector<GrayImg> &imgs,
                  const std::vector<GrayImg> &masks);
  int init_anchors(const std::vector<uvio_hp_anchor_t> &anchors);
  int do_feature_propagate_update(double t, const std::vector<int> &camids);
  int do_uwb_propagate_update(const UwbMsg &m);
  // UVioManager.cpp:147-205 after the tracker: ZUPT, UWB ranges, feature propagate / update
  int after_tracking(double t, const std::vector<int> &camids, std::chrono::steady_clock::time_point rT1,
                     bool try_init = false);
  // VioManager::try_to_initialize (VioManagerHelper.cpp:78-190), single-threaded
  bool try_to_initialize();
  void retriangulate_active_tracks(double t, const std::vector<int> &camids);
};

}  // namespace orc
