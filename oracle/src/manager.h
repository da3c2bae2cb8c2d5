// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_msckf/src/core/VioManager.cpp:166-651 (feed_measurement_imu,
// feed_measurement_simulation, feed_measurement_camera / track_image_and_update,
// do_feature_propagate_update), VioManagerHelper.cpp:40-76
// (initialize_with_gt), ov_core/src/track/TrackSIM.cpp:30-79 and
// uvio/src/core/UVioManager.cpp:26-344 (UWB buffering, anchors, do_uwb_propagate_update).
// retriangulate_active_tracks (VioManagerHelper.cpp:190) only feeds visualization and is not
// restated (it changes neither the state nor the feature database).
#pragma once
#include <chrono>

#include "propagator.h"
#include "tracker.h"
#include "updater.h"

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
  TrackKLT tracker;
  size_t currid;
  bool is_initialized = false;
  double startup_time = -1;
  double distance = 0;
  double timelastupdate = -1;
  bool anchors_initialized = false;
  std::map<double, UwbMsg> past_uwb;
  uvio_hp_timing_t timing{};
  UpdateStats last_msckf{};

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
};

}  // namespace orc
