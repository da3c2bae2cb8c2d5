// ORACLE — test infrastructure only (see la.h header).
// UpdaterZeroVelocity restatement (ov_msckf/src/update/UpdaterZeroVelocity.cpp:65-329), see zupt.cpp.
#pragma once
#include <map>

#include "propagator.h"
#include "updater.h"

namespace orc {

struct UpdaterZUPT {
  double chi2_mult, max_velocity, noise_multiplier, max_disparity;
  double sigma_w, sigma_a, sigma_wb, sigma_ab;
  Mat gravity;
  std::map<int, double> chi2_table;
  std::vector<ImuData> imu_data;
  bool have_last_prop_time_offset = false;
  double last_prop_time_offset = 0.0;
  double last_zupt_state_timestamp = 0.0;
  int last_zupt_count = 0;
  // diagnostics of the last try_update
  bool last_accepted = false;
  double last_chi2 = 0, last_disparity = 0;

  explicit UpdaterZUPT(const uvio_hp_options_t &o);
  void feed_imu(const ImuData &m, double oldest_time);
  void clean_old_imu_measurements(double oldest_time);
  // 1: zero-velocity update applied (state time moved to `timestamp`), 0: not, < 0: fatal numeric error
  int try_update(State &s, FeatureDatabase &db, double timestamp);
};

}  // namespace orc
