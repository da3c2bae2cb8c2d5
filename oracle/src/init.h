// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_init/src/init/InertialInitializer.cpp:49-147 (feed_imu, initialize),
// ov_init/src/static/StaticInitializer.cpp:37-165, InitializerHelper::gram_schmidt (ov_init/src/utils/helper.h:138-170)
// and FeatureHelper::compute_disparity (ov_core/src/feat/FeatureHelper.h:123-181).  The dynamic initializer
// (DynamicInitializer.cpp, Ceres) is not restated: its branch returns false, as the product does.
#pragma once
#include <vector>

#include "feat.h"
#include "propagator.h"

namespace orc {

struct InertialInitializer {
  uvio_hp_options_t o;
  std::vector<ImuData> imu_data;
  explicit InertialInitializer(const uvio_hp_options_t &opt) : o(opt) {}
  void feed_imu(const ImuData &m, double oldest_time);
  // true: imu_state (16) and covariance (15x15) of the IMU at *timestamp
  bool initialize(FeatureDatabase &db, double *timestamp, Mat &covariance, Mat &imu_state, bool wait_for_jerk);
  bool static_initialize(double *timestamp, Mat &covariance, Mat &imu_state, bool wait_for_jerk);
};

}  // namespace orc
