// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_msckf/src/state/Propagator.{h,cpp} (propagate_and_clone :33-138,
// select_imu_readings :269-393, predict_and_compute :395-480, predict_mean_{discrete,rk4,analytic},
// compute_Xi_sum :588-665, compute_F_and_G_{analytic,discrete} :683-962, compute_H_{Dw,Da,Tg}
// :964-1015) and uvio/src/state/UVioPropagator.cpp:27-115.
#pragma once
#include <vector>

#include "state.h"

namespace orc {

struct ImuData {
  double t;
  double wm[3], am[3];
};

struct Propagator {
  double sigma_w, sigma_a, sigma_wb, sigma_ab;
  Mat gravity;  // (0,0,g)
  std::vector<ImuData> imu_data;
  bool have_last_prop_time_offset = false;
  // ORC_EXPERIMENT_UWB_DT=1: not the reference (see propagate_uwb); the cfg5 ATE study only
  bool experiment_uwb_dt = false;
  double last_prop_time_offset = 0.0;

  explicit Propagator(const uvio_hp_options_t &o);
  void feed_imu(const ImuData &m, double oldest_time);
  void clean_old_imu_measurements(double oldest_time);
  static std::vector<ImuData> select_imu_readings(const std::vector<ImuData> &d, double t0, double t1);
  static ImuData interpolate(const ImuData &a, const ImuData &b, double t);

  // returns false on a fatal numeric condition (negative covariance diagonal)
  bool propagate_and_clone(State &s, double timestamp, int *status);
  // UVioPropagator::propagate (no clone; time0 uses last_prop_time_offset, time1 has no offset)
  bool propagate_uwb(State &s, double timestamp);

  void predict_and_compute(State &s, const ImuData &dm, const ImuData &dp, Mat &F, Mat &Qd);
  void predict_mean_discrete(State &s, double dt, const Mat &w, const Mat &a, Mat &nq, Mat &nv, Mat &np);
  void predict_mean_rk4(State &s, double dt, const Mat &w1, const Mat &a1, const Mat &w2, const Mat &a2, Mat &nq, Mat &nv,
                        Mat &np);
  void predict_mean_analytic(State &s, double dt, const Mat &w, const Mat &a, Mat &nq, Mat &nv, Mat &np, const Mat &Xi);
  void compute_Xi_sum(double dt, const Mat &w, const Mat &a, Mat &Xi);
  void compute_F_and_G_analytic(State &s, double dt, const Mat &w_hat, const Mat &a_hat, const Mat &w_unc,
                                const Mat &a_unc, const Mat &nq, const Mat &nv, const Mat &np, const Mat &Xi, Mat &F, Mat &G);
  void compute_F_and_G_discrete(State &s, double dt, const Mat &w_hat, const Mat &a_hat, const Mat &w_unc,
                                const Mat &a_unc, const Mat &nq, const Mat &nv, const Mat &np, Mat &F, Mat &G);
  std::vector<Ref> phi_order(const State &s) const;
  void accumulate(State &s, const std::vector<ImuData> &prop, Mat &Phi, Mat &Qd);
  void last_w_of(State &s, const std::vector<ImuData> &prop, Mat &last_w);
};

}  // namespace orc
