// ORACLE — test infrastructure only (see la.h header).
// Restatement of the reference state and covariance algebra:
//   ov_core/src/types/{Type,Vec,JPLQuat,PoseJPL,IMU,Landmark}.h, Landmark.cpp:26-144
//   uvio/src/types/UWB_anchor.h:37-197
//   ov_msckf/src/state/State.{h,cpp}  (State.cpp:28-166 layout + priors)
//   ov_msckf/src/state/StateHelper.cpp:36-645
#pragma once
#include <map>
#include <memory>
#include <string>
#include <unordered_map>

#include "cam.h"
#include "uvio_hp.h"

namespace orc {

enum Kind { K_IMU = 0, K_VEC = 1, K_QUAT = 2, K_POSE = 3, K_LANDMARK = 4, K_ANCHOR = 5 };

// LandmarkRepresentation::Representation (LandmarkRepresentation.h:38)
enum Rep {
  GLOBAL_3D = 0,
  GLOBAL_FULL_INVERSE_DEPTH = 1,
  ANCHORED_3D = 2,
  ANCHORED_FULL_INVERSE_DEPTH = 3,
  ANCHORED_MSCKF_INVERSE_DEPTH = 4,
  ANCHORED_INVERSE_DEPTH_SINGLE = 5,
  UNKNOWN = 6
};
inline bool is_relative(int r) {
  return r == ANCHORED_3D || r == ANCHORED_FULL_INVERSE_DEPTH || r == ANCHORED_MSCKF_INVERSE_DEPTH ||
         r == ANCHORED_INVERSE_DEPTH_SINGLE;
}

struct Var {
  Kind kind;
  int id = -1;
  int size = 0;
  Mat val, fej;  // column vectors
  // landmark
  size_t featid = 0;
  int rep = UNKNOWN;
  int anchor_cam = -1;
  double anchor_time = -1;
  int unique_cam = -1;
  bool should_marg = false;
  int fail_count = 0;
  bool has_anchor_change = false;
  Mat uvn0, uvn0_fej;
  // uwb anchor
  uint64_t anchor_id = 0;
  bool fixed = false;

  Var(Kind k, int sz, int vlen) : kind(k), size(sz), val(vlen, 1), fej(vlen, 1) {}

  // quaternion part helpers for IMU / POSE / QUAT
  Mat quat() const { return val.block(0, 0, 4, 1); }
  Mat quat_fej() const { return fej.block(0, 0, 4, 1); }
  Mat Rot() const { return quat_2_Rot(quat()); }
  Mat Rot_fej() const { return quat_2_Rot(quat_fej()); }
  Mat pos() const { return val.block(4, 0, 3, 1); }
  Mat pos_fej() const { return fej.block(4, 0, 3, 1); }
  // IMU extras
  Mat vel() const { return val.block(7, 0, 3, 1); }
  Mat vel_fej() const { return fej.block(7, 0, 3, 1); }
  Mat bias_g() const { return val.block(10, 0, 3, 1); }
  Mat bias_a() const { return val.block(13, 0, 3, 1); }

  void update(const Mat &dx);  // Type::update family
  // Landmark::get_xyz / set_from_xyz (Landmark.cpp:26,65)
  Mat get_xyz(bool getfej) const;
  void set_from_xyz(const Mat &p, bool isfej);
};
using VarP = std::shared_ptr<Var>;

inline VarP make_imu() {
  auto v = std::make_shared<Var>(K_IMU, 15, 16);
  v->val[3] = 1;
  v->fej[3] = 1;
  return v;
}
inline VarP make_vec(int n) { return std::make_shared<Var>(K_VEC, n, n); }
inline VarP make_quat() {
  auto v = std::make_shared<Var>(K_QUAT, 3, 4);
  v->val[3] = 1;
  v->fej[3] = 1;
  return v;
}
inline VarP make_pose() {
  auto v = std::make_shared<Var>(K_POSE, 6, 7);
  v->val[3] = 1;
  v->fej[3] = 1;
  return v;
}

// A (id,size) reference into the covariance: H_order entries. For sub-variables (imu->pose(),
// imu->q()) only the covariance slice matters.
struct Ref {
  const Var *var;
  int off;   // offset inside var (sub-variable), e.g. pose() = (imu, 0, 6)
  int size;
  int id() const { return var->id + off; }
  bool operator==(const Ref &o) const { return var == o.var && off == o.off && size == o.size; }
};

struct State {
  uvio_hp_options_t opt;
  double timestamp = -1;
  VarP imu;
  std::map<double, VarP> clones;                     // State.h:150
  std::unordered_map<size_t, VarP> features_SLAM;    // State.h:153
  VarP calib_dt;
  std::unordered_map<size_t, VarP> calib_IMUtoCAM;   // State.h:159
  std::unordered_map<size_t, VarP> cam_intrinsics;   // State.h:162
  std::unordered_map<size_t, Camera> cams;           // State.h:165
  VarP dw, da, tg, q_GYROtoIMU, q_ACCtoIMU;
  // uvio (UVioState.h:40)
  VarP calib_UWBtoIMU;                               // p_IinU (3)
  std::map<size_t, VarP> anchors;                    // _calib_GLOBALtoANCHORS (std::map)
  Mat Cov;
  std::vector<VarP> variables;

  explicit State(const uvio_hp_options_t &o);
  int max_covariance_size() const { return Cov.r; }
  double margtimestep() const {
    double t = INFINITY;
    for (auto &c : clones)
      if (c.first < t) t = c.first;
    return t;
  }
  int imu_intrinsic_size() const {
    int sz = 0;
    if (opt.do_calib_imu_intrinsics) {
      sz += 15;
      if (opt.do_calib_imu_g_sensitivity) sz += 9;
    }
    return sz;
  }
  Mat Dm(const Mat &v) const;  // State::Dm (State.h:92)
  Mat Tg(const Mat &v) const;  // State::Tg (State.h:104)
};

// ---- StateHelper (StateHelper.cpp) ----
namespace StateHelper {
// returns false on negative diagonal (reference exits)
bool EKFPropagation(State &s, const std::vector<Ref> &order_NEW, const std::vector<Ref> &order_OLD, const Mat &Phi,
                    const Mat &Q);
bool EKFUpdate(State &s, const std::vector<Ref> &H_order, const Mat &H, const Mat &res, double sigma2);
Mat get_marginal_covariance(const State &s, const std::vector<Ref> &vars);
void set_initial_covariance(State &s, const Mat &cov, const std::vector<Ref> &order);
void marginalize(State &s, VarP marg);
VarP clone(State &s, const Ref &var);
double initialize_split(const State &s, const std::vector<Ref> &H_order, Mat &H_R, Mat &H_L, double sigma2, Mat &res,
                        Mat &Hup, Mat &resup);
bool initialize(State &s, VarP new_var, const std::vector<Ref> &H_order, Mat &H_R, Mat &H_L, double sigma2, Mat &res,
                double chi2_mult, int *status);
void initialize_invertible(State &s, VarP new_var, const std::vector<Ref> &H_order, const Mat &H_R, const Mat &H_L,
                           const Mat &R, const Mat &res);
void augment_clone(State &s, const Mat &last_w);
void marginalize_old_clone(State &s);
void marginalize_slam(State &s);
}  // namespace StateHelper

inline Ref ref_of(const VarP &v) { return Ref{v.get(), 0, v->size}; }
inline Ref imu_pose_ref(const State &s) { return Ref{s.imu.get(), 0, 6}; }
inline Ref imu_q_ref(const State &s) { return Ref{s.imu.get(), 0, 3}; }

double chi2_quantile95(int dof);  // boost::math::quantile(chi_squared(dof), 0.95)

}  // namespace orc
