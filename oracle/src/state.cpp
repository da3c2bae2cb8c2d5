// ORACLE — test infrastructure only (see la.h header).
#include "state.h"

#include <cstdio>

namespace orc {

// JPLQuat::update (JPLQuat.h:114), PoseJPL::update (PoseJPL.h:74), IMU::update (IMU.h:78),
// Vec::update (Vec.h:55), Landmark::update (Landmark.h:80), UWB_anchor::update (UWB_anchor.h:81)
void Var::update(const Mat &dx) {
  assert(dx.r == size);
  if (kind == K_QUAT || kind == K_POSE || kind == K_IMU) {
    Mat dq(4, 1);
    dq[0] = .5 * dx[0];
    dq[1] = .5 * dx[1];
    dq[2] = .5 * dx[2];
    dq[3] = 1.0;
    dq = quatnorm(dq);
    Mat q = quat_multiply(dq, quat());
    for (int i = 0; i < 4; i++) val[i] = q[i];
    for (int i = 3; i < size; i++) val[i + 1] += dx[i];
  } else {
    for (int i = 0; i < size; i++) val[i] += dx[i];
  }
}

Mat Var::get_xyz(bool getfej) const {
  if (rep == GLOBAL_3D || rep == ANCHORED_3D) return getfej ? fej : val;
  if (rep == GLOBAL_FULL_INVERSE_DEPTH || rep == ANCHORED_FULL_INVERSE_DEPTH) {
    const Mat &p = getfej ? fej : val;
    return V3((1 / p[2]) * std::cos(p[0]) * std::sin(p[1]), (1 / p[2]) * std::sin(p[0]) * std::sin(p[1]),
              (1 / p[2]) * std::cos(p[1]));
  }
  if (rep == ANCHORED_MSCKF_INVERSE_DEPTH) {
    // reference quirk (Landmark.cpp:47-52): fej is ignored for this representation
    const Mat &p = val;
    return V3((1 / p[2]) * p[0], (1 / p[2]) * p[1], 1 / p[2]);
  }
  if (rep == ANCHORED_INVERSE_DEPTH_SINGLE) return (1.0 / val[0]) * uvn0;
  assert(false);
  return Mat(3, 1);
}

void Var::set_from_xyz(const Mat &p, bool isfej) {
  Mat &dst = isfej ? fej : val;
  if (rep == GLOBAL_3D || rep == ANCHORED_3D) {
    dst = p;
    return;
  }
  if (rep == GLOBAL_FULL_INVERSE_DEPTH || rep == ANCHORED_FULL_INVERSE_DEPTH) {
    double g_rho = 1 / norm(p);
    double g_phi = std::acos(g_rho * p[2]);
    double g_theta = std::atan2(p[1], p[0]);
    dst = V3(g_theta, g_phi, g_rho);
    return;
  }
  if (rep == ANCHORED_MSCKF_INVERSE_DEPTH) {
    dst = V3(p[0] / p[2], p[1] / p[2], 1 / p[2]);
    return;
  }
  if (rep == ANCHORED_INVERSE_DEPTH_SINGLE) {
    Mat t(1, 1);
    t[0] = 1.0 / p[2];
    if (!isfej)
      uvn0 = (1.0 / p[2]) * p;
    else
      uvn0_fej = (1.0 / p[2]) * p;
    dst = t;
    return;
  }
  assert(false);
}

static Mat vecn(const double *x, int n) {
  Mat m(n, 1);
  for (int i = 0; i < n; i++) m[i] = x[i];
  return m;
}

// State::State (State.cpp:28-166)
State::State(const uvio_hp_options_t &o) : opt(o) {
  int current_id = 0;
  imu = make_imu();
  imu->id = current_id;
  variables.push_back(imu);
  current_id += imu->size;

  dw = make_vec(6);
  da = make_vec(6);
  double def6[6] = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
  dw->val = dw->fej = vecn(def6, 6);
  da->val = da->fej = vecn(def6, 6);
  tg = make_vec(9);
  q_GYROtoIMU = make_quat();
  q_ACCtoIMU = make_quat();
  // values from the imu chain yaml (VioManagerOptions print_and_load_state)
  dw->val = dw->fej = vecn(opt.imu_dw, 6);
  da->val = da->fej = vecn(opt.imu_da, 6);
  tg->val = tg->fej = vecn(opt.imu_tg, 9);
  q_GYROtoIMU->val = q_GYROtoIMU->fej = vecn(opt.q_GYROtoIMU, 4);
  q_ACCtoIMU->val = q_ACCtoIMU->fej = vecn(opt.q_ACCtoIMU, 4);
  if (opt.do_calib_imu_intrinsics) {
    dw->id = current_id;
    variables.push_back(dw);
    current_id += 6;
    da->id = current_id;
    variables.push_back(da);
    current_id += 6;
    if (opt.do_calib_imu_g_sensitivity) {
      tg->id = current_id;
      variables.push_back(tg);
      current_id += 9;
    }
    if (opt.imu_model == 0) {
      q_GYROtoIMU->id = current_id;
      variables.push_back(q_GYROtoIMU);
      current_id += 3;
    } else {
      q_ACCtoIMU->id = current_id;
      variables.push_back(q_ACCtoIMU);
      current_id += 3;
    }
  }
  calib_dt = make_vec(1);
  calib_dt->val[0] = calib_dt->fej[0] = opt.calib_camimu_dt;
  if (opt.do_calib_camera_timeoffset) {
    calib_dt->id = current_id;
    variables.push_back(calib_dt);
    current_id += 1;
  }
  for (int i = 0; i < opt.num_cameras; i++) {
    auto pose = make_pose();
    auto intr = make_vec(8);
    const uvio_hp_camera_t &c = opt.cams[i];
    for (int k = 0; k < 4; k++) pose->val[k] = pose->fej[k] = c.q_ItoC[k];
    for (int k = 0; k < 3; k++) pose->val[4 + k] = pose->fej[4 + k] = c.p_IinC[k];
    intr->val = intr->fej = vecn(c.intrinsics, 8);
    calib_IMUtoCAM.insert({(size_t)i, pose});
    cam_intrinsics.insert({(size_t)i, intr});
    Camera cam;
    cam.model = c.model;
    cam.w = c.width;
    cam.h = c.height;
    for (int k = 0; k < 8; k++) cam.v[k] = c.intrinsics[k];
    cams.insert({(size_t)i, cam});
    if (opt.do_calib_camera_pose) {
      pose->id = current_id;
      variables.push_back(pose);
      current_id += 6;
    }
    if (opt.do_calib_camera_intrinsics) {
      intr->id = current_id;
      variables.push_back(intr);
      current_id += 8;
    }
  }
  Cov = std::pow(1e-3, 2) * Mat::Identity(current_id);
  auto setdiag = [&](int id, int n, double v) {
    for (int k = 0; k < n; k++) Cov(id + k, id + k) = v;
  };
  if (opt.do_calib_imu_intrinsics) {
    setdiag(dw->id, 6, std::pow(0.005, 2));
    setdiag(da->id, 6, std::pow(0.008, 2));
    if (opt.do_calib_imu_g_sensitivity) setdiag(tg->id, 9, std::pow(0.005, 2));
    if (opt.imu_model == 0)
      setdiag(q_GYROtoIMU->id, 3, std::pow(0.005, 2));
    else
      setdiag(q_ACCtoIMU->id, 3, std::pow(0.005, 2));
  }
  if (opt.do_calib_camera_timeoffset) Cov(calib_dt->id, calib_dt->id) = std::pow(0.01, 2);
  if (opt.do_calib_camera_pose)
    for (int i = 0; i < opt.num_cameras; i++) {
      setdiag(calib_IMUtoCAM.at(i)->id, 3, std::pow(0.005, 2));
      setdiag(calib_IMUtoCAM.at(i)->id + 3, 3, std::pow(0.015, 2));
    }
  if (opt.do_calib_camera_intrinsics)
    for (int i = 0; i < opt.num_cameras; i++) {
      setdiag(cam_intrinsics.at(i)->id, 4, std::pow(1.0, 2));
      setdiag(cam_intrinsics.at(i)->id + 4, 4, std::pow(0.005, 2));
    }
  // uvio state (UVioState ctor): p_IinU vector, not in covariance until initialized
  calib_UWBtoIMU = make_vec(3);
  calib_UWBtoIMU->val = calib_UWBtoIMU->fej = vecn(opt.p_IinU, 3);
}

Mat State::Dm(const Mat &v) const {
  Mat D(3, 3);
  if (opt.imu_model == 0) {
    D(0, 0) = v[0];
    D(1, 0) = v[1]; D(1, 1) = v[3];
    D(2, 0) = v[2]; D(2, 1) = v[4]; D(2, 2) = v[5];
  } else {
    D(0, 0) = v[0]; D(0, 1) = v[1]; D(0, 2) = v[3];
    D(1, 1) = v[2]; D(1, 2) = v[4];
    D(2, 2) = v[5];
  }
  return D;
}
Mat State::Tg(const Mat &v) const {
  Mat T(3, 3);
  T(0, 0) = v[0]; T(0, 1) = v[3]; T(0, 2) = v[6];
  T(1, 0) = v[1]; T(1, 1) = v[4]; T(1, 2) = v[7];
  T(2, 0) = v[2]; T(2, 1) = v[5]; T(2, 2) = v[8];
  return T;
}

namespace StateHelper {

static bool check_diag(const State &s, const char *who) {
  bool neg = false;
  for (int i = 0; i < s.Cov.r; i++)
    if (s.Cov(i, i) < 0.0) {
      std::fprintf(stderr, "[oracle] %s - diagonal at %d is %.2f\n", who, i, s.Cov(i, i));
      neg = true;
    }
  return !neg;
}

// StateHelper.cpp:36-114
bool EKFPropagation(State &s, const std::vector<Ref> &order_NEW, const std::vector<Ref> &order_OLD, const Mat &Phi,
                    const Mat &Q) {
  assert(!order_NEW.empty() && !order_OLD.empty());
  for (size_t i = 0; i + 1 < order_NEW.size(); i++) assert(order_NEW[i].id() + order_NEW[i].size == order_NEW[i + 1].id());
  std::vector<int> Phi_id;
  int current_it = 0;
  for (auto &v : order_OLD) {
    Phi_id.push_back(current_it);
    current_it += v.size;
  }
  int N = s.Cov.r;
  Mat Cov_PhiT(N, Phi.r);
  for (size_t i = 0; i < order_OLD.size(); i++) {
    const Ref &v = order_OLD[i];
    Cov_PhiT = Cov_PhiT + s.Cov.block(0, v.id(), N, v.size) * Phi.block(0, Phi_id[i], Phi.r, v.size).T();
  }
  // Q.selfadjointView<Upper>()
  Mat Phi_Cov_PhiT(Q.r, Q.c);
  for (int i = 0; i < Q.r; i++)
    for (int j = 0; j < Q.c; j++) Phi_Cov_PhiT(i, j) = (j >= i) ? Q(i, j) : Q(j, i);
  for (size_t i = 0; i < order_OLD.size(); i++) {
    const Ref &v = order_OLD[i];
    Phi_Cov_PhiT = Phi_Cov_PhiT + Phi.block(0, Phi_id[i], Phi.r, v.size) * Cov_PhiT.block(v.id(), 0, v.size, Phi.r);
  }
  int start_id = order_NEW[0].id();
  int phi_size = Phi.r;
  s.Cov.set_block(start_id, 0, Cov_PhiT.T());
  s.Cov.set_block(0, start_id, Cov_PhiT);
  s.Cov.set_block(start_id, start_id, Phi_Cov_PhiT);
  (void)phi_size;
  return check_diag(s, "EKFPropagation");
}

// StateHelper.cpp:116-197
bool EKFUpdate(State &s, const std::vector<Ref> &H_order, const Mat &H, const Mat &res, double sigma2) {
  assert(H.r == res.r);
  int N = s.Cov.r, r = res.r;
  Mat M_a(N, r);
  std::vector<int> H_id;
  int current_it = 0;
  for (auto &m : H_order) {
    H_id.push_back(current_it);
    current_it += m.size;
  }
  for (auto &var : s.variables) {
    Mat M_i(var->size, r);
    for (size_t i = 0; i < H_order.size(); i++) {
      const Ref &mv = H_order[i];
      M_i = M_i + s.Cov.block(var->id, mv.id(), var->size, mv.size) * H.block(0, H_id[i], H.r, mv.size).T();
    }
    M_a.set_block(var->id, 0, M_i);
  }
  Mat P_small = get_marginal_covariance(s, H_order);
  Mat S = H * P_small * H.T();
  for (int i = 0; i < r; i++) S(i, i) += sigma2;
  Mat Sinv = Mat::Identity(r);
  if (!llt_solve(S, Sinv)) return false;
  // Sinv.selfadjointView<Upper>()
  for (int i = 0; i < r; i++)
    for (int j = 0; j < i; j++) Sinv(i, j) = Sinv(j, i);
  Mat K = M_a * Sinv;
  Mat KM = K * M_a.T();
  for (int i = 0; i < N; i++)
    for (int j = i; j < N; j++) s.Cov(i, j) -= KM(i, j);
  for (int i = 0; i < N; i++)
    for (int j = 0; j < i; j++) s.Cov(i, j) = s.Cov(j, i);
  if (!check_diag(s, "EKFUpdate")) return false;
  Mat dx = K * res;
  for (auto &var : s.variables) var->update(dx.block(var->id, 0, var->size, 1));
  if (s.opt.do_calib_camera_intrinsics)
    for (auto &c : s.cam_intrinsics)
      for (int k = 0; k < 8; k++) s.cams.at(c.first).v[k] = c.second->val[k];
  return true;
}

// StateHelper.cpp:199-223
void set_initial_covariance(State &s, const Mat &cov, const std::vector<Ref> &order) {
  int i_index = 0;
  for (size_t i = 0; i < order.size(); i++) {
    int k_index = 0;
    for (size_t k = 0; k < order.size(); k++) {
      s.Cov.set_block(order[i].id(), order[k].id(), cov.block(i_index, k_index, order[i].size, order[k].size));
      k_index += order[k].size;
    }
    i_index += order[i].size;
  }
  for (int i = 0; i < s.Cov.r; i++)
    for (int j = 0; j < i; j++) s.Cov(i, j) = s.Cov(j, i);
}

// StateHelper.cpp:225-254
Mat get_marginal_covariance(const State &s, const std::vector<Ref> &vars) {
  int n = 0;
  for (auto &v : vars) n += v.size;
  Mat C(n, n);
  int i_index = 0;
  for (size_t i = 0; i < vars.size(); i++) {
    int k_index = 0;
    for (size_t k = 0; k < vars.size(); k++) {
      C.set_block(i_index, k_index, s.Cov.block(vars[i].id(), vars[k].id(), vars[i].size, vars[k].size));
      k_index += vars[k].size;
    }
    i_index += vars[i].size;
  }
  return C;
}

// StateHelper.cpp:271-339
void marginalize(State &s, VarP marg) {
  int marg_size = marg->size, marg_id = marg->id;
  int N = s.Cov.r;
  int x2_size = N - marg_id - marg_size;
  Mat Cn(N - marg_size, N - marg_size);
  Cn.set_block(0, 0, s.Cov.block(0, 0, marg_id, marg_id));
  Cn.set_block(0, marg_id, s.Cov.block(0, marg_id + marg_size, marg_id, x2_size));
  Cn.set_block(marg_id, 0, Cn.block(0, marg_id, marg_id, x2_size).T());
  Cn.set_block(marg_id, marg_id, s.Cov.block(marg_id + marg_size, marg_id + marg_size, x2_size, x2_size));
  s.Cov = Cn;
  std::vector<VarP> remaining;
  for (auto &v : s.variables) {
    if (v != marg) {
      if (v->id > marg_id) v->id -= marg_size;
      remaining.push_back(v);
    }
  }
  marg->id = -1;
  s.variables = remaining;
}

// StateHelper.cpp:341-391 (only ever called on imu->pose() here)
VarP clone(State &s, const Ref &var) {
  int total_size = var.size;
  int old_size = s.Cov.r;
  int new_loc = s.Cov.r;
  s.Cov.conservative_resize(old_size + total_size, old_size + total_size);
  int old_loc = var.id();
  s.Cov.set_block(new_loc, new_loc, s.Cov.block(old_loc, old_loc, total_size, total_size));
  s.Cov.set_block(0, new_loc, s.Cov.block(0, old_loc, old_size, total_size));
  s.Cov.set_block(new_loc, 0, s.Cov.block(old_loc, 0, total_size, old_size));
  assert(var.var->kind == K_IMU && var.off == 0 && var.size == 6);
  auto pose = make_pose();
  for (int k = 0; k < 7; k++) {
    pose->val[k] = var.var->val[k];
    pose->fej[k] = var.var->fej[k];
  }
  pose->id = new_loc;
  s.variables.push_back(pose);
  return pose;
}

// StateHelper.cpp:407-470: Givens rotations separating the landmark's rows (H_L, H_R and res are
// rotated in place), then the chi2 of the update rows (returned; Hup / resup receive those rows)
double initialize_split(const State &s, const std::vector<Ref> &H_order, Mat &H_R, Mat &H_L, double sigma2, Mat &res,
                        Mat &Hup, Mat &resup) {
  int new_var_size = H_L.c;
  Givens G;
  for (int n = 0; n < H_L.c; ++n) {
    for (int m = H_L.r - 1; m > n; m--) {
      G.make(H_L(m - 1, n), H_L(m, n));
      for (int j = n; j < H_L.c; j++) G.apply(H_L(m - 1, j), H_L(m, j));
      G.apply(res[m - 1], res[m]);
      for (int j = 0; j < H_R.c; j++) G.apply(H_R(m - 1, j), H_R(m, j));
    }
  }
  int nup = H_R.r - new_var_size;
  Hup = H_R.block(new_var_size, 0, nup, H_R.c);
  resup = res.block(new_var_size, 0, nup, 1);
  Mat P_up = get_marginal_covariance(s, H_order);
  Mat S = Hup * P_up * Hup.T();
  for (int i = 0; i < nup; i++) S(i, i) += sigma2;
  Mat sol = resup;
  llt_solve(S, sol);
  return dot(resup, sol);
}

// StateHelper.cpp:393-482. R = sigma2 * I (isotropic, asserted in the reference)
bool initialize(State &s, VarP new_var, const std::vector<Ref> &H_order, Mat &H_R, Mat &H_L, double sigma2, Mat &res,
                double chi2_mult, int *status) {
  *status = 0;
  int new_var_size = new_var->size;
  assert(new_var_size == H_L.c);
  Mat Hup, resup;
  double chi2 = initialize_split(s, H_order, H_R, H_L, sigma2, res, Hup, resup);
  Mat Hxinit = H_R.block(0, 0, new_var_size, H_R.c);
  Mat H_finit = H_L.block(0, 0, new_var_size, new_var_size);
  Mat resinit = res.block(0, 0, new_var_size, 1);
  Mat Rinit = sigma2 * Mat::Identity(new_var_size);
  int nup = Hup.r;
  double chi2_check = chi2_quantile95(res.r);
  if (chi2 > chi2_mult * chi2_check) return false;
  initialize_invertible(s, new_var, H_order, Hxinit, H_finit, Rinit, resinit);
  if (nup > 0) {
    if (!EKFUpdate(s, H_order, Hup, resup, sigma2)) *status = -1;
  }
  return true;
}

// StateHelper.cpp:484-577
void initialize_invertible(State &s, VarP new_var, const std::vector<Ref> &H_order, const Mat &H_R, const Mat &H_L,
                           const Mat &R, const Mat &res) {
  int N = s.Cov.r, r = res.r;
  Mat M_a(N, r);
  std::vector<int> H_id;
  int current_it = 0;
  for (auto &m : H_order) {
    H_id.push_back(current_it);
    current_it += m.size;
  }
  for (auto &var : s.variables) {
    Mat M_i(var->size, r);
    for (size_t i = 0; i < H_order.size(); i++) {
      const Ref &mv = H_order[i];
      M_i = M_i + s.Cov.block(var->id, mv.id(), var->size, mv.size) * H_R.block(0, H_id[i], H_R.r, mv.size).T();
    }
    M_a.set_block(var->id, 0, M_i);
  }
  Mat P_small = get_marginal_covariance(s, H_order);
  Mat M = H_R * P_small * H_R.T() + R;
  // M.selfadjointView<Upper>()
  for (int i = 0; i < M.r; i++)
    for (int j = 0; j < i; j++) M(i, j) = M(j, i);
  Mat H_Linv = colpiv_qr_solve(H_L, Mat::Identity(H_L.r));  // H_L.inverse()
  Mat P_LL = H_Linv * M * H_Linv.T();
  int oldSize = N;
  s.Cov.conservative_resize(oldSize + new_var->size, oldSize + new_var->size);
  Mat cross = -(M_a * H_Linv.T());
  s.Cov.set_block(0, oldSize, cross);
  s.Cov.set_block(oldSize, 0, cross.T());
  s.Cov.set_block(oldSize, oldSize, P_LL);
  new_var->update(H_Linv * res);
  new_var->id = oldSize;
  s.variables.push_back(new_var);
}

// StateHelper.cpp:579-616
void augment_clone(State &s, const Mat &last_w) {
  assert(s.clones.find(s.timestamp) == s.clones.end());
  VarP pose = clone(s, imu_pose_ref(s));
  s.clones[s.timestamp] = pose;
  if (s.opt.do_calib_camera_timeoffset) {
    Mat dnc_dt(6, 1);
    for (int k = 0; k < 3; k++) {
      dnc_dt[k] = last_w[k];
      dnc_dt[3 + k] = s.imu->vel()[k];
    }
    int N = s.Cov.r;
    s.Cov.add_block(0, pose->id, s.Cov.block(0, s.calib_dt->id, N, 1) * dnc_dt.T());
    s.Cov.add_block(pose->id, 0, dnc_dt * s.Cov.block(s.calib_dt->id, 0, 1, N));
  }
}

// StateHelper.cpp:618-629
void marginalize_old_clone(State &s) {
  if ((int)s.clones.size() > s.opt.max_clone_size) {
    double t = s.margtimestep();
    marginalize(s, s.clones.at(t));
    s.clones.erase(t);
  }
}

// StateHelper.cpp:631-645
void marginalize_slam(State &s) {
  auto it0 = s.features_SLAM.begin();
  while (it0 != s.features_SLAM.end()) {
    if (it0->second->should_marg && (int)it0->first > 4 * s.opt.max_aruco_features) {
      marginalize(s, it0->second);
      it0 = s.features_SLAM.erase(it0);
    } else {
      it0++;
    }
  }
}

}  // namespace StateHelper

// ---- chi-squared 0.95 quantile (boost::math::quantile(chi_squared(dof), 0.95)) ----
// Regularized lower incomplete gamma P(a,x) by series / continued fraction, then bisection+Newton.
static double gammp(double a, double x) {
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
  double b = x + 1.0 - a, c = 1.0 / 1e-300, d = 1.0 / b, h = d;
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
  double k = dof;
  double a = 0.5 * k;
  double lo = 0, hi = std::max(10.0, 4 * k + 50);
  for (int it = 0; it < 200; it++) {
    double mid = 0.5 * (lo + hi);
    if (gammp(a, 0.5 * mid) < 0.95)
      lo = mid;
    else
      hi = mid;
    if (hi - lo < 1e-14 * std::max(1.0, hi)) break;
  }
  return 0.5 * (lo + hi);
}

}  // namespace orc
