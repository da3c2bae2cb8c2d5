// ORACLE — test infrastructure only (see la.h header).
#include "updater.h"
#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <map>

namespace orc {

namespace UpdaterHelper {

// UpdaterHelper.cpp:32-190
void get_feature_jacobian_representation(State &s, HelperFeature &feature, Mat &H_f, std::vector<Mat> &H_x,
                                         std::vector<Ref> &x_order) {
  if (feature.rep == GLOBAL_3D) {
    H_f = Mat::Identity(3);
    return;
  }
  if (feature.rep == GLOBAL_FULL_INVERSE_DEPTH) {
    Mat p_FinG = s.opt.do_fej ? feature.p_FinG_fej : feature.p_FinG;
    double g_rho = 1 / norm(p_FinG);
    double g_phi = std::acos(g_rho * p_FinG[2]);
    double g_theta = std::atan2(p_FinG[1], p_FinG[0]);
    double sin_th = std::sin(g_theta), cos_th = std::cos(g_theta), sin_phi = std::sin(g_phi), cos_phi = std::cos(g_phi);
    double rho = g_rho;
    H_f = Mat(3, 3);
    H_f(0, 0) = -(1.0 / rho) * sin_th * sin_phi;
    H_f(0, 1) = (1.0 / rho) * cos_th * cos_phi;
    H_f(0, 2) = -(1.0 / (rho * rho)) * cos_th * sin_phi;
    H_f(1, 0) = (1.0 / rho) * cos_th * sin_phi;
    H_f(1, 1) = (1.0 / rho) * sin_th * cos_phi;
    H_f(1, 2) = -(1.0 / (rho * rho)) * sin_th * sin_phi;
    H_f(2, 0) = 0.0;
    H_f(2, 1) = -(1.0 / rho) * sin_phi;
    H_f(2, 2) = -(1.0 / (rho * rho)) * cos_phi;
    return;
  }
  assert(feature.anchor_cam_id != -1);
  VarP calib = s.calib_IMUtoCAM.at(feature.anchor_cam_id);
  VarP anchor = s.clones.at(feature.anchor_clone_timestamp);
  Mat R_ItoC = calib->Rot(), p_IinC = calib->pos();
  Mat R_GtoI = anchor->Rot(), p_IinG = anchor->pos();
  Mat p_FinA = feature.p_FinA;
  if (s.opt.do_fej) {
    Mat p_FinG_best = R_GtoI.T() * R_ItoC.T() * (feature.p_FinA - p_IinC) + p_IinG;
    R_GtoI = anchor->Rot_fej();
    p_IinG = anchor->pos_fej();
    p_FinA = (R_GtoI.T() * R_ItoC.T()).T() * (p_FinG_best - p_IinG) + p_IinC;
  }
  Mat R_CtoG = R_GtoI.T() * R_ItoC.T();
  Mat H_anc(3, 6);
  H_anc.set_block(0, 0, -(R_GtoI.T() * skew_x(R_ItoC.T() * (p_FinA - p_IinC))));
  H_anc.set_block(0, 3, Mat::Identity(3));
  x_order.push_back(ref_of(anchor));
  H_x.push_back(H_anc);
  if (s.opt.do_calib_camera_pose) {
    Mat H_calib(3, 6);
    H_calib.set_block(0, 0, -(R_CtoG * skew_x(p_FinA - p_IinC)));
    H_calib.set_block(0, 3, -R_CtoG);
    x_order.push_back(ref_of(calib));
    H_x.push_back(H_calib);
  }
  if (feature.rep == ANCHORED_3D) {
    H_f = R_CtoG;
    return;
  }
  if (feature.rep == ANCHORED_FULL_INVERSE_DEPTH) {
    double a_rho = 1 / norm(p_FinA);
    double a_phi = std::acos(a_rho * p_FinA[2]);
    double a_theta = std::atan2(p_FinA[1], p_FinA[0]);
    double sin_th = std::sin(a_theta), cos_th = std::cos(a_theta), sin_phi = std::sin(a_phi), cos_phi = std::cos(a_phi);
    double rho = a_rho;
    Mat d(3, 3);
    d(0, 0) = -(1.0 / rho) * sin_th * sin_phi;
    d(0, 1) = (1.0 / rho) * cos_th * cos_phi;
    d(0, 2) = -(1.0 / (rho * rho)) * cos_th * sin_phi;
    d(1, 0) = (1.0 / rho) * cos_th * sin_phi;
    d(1, 1) = (1.0 / rho) * sin_th * cos_phi;
    d(1, 2) = -(1.0 / (rho * rho)) * sin_th * sin_phi;
    d(2, 1) = -(1.0 / rho) * sin_phi;
    d(2, 2) = -(1.0 / (rho * rho)) * cos_phi;
    H_f = R_CtoG * d;
    return;
  }
  if (feature.rep == ANCHORED_MSCKF_INVERSE_DEPTH) {
    double alpha = p_FinA[0] / p_FinA[2], beta = p_FinA[1] / p_FinA[2], rho = 1 / p_FinA[2];
    Mat d(3, 3);
    d(0, 0) = (1.0 / rho);
    d(0, 2) = -(1.0 / (rho * rho)) * alpha;
    d(1, 1) = (1.0 / rho);
    d(1, 2) = -(1.0 / (rho * rho)) * beta;
    d(2, 2) = -(1.0 / (rho * rho));
    H_f = R_CtoG * d;
    return;
  }
  if (feature.rep == ANCHORED_INVERSE_DEPTH_SINGLE) {
    double rho = 1.0 / p_FinA[2];
    Mat bearing = rho * p_FinA;
    Mat d = (-(1.0 / (rho * rho))) * bearing;
    H_f = R_CtoG * d;
    return;
  }
  assert(false);
}

// UpdaterHelper.cpp:192-424
void get_feature_jacobian_full(State &s, HelperFeature &feature, Mat &H_f, Mat &H_x, Mat &res,
                               std::vector<Ref> &x_order) {
  const Feature &F = *feature.f;
  int total_meas = 0;
  for (auto const &pair : F.timestamps) total_meas += (int)pair.second.size();
  int total_hx = 0;
  std::map<const Var *, int> map_hx;
  for (auto const &pair : F.timestamps) {
    VarP calibration = s.calib_IMUtoCAM.at(pair.first);
    VarP distortion = s.cam_intrinsics.at(pair.first);
    if (s.opt.do_calib_camera_pose) {
      map_hx.insert({calibration.get(), total_hx});
      x_order.push_back(ref_of(calibration));
      total_hx += calibration->size;
    }
    if (s.opt.do_calib_camera_intrinsics) {
      map_hx.insert({distortion.get(), total_hx});
      x_order.push_back(ref_of(distortion));
      total_hx += distortion->size;
    }
    for (size_t m = 0; m < pair.second.size(); m++) {
      VarP clone = s.clones.at(pair.second[m]);
      if (map_hx.find(clone.get()) == map_hx.end()) {
        map_hx.insert({clone.get(), total_hx});
        x_order.push_back(ref_of(clone));
        total_hx += clone->size;
      }
    }
  }
  if (is_relative(feature.rep)) {
    VarP clone_Ai = s.clones.at(feature.anchor_clone_timestamp);
    if (map_hx.find(clone_Ai.get()) == map_hx.end()) {
      map_hx.insert({clone_Ai.get(), total_hx});
      x_order.push_back(ref_of(clone_Ai));
      total_hx += clone_Ai->size;
    }
    if (s.opt.do_calib_camera_pose) {
      VarP cc = s.calib_IMUtoCAM.at(feature.anchor_cam_id);
      if (map_hx.find(cc.get()) == map_hx.end()) {
        map_hx.insert({cc.get(), total_hx});
        x_order.push_back(ref_of(cc));
        total_hx += cc->size;
      }
    }
  }
  Mat p_FinG = feature.p_FinG;
  if (is_relative(feature.rep)) {
    VarP calib = s.calib_IMUtoCAM.at(feature.anchor_cam_id);
    VarP anchor = s.clones.at(feature.anchor_clone_timestamp);
    p_FinG = anchor->Rot().T() * calib->Rot().T() * (feature.p_FinA - calib->pos()) + anchor->pos();
  }
  Mat p_FinG_fej = feature.p_FinG_fej;
  if (is_relative(feature.rep)) p_FinG_fej = p_FinG;

  int c = 0;
  int jacobsize = (feature.rep != ANCHORED_INVERSE_DEPTH_SINGLE) ? 3 : 1;
  res = Mat(2 * total_meas, 1);
  H_f = Mat(2 * total_meas, jacobsize);
  H_x = Mat(2 * total_meas, total_hx);
  Mat dpfg_dlambda;
  std::vector<Mat> dpfg_dx;
  std::vector<Ref> dpfg_dx_order;
  get_feature_jacobian_representation(s, feature, dpfg_dlambda, dpfg_dx, dpfg_dx_order);

  for (auto const &pair : F.timestamps) {
    VarP distortion = s.cam_intrinsics.at(pair.first);
    VarP calibration = s.calib_IMUtoCAM.at(pair.first);
    const Camera &cam = s.cams.at(pair.first);
    Mat R_ItoC = calibration->Rot(), p_IinC = calibration->pos();
    for (size_t m = 0; m < pair.second.size(); m++) {
      VarP clone_Ii = s.clones.at(pair.second[m]);
      Mat R_GtoIi = clone_Ii->Rot(), p_IiinG = clone_Ii->pos();
      Mat p_FinIi = R_GtoIi * (p_FinG - p_IiinG);
      Mat p_FinCi = R_ItoC * p_FinIi + p_IinC;
      double xn = p_FinCi[0] / p_FinCi[2], yn = p_FinCi[1] / p_FinCi[2];
      double ud, vd;
      cam.distort_d(xn, yn, ud, vd);
      auto uvm = F.uvs.at(pair.first)[m];
      res[2 * c] = (double)uvm.first - ud;
      res[2 * c + 1] = (double)uvm.second - vd;
      if (const char *md = std::getenv("ORC_MEAS_DUMP")) {  // debug only
        FILE *fp = std::fopen(md, "ab");
        double rec[9] = {(double)feature.featid, (double)pair.first, xn, yn, ud, vd, (double)uvm.first, (double)uvm.second,
                         p_FinCi[2]};
        std::fwrite(rec, sizeof(double), 9, fp);
        std::fclose(fp);
      }
      if (s.opt.do_fej) {
        R_GtoIi = clone_Ii->Rot_fej();
        p_IiinG = clone_Ii->pos_fej();
        p_FinIi = R_GtoIi * (p_FinG_fej - p_IiinG);
        p_FinCi = R_ItoC * p_FinIi + p_IinC;
      }
      Mat dz_dzn, dz_dzeta;
      cam.distort_jacobian(xn, yn, dz_dzn, dz_dzeta);
      Mat dzn_dpfc(2, 3);
      dzn_dpfc(0, 0) = 1 / p_FinCi[2];
      dzn_dpfc(0, 2) = -p_FinCi[0] / (p_FinCi[2] * p_FinCi[2]);
      dzn_dpfc(1, 1) = 1 / p_FinCi[2];
      dzn_dpfc(1, 2) = -p_FinCi[1] / (p_FinCi[2] * p_FinCi[2]);
      Mat dpfc_dpfg = R_ItoC * R_GtoIi;
      Mat dpfc_dclone(3, 6);
      dpfc_dclone.set_block(0, 0, R_ItoC * skew_x(p_FinIi));
      dpfc_dclone.set_block(0, 3, -dpfc_dpfg);
      Mat dz_dpfc = dz_dzn * dzn_dpfc;
      Mat dz_dpfg = dz_dpfc * dpfc_dpfg;
      H_f.set_block(2 * c, 0, dz_dpfg * dpfg_dlambda);
      H_x.set_block(2 * c, map_hx[clone_Ii.get()], dz_dpfc * dpfc_dclone);
      for (size_t i = 0; i < dpfg_dx_order.size(); i++)
        H_x.add_block(2 * c, map_hx[dpfg_dx_order[i].var], dz_dpfg * dpfg_dx[i]);
      if (s.opt.do_calib_camera_pose) {
        Mat dpfc_dcalib(3, 6);
        dpfc_dcalib.set_block(0, 0, skew_x(p_FinCi - p_IinC));
        dpfc_dcalib.set_block(0, 3, Mat::Identity(3));
        H_x.add_block(2 * c, map_hx[calibration.get()], dz_dpfc * dpfc_dcalib);
      }
      if (s.opt.do_calib_camera_intrinsics) H_x.set_block(2 * c, map_hx[distortion.get()], dz_dzeta);
      c++;
    }
  }
}

// UpdaterHelper.cpp:426-454
void nullspace_project_inplace(Mat &H_f, Mat &H_x, Mat &res) {
  Givens G;
  for (int n = 0; n < H_f.c; ++n) {
    for (int m = H_f.r - 1; m > n; m--) {
      G.make(H_f(m - 1, n), H_f(m, n));
      for (int j = n; j < H_f.c; j++) G.apply(H_f(m - 1, j), H_f(m, j));
      for (int j = 0; j < H_x.c; j++) G.apply(H_x(m - 1, j), H_x(m, j));
      G.apply(res[m - 1], res[m]);
    }
  }
  H_x = H_x.block(H_f.c, 0, H_x.r - H_f.c, H_x.c);
  res = res.block(H_f.c, 0, res.r - H_f.c, res.c);
}

// UpdaterHelper.cpp:456-487
void measurement_compress_inplace(Mat &H_x, Mat &res) {
  if (H_x.r <= H_x.c) return;
  Givens G;
  for (int n = 0; n < H_x.c; n++) {
    for (int m = H_x.r - 1; m > n; m--) {
      G.make(H_x(m - 1, n), H_x(m, n));
      for (int j = n; j < H_x.c; j++) G.apply(H_x(m - 1, j), H_x(m, j));
      G.apply(res[m - 1], res[m]);
    }
  }
  int r = std::min(H_x.r, H_x.c);
  H_x.conservative_resize(r, H_x.c);
  res.conservative_resize(r, res.c);
}

}  // namespace UpdaterHelper

// Lock-step steering (updater.h FrameDebug, flip.h): run() once recording the near-tie casts; when
// miss() exceeds tol, re-run with one candidate cast rounded the other way (smallest margin first) until
// miss() <= tol.  Without a target, run() runs once, unobserved.
static const double kSteerThresh = 1e-9;  // casts recorded as candidates: relative margin below this
static const int kSteerMaxTries = 64;

template <class Run, class Miss>
static void steer_stage(FrameDebug *dbg, const SteerTarget *t, int kind, size_t featid, int stage, double tol, Run run,
                        Miss miss) {
  if (!t) {
    run();
    return;
  }
  FlipCtl ctl;
  ctl.thresh = kSteerThresh;
  {
    FlipScope fs(&ctl);
    run();
  }
  const double m0 = miss();
  if (!(m0 > tol)) return;
  auto cands = ctl.near;
  std::sort(cands.begin(), cands.end(), [](const std::pair<long, double> &a, const std::pair<long, double> &b) {
    return a.second < b.second || (a.second == b.second && a.first < b.first);
  });
  if ((int)cands.size() > kSteerMaxTries) cands.resize(kSteerMaxTries);
  for (const auto &c : cands) {
    FlipCtl f;
    f.thresh = 0;
    f.force = c.first;
    {
      FlipScope fs(&f);
      run();
    }
    const double m = miss();
    if (m <= tol) {
      dbg->log.push_back(SteerEvent{kind, featid, stage, c.first, c.second, m0, m, 1, (int)cands.size()});
      return;
    }
  }
  {
    FlipCtl f;
    f.thresh = 0;
    FlipScope fs(&f);
    run();
  }
  dbg->log.push_back(SteerEvent{kind, featid, stage, -1, 0.0, m0, miss(), 0, (int)cands.size()});
}

// stage 0 disagreement: the accept decision, then the triangulated position (m)
static double tri_miss(const SteerTarget *t, bool ok, const Feature &f) {
  const bool dev_ok = t->status != 1;
  if (ok != dev_ok) return INFINITY;
  if (!ok) return 0.0;
  double d = 0;
  for (int k = 0; k < 3; k++) d = std::max(d, std::fabs(f.p_FinG[k] - t->p_FinG[k]));
  return d;
}

// stage 1 disagreement: chi2 relative to max(|chi2|, 1) (tests/test_gpu_parity.py _compare_feats)
static double chi2_miss(const SteerTarget *t, double chi2) {
  if (t->status == 1) return 0.0;
  return std::fabs(chi2 - t->chi2) / std::max(std::fabs(t->chi2), 1.0);
}

static const double kTolP = 1e-9, kTolChi2 = 1e-11;  // the strict lock-step bounds

static ClonesCam make_clones_cam(State &s) {
  ClonesCam clones_cam;
  for (const auto &cc : s.calib_IMUtoCAM) {
    std::unordered_map<double, ClonePose> ci;
    for (const auto &ci_imu : s.clones) {
      Mat R_GtoCi = cc.second->Rot() * ci_imu.second->Rot();
      Mat p = ci_imu.second->pos() - R_GtoCi.T() * cc.second->pos();
      ci.insert({ci_imu.first, ClonePose{R_GtoCi, p}});
    }
    clones_cam.insert({cc.first, ci});
  }
  return clones_cam;
}

static void fill_chi2(std::map<int, double> &t) {
  for (int i = 1; i < 500; i++) t[i] = chi2_quantile95(i);
}

UpdaterMSCKF::UpdaterMSCKF(const uvio_hp_options_t &o)
    : sigma_pix_sq(o.msckf_sigma_pix * o.msckf_sigma_pix), chi2_mult(o.msckf_chi2_multipler), init(o) {
  fill_chi2(chi_squared_table);
}

// UpdaterMSCKF.cpp:58-295
int UpdaterMSCKF::update(State &s, std::vector<FeatP> &feature_vec, UpdateStats *st) {
  if (feature_vec.empty()) return 0;
  std::vector<double> clonetimes;
  for (const auto &c : s.clones) clonetimes.push_back(c.first);
  auto it0 = feature_vec.begin();
  while (it0 != feature_vec.end()) {
    (*it0)->clean_old_measurements(clonetimes);
    int ct_meas = 0;
    for (const auto &pair : (*it0)->timestamps) ct_meas += (int)pair.second.size();
    if (ct_meas < 2) {
      (*it0)->to_delete = true;
      it0 = feature_vec.erase(it0);
    } else {
      it0++;
    }
  }
  ClonesCam clones_cam = make_clones_cam(s);
  auto it1 = feature_vec.begin();
  while (it1 != feature_vec.end()) {
    bool ok = false;
    Feature &F = **it1;
    const SteerTarget *tg = dbg ? dbg->target(0, F.featid) : nullptr;
    steer_stage(
        dbg, tg, 0, F.featid, 0, kTolP,
        [&]() {
          bool ok_tri = init.o.fi_triangulate_1d ? init.single_triangulation_1d(F, clones_cam)
                                                 : init.single_triangulation(F, clones_cam);
          bool ok_ref = true;
          if (init.o.fi_refine_features) ok_ref = init.single_gaussnewton(F, clones_cam);
          ok = ok_tri && ok_ref;
        },
        [&]() { return tri_miss(tg, ok, F); });
    if (!ok) {
      if (st) st->feats.push_back(FeatDebug{(*it1)->featid, {0, 0, 0}, 1, -1.0});
      if (dbg) dbg->record(0, FeatDebug{(*it1)->featid, {0, 0, 0}, 1, -1.0});
      (*it1)->to_delete = true;
      it1 = feature_vec.erase(it1);
      continue;
    }
    it1++;
  }
  size_t max_meas_size = 0;
  for (auto &f : feature_vec)
    for (const auto &pair : f->timestamps) max_meas_size += 2 * pair.second.size();
  size_t max_hx_size = s.max_covariance_size();
  for (auto &l : s.features_SLAM) max_hx_size -= l.second->size;
  Mat res_big(max_meas_size, 1);
  Mat Hx_big(max_meas_size, max_hx_size);
  std::map<const Var *, int> Hx_mapping;
  std::vector<Ref> Hx_order_big;
  int ct_jacob = 0, ct_meas = 0;
  auto it2 = feature_vec.begin();
  while (it2 != feature_vec.end()) {
    HelperFeature feat;
    feat.featid = (*it2)->featid;
    feat.f = it2->get();
    feat.rep = s.opt.feat_rep_msckf;
    if (feat.rep == ANCHORED_INVERSE_DEPTH_SINGLE) feat.rep = ANCHORED_MSCKF_INVERSE_DEPTH;
    if (is_relative(feat.rep)) {
      feat.anchor_cam_id = (*it2)->anchor_cam_id;
      feat.anchor_clone_timestamp = (*it2)->anchor_clone_timestamp;
      feat.p_FinA = (*it2)->p_FinA;
      feat.p_FinA_fej = (*it2)->p_FinA;
    } else {
      feat.p_FinG = (*it2)->p_FinG;
      feat.p_FinG_fej = (*it2)->p_FinG;
    }
    Mat H_f, H_x, res;
    std::vector<Ref> Hx_order;
    double chi2 = 0;
    const SteerTarget *tg = dbg ? dbg->target(0, feat.featid) : nullptr;
    steer_stage(
        dbg, tg, 0, feat.featid, 1, kTolChi2,
        [&]() {
          H_f = Mat();
          H_x = Mat();
          res = Mat();
          Hx_order.clear();
          UpdaterHelper::get_feature_jacobian_full(s, feat, H_f, H_x, res, Hx_order);
          UpdaterHelper::nullspace_project_inplace(H_f, H_x, res);
          Mat P_marg = StateHelper::get_marginal_covariance(s, Hx_order);
          Mat S = H_x * P_marg * H_x.T();
          for (int i = 0; i < S.r; i++) S(i, i) += sigma_pix_sq;
          Mat sol = res;
          llt_solve(S, sol);
          chi2 = dot(res, sol);
        },
        [&]() { return chi2_miss(tg, chi2); });
    if (const char *dump = std::getenv("ORC_DUMP")) {  // debug: projected rows per feature
      FILE *fp = std::fopen(dump, "ab");
      std::vector<double> hdr = {(double)feat.featid, (double)H_x.r, (double)H_x.c};
      for (auto &rf : Hx_order)
        for (int k = 0; k < rf.size; k++) hdr.push_back(rf.id() + k);
      std::fwrite(hdr.data(), sizeof(double), hdr.size(), fp);
      for (int i = 0; i < H_x.r; i++) {
        for (int j = 0; j < H_x.c; j++) std::fwrite(&H_x(i, j), sizeof(double), 1, fp);
        std::fwrite(&res[i], sizeof(double), 1, fp);
      }
      std::fclose(fp);
    }
    double chi2_check = (res.r < 500) ? chi_squared_table[res.r] : chi2_quantile95(res.r);
    {
      FeatDebug d{(*it2)->featid, {(*it2)->p_FinG[0], (*it2)->p_FinG[1], (*it2)->p_FinG[2]}, 0, chi2};
      if (chi2 > chi2_mult * chi2_check) d.status = 3;
      if (st) st->feats.push_back(d);
      if (dbg) dbg->record(0, d);
    }
    if (chi2 > chi2_mult * chi2_check) {
      (*it2)->to_delete = true;
      it2 = feature_vec.erase(it2);
      continue;
    }
    int ct_hx = 0;
    for (const auto &var : Hx_order) {
      if (Hx_mapping.find(var.var) == Hx_mapping.end()) {
        Hx_mapping.insert({var.var, ct_jacob});
        Hx_order_big.push_back(var);
        ct_jacob += var.size;
      }
      Hx_big.set_block(ct_meas, Hx_mapping[var.var], H_x.block(0, ct_hx, H_x.r, var.size));
      ct_hx += var.size;
    }
    res_big.set_block(ct_meas, 0, res);
    ct_meas += res.r;
    it2++;
  }
  for (auto &f : feature_vec) f->to_delete = true;
  if (st) {
    st->accepted = (int)feature_vec.size();
    st->rows_stacked = ct_meas;
    st->cols = ct_jacob;
  }
  if (ct_meas < 1) return 0;
  res_big.conservative_resize(ct_meas, 1);
  Hx_big.conservative_resize(ct_meas, ct_jacob);
  UpdaterHelper::measurement_compress_inplace(Hx_big, res_big);
  if (st) st->rows_compressed = Hx_big.r;
  if (Hx_big.r < 1) return 0;
  if (!StateHelper::EKFUpdate(s, Hx_order_big, Hx_big, res_big, sigma_pix_sq)) return UVIO_HP_E_NUMERIC;
  return 0;
}

UpdaterSLAM::UpdaterSLAM(const uvio_hp_options_t &o)
    : sigma_pix_sq(o.slam_sigma_pix * o.slam_sigma_pix), chi2_mult(o.slam_chi2_multipler), init(o) {
  fill_chi2(chi_squared_table);
}

// UpdaterSLAM.cpp:61-251 (aruco branches omitted: no aruco tracker in the target configs)
int UpdaterSLAM::delayed_init(State &s, std::vector<FeatP> &feature_vec) {
  if (feature_vec.empty()) return 0;
  std::vector<double> clonetimes;
  for (const auto &c : s.clones) clonetimes.push_back(c.first);
  auto it0 = feature_vec.begin();
  while (it0 != feature_vec.end()) {
    (*it0)->clean_old_measurements(clonetimes);
    int ct_meas = 0;
    for (const auto &pair : (*it0)->timestamps) ct_meas += (int)pair.second.size();
    if (ct_meas < 2) {
      (*it0)->to_delete = true;
      it0 = feature_vec.erase(it0);
    } else {
      it0++;
    }
  }
  ClonesCam clones_cam = make_clones_cam(s);
  auto it1 = feature_vec.begin();
  while (it1 != feature_vec.end()) {
    bool ok = false;
    Feature &F = **it1;
    const SteerTarget *tg = dbg ? dbg->target(2, F.featid) : nullptr;
    steer_stage(
        dbg, tg, 2, F.featid, 0, kTolP,
        [&]() {
          bool ok_tri = init.o.fi_triangulate_1d ? init.single_triangulation_1d(F, clones_cam)
                                                 : init.single_triangulation(F, clones_cam);
          bool ok_ref = true;
          if (init.o.fi_refine_features) ok_ref = init.single_gaussnewton(F, clones_cam);
          ok = ok_tri && ok_ref;
        },
        [&]() { return tri_miss(tg, ok, F); });
    if (!ok) {
      if (dbg) dbg->record(2, FeatDebug{(*it1)->featid, {0, 0, 0}, 1, 0.0});
      (*it1)->to_delete = true;
      it1 = feature_vec.erase(it1);
      continue;
    }
    it1++;
  }
  auto it2 = feature_vec.begin();
  while (it2 != feature_vec.end()) {
    HelperFeature feat;
    feat.featid = (*it2)->featid;
    feat.f = it2->get();
    int feat_rep = s.opt.feat_rep_slam;
    feat.rep = feat_rep;
    if (feat_rep == ANCHORED_INVERSE_DEPTH_SINGLE) feat.rep = ANCHORED_MSCKF_INVERSE_DEPTH;
    if (is_relative(feat.rep)) {
      feat.anchor_cam_id = (*it2)->anchor_cam_id;
      feat.anchor_clone_timestamp = (*it2)->anchor_clone_timestamp;
      feat.p_FinA = (*it2)->p_FinA;
      feat.p_FinA_fej = (*it2)->p_FinA;
    } else {
      feat.p_FinG = (*it2)->p_FinG;
      feat.p_FinG_fej = (*it2)->p_FinG;
    }
    Mat H_f, H_x, res;
    std::vector<Ref> Hx_order;
    double chi2 = 0;
    const SteerTarget *tg = dbg ? dbg->target(2, feat.featid) : nullptr;
    steer_stage(
        dbg, tg, 2, feat.featid, 1, kTolChi2,
        [&]() {
          H_f = Mat();
          H_x = Mat();
          res = Mat();
          Hx_order.clear();
          UpdaterHelper::get_feature_jacobian_full(s, feat, H_f, H_x, res, Hx_order);
          if (feat_rep == ANCHORED_INVERSE_DEPTH_SINGLE) {
            Mat H_xf(H_x.r, H_x.c + 1);
            H_xf.set_block(0, 0, H_x);
            H_xf.set_block(0, H_x.c, H_f.block(0, H_f.c - 1, H_f.r, 1));
            Mat H_fb = H_f.block(0, 0, H_f.r, H_f.c - 1);
            UpdaterHelper::nullspace_project_inplace(H_fb, H_xf, res);
            H_x = H_xf.block(0, 0, H_xf.r, H_xf.c - 1);
            H_f = H_xf.block(0, H_xf.c - 1, H_xf.r, 1);
          }
          if (dbg) {  // initialize's chi2 on copies (the state is not touched)
            Mat a = H_x, b = H_f, r = res, Hup, resup;
            chi2 = StateHelper::initialize_split(s, Hx_order, a, b, sigma_pix_sq, r, Hup, resup);
          }
        },
        [&]() { return chi2_miss(tg, chi2); });
    int landmark_size = (feat_rep == ANCHORED_INVERSE_DEPTH_SINGLE) ? 1 : 3;
    auto landmark = std::make_shared<Var>(K_LANDMARK, landmark_size, landmark_size);
    landmark->featid = feat.featid;
    landmark->rep = feat_rep;
    landmark->unique_cam = (*it2)->anchor_cam_id;
    if (is_relative(feat.rep)) {
      landmark->anchor_cam = feat.anchor_cam_id;
      landmark->anchor_time = feat.anchor_clone_timestamp;
      landmark->set_from_xyz(feat.p_FinA, false);
      landmark->set_from_xyz(feat.p_FinA_fej, true);
    } else {
      landmark->set_from_xyz(feat.p_FinG, false);
      landmark->set_from_xyz(feat.p_FinG_fej, true);
    }
    int st = 0;
    const Mat p_tri = (*it2)->p_FinG;
    const bool init_ok = StateHelper::initialize(s, landmark, Hx_order, H_x, H_f, sigma_pix_sq, res, chi2_mult, &st);
    if (dbg) dbg->record(2, FeatDebug{feat.featid, {p_tri[0], p_tri[1], p_tri[2]}, init_ok ? 0 : 3, chi2});
    if (init_ok) {
      if (st < 0) return UVIO_HP_E_NUMERIC;
      s.features_SLAM.insert({(*it2)->featid, landmark});
      (*it2)->to_delete = true;
      it2++;
    } else {
      (*it2)->to_delete = true;
      it2 = feature_vec.erase(it2);
    }
  }
  return 0;
}

// UpdaterSLAM.cpp:253-479
int UpdaterSLAM::update(State &s, std::vector<FeatP> &feature_vec) {
  if (feature_vec.empty()) return 0;
  std::vector<double> clonetimes;
  for (const auto &c : s.clones) clonetimes.push_back(c.first);
  auto it0 = feature_vec.begin();
  while (it0 != feature_vec.end()) {
    (*it0)->clean_old_measurements(clonetimes);
    int ct_meas = 0;
    for (const auto &pair : (*it0)->timestamps) ct_meas += (int)pair.second.size();
    VarP landmark = s.features_SLAM.at((*it0)->featid);
    int required = (landmark->rep == ANCHORED_INVERSE_DEPTH_SINGLE) ? 2 : 1;
    if (ct_meas < 1) {
      (*it0)->to_delete = true;
      it0 = feature_vec.erase(it0);
    } else if (ct_meas < required) {
      it0 = feature_vec.erase(it0);
    } else {
      it0++;
    }
  }
  size_t max_meas_size = 0;
  for (auto &f : feature_vec)
    for (const auto &pair : f->timestamps) max_meas_size += 2 * pair.second.size();
  size_t max_hx_size = s.max_covariance_size();
  Mat res_big(max_meas_size, 1);
  Mat Hx_big(max_meas_size, max_hx_size);
  std::map<const Var *, int> Hx_mapping;
  std::vector<Ref> Hx_order_big;
  int ct_jacob = 0, ct_meas = 0;
  auto it2 = feature_vec.begin();
  while (it2 != feature_vec.end()) {
    VarP landmark = s.features_SLAM.at((*it2)->featid);
    HelperFeature feat;
    feat.featid = (*it2)->featid;
    feat.f = it2->get();
    feat.rep = landmark->rep;
    if (landmark->rep == ANCHORED_INVERSE_DEPTH_SINGLE) feat.rep = ANCHORED_MSCKF_INVERSE_DEPTH;
    if (is_relative(feat.rep)) {
      feat.anchor_cam_id = landmark->anchor_cam;
      feat.anchor_clone_timestamp = landmark->anchor_time;
      feat.p_FinA = landmark->get_xyz(false);
      feat.p_FinA_fej = landmark->get_xyz(true);
    } else {
      feat.p_FinG = landmark->get_xyz(false);
      feat.p_FinG_fej = landmark->get_xyz(true);
    }
    Mat H_f, H_x, res, H_xf;
    std::vector<Ref> Hx_order, Hxf_order;
    double chi2 = 0;
    const SteerTarget *tg = dbg ? dbg->target(1, feat.featid) : nullptr;
    steer_stage(
        dbg, tg, 1, feat.featid, 1, kTolChi2,
        [&]() {
          H_f = Mat();
          H_x = Mat();
          res = Mat();
          Hx_order.clear();
          UpdaterHelper::get_feature_jacobian_full(s, feat, H_f, H_x, res, Hx_order);
          if (landmark->rep == ANCHORED_INVERSE_DEPTH_SINGLE) {
            H_xf = Mat(H_x.r, H_x.c + 1);
            H_xf.set_block(0, 0, H_x);
            H_xf.set_block(0, H_x.c, H_f.block(0, H_f.c - 1, H_f.r, 1));
            Mat H_fb = H_f.block(0, 0, H_f.r, H_f.c - 1);
            UpdaterHelper::nullspace_project_inplace(H_fb, H_xf, res);
          } else {
            H_xf = Mat(H_x.r, H_x.c + H_f.c);
            H_xf.set_block(0, 0, H_x);
            H_xf.set_block(0, H_x.c, H_f);
          }
          Hxf_order = Hx_order;
          Hxf_order.push_back(ref_of(landmark));
          Mat P_marg = StateHelper::get_marginal_covariance(s, Hxf_order);
          Mat S = H_xf * P_marg * H_xf.T();
          for (int i = 0; i < S.r; i++) S(i, i) += sigma_pix_sq;
          Mat sol = res;
          llt_solve(S, sol);
          chi2 = dot(res, sol);
        },
        [&]() { return chi2_miss(tg, chi2); });
    double chi2_check = (res.r < 500) ? chi_squared_table[res.r] : chi2_quantile95(res.r);
    if (dbg) dbg->record(1, FeatDebug{feat.featid, {0, 0, 0}, chi2 > chi2_mult * chi2_check ? 3 : 0, chi2});
    if (chi2 > chi2_mult * chi2_check) {
      landmark->fail_count++;
      (*it2)->to_delete = true;
      it2 = feature_vec.erase(it2);
      continue;
    }
    int ct_hx = 0;
    for (const auto &var : Hxf_order) {
      if (Hx_mapping.find(var.var) == Hx_mapping.end()) {
        Hx_mapping.insert({var.var, ct_jacob});
        Hx_order_big.push_back(var);
        ct_jacob += var.size;
      }
      Hx_big.set_block(ct_meas, Hx_mapping[var.var], H_xf.block(0, ct_hx, H_xf.r, var.size));
      ct_hx += var.size;
    }
    res_big.set_block(ct_meas, 0, res);
    ct_meas += res.r;
    it2++;
  }
  for (auto &f : feature_vec) f->to_delete = true;
  if (ct_meas < 1) return 0;
  res_big.conservative_resize(ct_meas, 1);
  Hx_big.conservative_resize(ct_meas, ct_jacob);
  if (!StateHelper::EKFUpdate(s, Hx_order_big, Hx_big, res_big, sigma_pix_sq)) return UVIO_HP_E_NUMERIC;
  return 0;
}

// UpdaterSLAM.cpp:481-503
int UpdaterSLAM::change_anchors(State &s) {
  if ((int)s.clones.size() <= s.opt.max_clone_size) return 0;
  int changed = 0;
  double marg_timestep = s.margtimestep();
  for (auto &f : s.features_SLAM) {
    if (f.second->rep == GLOBAL_3D || f.second->rep == GLOBAL_FULL_INVERSE_DEPTH) continue;
    assert(marg_timestep <= f.second->anchor_time);
    if (f.second->anchor_time == marg_timestep) {
      int r = perform_anchor_change(s, f.second, s.timestamp, f.second->anchor_cam);
      if (r < 0) return r;
      changed++;
    }
  }
  return changed;
}

// UpdaterSLAM.cpp:505-647
int UpdaterSLAM::perform_anchor_change(State &s, VarP landmark, double new_anchor_timestamp, size_t new_cam_id) {
  HelperFeature old_feat;
  old_feat.featid = landmark->featid;
  old_feat.f = nullptr;
  old_feat.rep = landmark->rep;
  old_feat.anchor_cam_id = landmark->anchor_cam;
  old_feat.anchor_clone_timestamp = landmark->anchor_time;
  old_feat.p_FinA = landmark->get_xyz(false);
  old_feat.p_FinA_fej = landmark->get_xyz(true);
  Mat H_f_old;
  std::vector<Mat> H_x_old;
  std::vector<Ref> x_order_old;
  UpdaterHelper::get_feature_jacobian_representation(s, old_feat, H_f_old, H_x_old, x_order_old);
  HelperFeature new_feat;
  new_feat.featid = landmark->featid;
  new_feat.f = nullptr;
  new_feat.rep = landmark->rep;
  new_feat.anchor_cam_id = (int)new_cam_id;
  new_feat.anchor_clone_timestamp = new_anchor_timestamp;

  VarP cold = s.calib_IMUtoCAM.at(old_feat.anchor_cam_id), cnew = s.calib_IMUtoCAM.at(new_feat.anchor_cam_id);
  VarP iold = s.clones.at(old_feat.anchor_clone_timestamp), inew = s.clones.at(new_feat.anchor_clone_timestamp);
  Mat R_GtoOLD = cold->Rot() * iold->Rot();
  Mat p_OLDinG = iold->pos() - R_GtoOLD.T() * cold->pos();
  Mat R_GtoNEW = cnew->Rot() * inew->Rot();
  Mat p_NEWinG = inew->pos() - R_GtoNEW.T() * cnew->pos();
  Mat R_OLDtoNEW = R_GtoNEW * R_GtoOLD.T();
  Mat p_OLDinNEW = R_GtoNEW * (p_OLDinG - p_NEWinG);
  new_feat.p_FinA = R_OLDtoNEW * landmark->get_xyz(false) + p_OLDinNEW;
  Mat R_GtoOLD_fej = cold->Rot() * iold->Rot_fej();
  Mat p_OLDinG_fej = iold->pos_fej() - R_GtoOLD_fej.T() * cold->pos();
  Mat R_GtoNEW_fej = cnew->Rot() * inew->Rot_fej();
  Mat p_NEWinG_fej = inew->pos_fej() - R_GtoNEW_fej.T() * cnew->pos();
  Mat R_OLDtoNEW_fej = R_GtoNEW_fej * R_GtoOLD_fej.T();
  Mat p_OLDinNEW_fej = R_GtoNEW_fej * (p_OLDinG_fej - p_NEWinG_fej);
  new_feat.p_FinA_fej = R_OLDtoNEW_fej * landmark->get_xyz(true) + p_OLDinNEW_fej;

  Mat H_f_new;
  std::vector<Mat> H_x_new;
  std::vector<Ref> x_order_new;
  UpdaterHelper::get_feature_jacobian_representation(s, new_feat, H_f_new, H_x_new, x_order_new);

  std::vector<Ref> phi_order_NEW = {ref_of(landmark)};
  std::vector<Ref> phi_order_OLD;
  int current_it = 0;
  std::map<const Var *, int> Phi_id_map;
  for (const auto &var : x_order_old)
    if (Phi_id_map.find(var.var) == Phi_id_map.end()) {
      Phi_id_map.insert({var.var, current_it});
      phi_order_OLD.push_back(var);
      current_it += var.size;
    }
  for (const auto &var : x_order_new)
    if (Phi_id_map.find(var.var) == Phi_id_map.end()) {
      Phi_id_map.insert({var.var, current_it});
      phi_order_OLD.push_back(var);
      current_it += var.size;
    }
  Phi_id_map.insert({landmark.get(), current_it});
  phi_order_OLD.push_back(ref_of(landmark));
  current_it += landmark->size;
  int phisize = (new_feat.rep != ANCHORED_INVERSE_DEPTH_SINGLE) ? 3 : 1;
  Mat Phi(phisize, current_it), Q(phisize, phisize);
  Mat H_f_new_inv;
  if (phisize == 1) {
    double sq = dot(H_f_new, H_f_new);
    H_f_new_inv = (1.0 / sq) * H_f_new.T();
  } else {
    H_f_new_inv = colpiv_qr_solve(H_f_new, Mat::Identity(3));
  }
  for (size_t i = 0; i < H_x_old.size(); i++) Phi.add_block(0, Phi_id_map.at(x_order_old[i].var), H_f_new_inv * H_x_old[i]);
  Phi.set_block(0, Phi_id_map.at(landmark.get()), H_f_new_inv * H_f_old);
  for (size_t i = 0; i < H_x_new.size(); i++)
    Phi.add_block(0, Phi_id_map.at(x_order_new[i].var), -(H_f_new_inv * H_x_new[i]));
  if (!StateHelper::EKFPropagation(s, phi_order_NEW, phi_order_OLD, Phi, Q)) return UVIO_HP_E_NUMERIC;
  landmark->anchor_cam = new_feat.anchor_cam_id;
  landmark->anchor_time = new_feat.anchor_clone_timestamp;
  landmark->set_from_xyz(new_feat.p_FinA, false);
  landmark->set_from_xyz(new_feat.p_FinA_fej, true);
  landmark->has_anchor_change = true;
  return 0;
}

UpdaterUWB::UpdaterUWB(const uvio_hp_options_t &o) : sigma_range(o.uwb_sigma_range), chi2_mult(o.uwb_chi2_multipler) {
  fill_chi2(chi_squared_table);
}

// UVioUpdaterHelper::get_uwb_jacobian_single (UVioUpdaterHelper.cpp:147-241): residual and H_x of one range
void uwb_jacobian_single(State &s, const VarP &anchor, double range, Mat &res, Mat &H_x, std::vector<Ref> &x_order) {
  int total_hx = 0;
  Ref clone_I = imu_pose_ref(s);
  x_order.push_back(clone_I);
  int id_I = total_hx;
  total_hx += 6;
  int id_cal = -1, id_anc = -1;
  if (s.opt.do_calib_uwb_extrinsics) {
    x_order.push_back(ref_of(s.calib_UWBtoIMU));
    id_cal = total_hx;
    total_hx += 3;
  }
  if (!anchor->fixed) {
    x_order.push_back(ref_of(anchor));
    id_anc = total_hx;
    total_hx += 5;
  }
  Mat R_GtoI = s.imu->Rot(), p_IinG = s.imu->pos();
  Mat p_IinU = s.calib_UWBtoIMU->val;
  Mat p_AinG = anchor->val.block(0, 0, 3, 1);
  double const_bias = anchor->val[3], dist_bias = anchor->val[4];
  Mat d = p_AinG - (R_GtoI.T() * (-p_IinU) + p_IinG);
  double dn = norm(d);
  res = Mat(1, 1);
  res[0] = range - ((1 + dist_bias) * dn + const_bias);
  Mat H_n = (1.0 / dn) * d.T();
  Mat H_z_I(3, 6);
  H_z_I.set_block(0, 0, R_GtoI.T() * skew_x(-p_IinU));
  H_z_I.set_block(0, 3, -Mat::Identity(3));
  H_x = Mat(1, total_hx);
  H_x.set_block(0, id_I, (1 + dist_bias) * (H_n * H_z_I));
  if (id_cal >= 0) H_x.set_block(0, id_cal, (1 + dist_bias) * (H_n * R_GtoI.T()));
  if (id_anc >= 0) {
    Mat Ha(1, 5);
    // reference quirk, kept (UVioUpdaterHelper.cpp:236): the anchor-position block repeats the calibration
    // block's R_GtoI^T; d(range)/d(p_AinG) is (1 + dist_bias) H_n (tests/test_fd_goldens.py measures the gap)
    Ha.set_block(0, 0, (1 + dist_bias) * (H_n * R_GtoI.T()));
    Ha[3] = 1;
    Ha[4] = dn;
    H_x.set_block(0, id_anc, Ha);
  }
}

// UpdaterUWB.cpp:53-90
int UpdaterUWB::update_single(State &s, double timestamp, size_t anchor_id, double range) {
  (void)timestamp;
  auto ait = s.anchors.find(anchor_id);
  if (ait == s.anchors.end()) return 0;
  VarP anchor = ait->second;
  std::vector<Ref> x_order;
  Mat res, H_x;
  uwb_jacobian_single(s, anchor, range, res, H_x, x_order);
  double R = sigma_range * sigma_range;
  Mat P_marg = StateHelper::get_marginal_covariance(s, x_order);
  Mat S = H_x * P_marg * H_x.T();
  S(0, 0) += R;
  Mat sol = res;
  llt_solve(S, sol);
  double chi2 = dot(res, sol);
  if (chi2 > chi2_mult * chi_squared_table[1]) return 0;
  if (!StateHelper::EKFUpdate(s, x_order, H_x, res, R)) return UVIO_HP_E_NUMERIC;
  return 1;
}

}  // namespace orc
