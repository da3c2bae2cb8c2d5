// ORACLE — test infrastructure only (see la.h header).
// Probes of single restated routines on a handle's current state, for the independent finite-difference and
// exact-answer goldens of SURVEY.md §8(c) (tests/test_fd_goldens.py).  Nothing here is used by the estimator.
//   orc_probe_boxplus            Type::update of every variable (ov_core/src/types/*.h, StateHelper.cpp:185-188)
//   orc_probe_predict            Propagator::predict_and_compute (Propagator.cpp:395-480): one IMU interval's mean
//                                and F (compute_F_and_G_analytic :683-828, compute_H_Dw/Da/Tg :964-1015)
//   orc_probe_uwb                UVioUpdaterHelper::get_uwb_jacobian_single (UVioUpdaterHelper.cpp:147-241)
//   orc_probe_feature_jacobian   UpdaterHelper::get_feature_jacobian_full (UpdaterHelper.cpp:192-424) for a
//                                landmark given in any LandmarkRepresentation (Landmark.cpp:26-144)
//   orc_probe_triangulate        FeatureInitializer::single_triangulation + single_gaussnewton
//                                (FeatureInitializer.cpp:30-375)
#include <cstring>
#include <string>

#include "handle.h"

using namespace orc;


namespace {

// H_x column blocks -> (covariance id, size) pairs
int write_order(const std::vector<Ref> &order, int *ids, int *sizes, int cap, int *n) {
  *n = (int)order.size();
  if ((int)order.size() > cap) return UVIO_HP_E_CAPACITY;
  for (size_t i = 0; i < order.size(); i++) {
    ids[i] = order[i].id();
    sizes[i] = order[i].size;
  }
  return 0;
}

void write_mat(const Mat &M, double *out) {
  for (int i = 0; i < M.r; i++)
    for (int j = 0; j < M.c; j++) out[(size_t)i * M.c + j] = M(i, j);
}

ClonesCam clones_cam_of(State &s) {
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

// a Feature with the given measurements, appended in order (FeatureDatabase::update_feature)
Feature make_feature(size_t featid, int nmeas, const int *cams, const double *times, const float *uv, const float *uvn) {
  Feature f;
  f.featid = featid;
  for (int i = 0; i < nmeas; i++) {
    size_t c = (size_t)cams[i];
    f.uvs[c].push_back({uv[2 * i], uv[2 * i + 1]});
    f.uvs_norm[c].push_back({uvn[2 * i], uvn[2 * i + 1]});
    f.timestamps[c].push_back(times[i]);
  }
  return f;
}

}  // namespace

extern "C" {

// x <- x boxplus dx over every variable of the state (dx indexed by covariance id); camera models follow the
// intrinsics (StateHelper.cpp:190-195)
int orc_probe_boxplus(orc_handle *h, const double *dx, int n) {
  State &s = h->m.state;
  if (n != s.Cov.r) return UVIO_HP_E_ARG;
  for (auto &v : s.variables) {
    Mat d(v->size, 1);
    for (int i = 0; i < v->size; i++) d[i] = dx[v->id + i];
    v->update(d);
  }
  if (s.opt.do_calib_camera_intrinsics)
    for (auto &c : s.cam_intrinsics)
      for (int i = 0; i < 8; i++) s.cams.at(c.first).v[i] = c.second->val[i];
  return 0;
}

// one IMU interval [dm, dp] (t, wm[3], am[3] each): the IMU mean is replaced by the prediction; F (n x n,
// n = 15 + IMU intrinsics) in the propagator's phi order, whose variables go to ids / sizes
int orc_probe_predict(orc_handle *h, const double dm[7], const double dp[7], double *F, double *Qd, int cap, int *n,
                      int *ids, int *sizes, int capv, int *nv) {
  State &s = h->m.state;
  ImuData a{dm[0], {dm[1], dm[2], dm[3]}, {dm[4], dm[5], dm[6]}};
  ImuData b{dp[0], {dp[1], dp[2], dp[3]}, {dp[4], dp[5], dp[6]}};
  Mat Fm, Qm;
  h->m.prop.predict_and_compute(s, a, b, Fm, Qm);
  *n = Fm.r;
  if ((size_t)Fm.r * Fm.c > (size_t)cap) return UVIO_HP_E_CAPACITY;
  if (F) write_mat(Fm, F);
  if (Qd) write_mat(Qm, Qd);
  return write_order(h->m.prop.phi_order(s), ids, sizes, capv, nv);
}

// predicted range (range - residual with range 0) and H_x of one anchor; H_x has *ncols columns over the
// variables ids / sizes
int orc_probe_uwb(orc_handle *h, uint64_t anchor_id, double *pred, double *H, int cap, int *ncols, int *ids, int *sizes,
                  int capv, int *nv) {
  State &s = h->m.state;
  auto it = s.anchors.find((size_t)anchor_id);
  if (it == s.anchors.end()) return UVIO_HP_E_ARG;
  Mat res, H_x;
  std::vector<Ref> order;
  uwb_jacobian_single(s, it->second, 0.0, res, H_x, order);
  *pred = -res[0];
  *ncols = H_x.c;
  if (H_x.c > cap) return UVIO_HP_E_CAPACITY;
  write_mat(H_x, H);
  return write_order(order, ids, sizes, capv, nv);
}

// residual (2 nmeas), H_f (2 nmeas x dim(rep)) and H_x (2 nmeas x *ncols) of a landmark whose value in its
// representation is lambda (3 values; 1 for ANCHORED_INVERSE_DEPTH_SINGLE, with its anchor bearing uvn0[2]);
// relative representations are anchored at clone anchor_time of camera anchor_cam.  The landmark's first
// estimate equals its value; the state's first estimates are the handle's.
int orc_probe_feature_jacobian(orc_handle *h, int rep, int nmeas, const int *cams, const double *times, const float *uv,
                               const float *uvn, const double *lambda, const double *uvn0, int anchor_cam,
                               double anchor_time, double *res, double *H_f, double *H_x, int cap, int *ncols, int *ids,
                               int *sizes, int capv, int *nv) {
  State &s = h->m.state;
  if (rep < 0 || rep > ANCHORED_INVERSE_DEPTH_SINGLE) return UVIO_HP_E_ARG;
  Feature f = make_feature(1, nmeas, cams, times, uv, uvn);
  const int dim = rep == ANCHORED_INVERSE_DEPTH_SINGLE ? 1 : 3;
  Var lm(K_LANDMARK, dim, dim);
  lm.rep = rep;
  for (int i = 0; i < dim; i++) lm.val[i] = lm.fej[i] = lambda[i];
  if (rep == ANCHORED_INVERSE_DEPTH_SINGLE) {
    lm.uvn0 = V3(uvn0[0], uvn0[1], 1.0);
    lm.uvn0_fej = lm.uvn0;
  }
  HelperFeature feat;
  feat.featid = 1;
  feat.f = &f;
  feat.rep = rep;
  if (is_relative(rep)) {
    feat.anchor_cam_id = anchor_cam;
    feat.anchor_clone_timestamp = anchor_time;
    feat.p_FinA = lm.get_xyz(false);
    feat.p_FinA_fej = lm.get_xyz(true);
  } else {
    feat.p_FinG = lm.get_xyz(false);
    feat.p_FinG_fej = lm.get_xyz(true);
  }
  Mat Hf, Hx, r;
  std::vector<Ref> order;
  UpdaterHelper::get_feature_jacobian_full(s, feat, Hf, Hx, r, order);
  *ncols = Hx.c;
  if (Hx.c > cap || Hf.c != dim) return UVIO_HP_E_CAPACITY;
  write_mat(r, res);
  write_mat(Hf, H_f);
  write_mat(Hx, H_x);
  return write_order(order, ids, sizes, capv, nv);
}

// single_triangulation (or _1d per the options) then, if refine, single_gaussnewton on the given measurements
// and the state's clones: out = [p_FinG(3), p_FinA(3)], anchor cam / time; returns 1 (success), 0 (rejected)
int orc_probe_triangulate(orc_handle *h, int nmeas, const int *cams, const double *times, const float *uv,
                          const float *uvn, int refine, double *out, int *anchor_cam, double *anchor_time) {
  State &s = h->m.state;
  Feature f = make_feature(1, nmeas, cams, times, uv, uvn);
  ClonesCam cc = clones_cam_of(s);
  FeatureInitializer init(s.opt);
  bool ok = init.o.fi_triangulate_1d ? init.single_triangulation_1d(f, cc) : init.single_triangulation(f, cc);
  if (ok && refine) ok = init.single_gaussnewton(f, cc);
  for (int k = 0; k < 3; k++) {
    out[k] = f.p_FinG[k];
    out[3 + k] = f.p_FinA[k];
  }
  *anchor_cam = f.anchor_cam_id;
  *anchor_time = f.anchor_clone_timestamp;
  return ok ? 1 : 0;
}

}  // extern "C"
