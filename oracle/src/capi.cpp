// ORACLE — test infrastructure only (see la.h header).
// C ABI of the CPU restatement, mirroring include/uvio_hp.h entry points with an orc_ prefix so
// tests / bench.py's cpu_baseline leg can drive both implementations with identical inputs.
#include <cstring>
#include <string>

#include "handle.h"

using namespace orc;


extern "C" {

int orc_create(const uvio_hp_options_t *opts, orc_handle **out) {
  if (!opts || !out) return UVIO_HP_E_ARG;
  *out = new orc_handle(*opts);
  return 0;
}
int orc_destroy(orc_handle *h) {
  delete h;
  return 0;
}
int orc_initialize_with_gt(orc_handle *h, const double x[17]) {
  h->m.initialize_with_gt(x);
  return 0;
}
int orc_feed_imu(orc_handle *h, double t, const double wm[3], const double am[3]) {
  h->m.feed_imu(t, wm, am);
  return 0;
}
int orc_feed_simulation(orc_handle *h, double t, int ncam, const int *cam_ids, const int *counts, const uint64_t *ids,
                        const float *uv) {
  std::vector<int> camids(cam_ids, cam_ids + ncam);
  std::vector<std::vector<std::pair<size_t, std::pair<float, float>>>> feats(ncam);
  size_t k = 0;
  for (int i = 0; i < ncam; i++)
    for (int j = 0; j < counts[i]; j++, k++) feats[i].push_back({(size_t)ids[k], {uv[2 * k], uv[2 * k + 1]}});
  return h->m.feed_simulation(t, camids, feats);
}
int orc_feed_camera(orc_handle *h, double t, int ncam, const int *cam_ids, const uint8_t *const *imgs, const int *strides,
                    const uint8_t *const *masks) {
  std::vector<int> camids(cam_ids, cam_ids + ncam);
  std::vector<GrayImg> im(ncam), mk(ncam);
  // downsample_cameras (VioManager.cpp:270-278): the configured size is the halved one, the inputs are the
  // raw 2w x 2h images and both image and mask are pyrDown'ed before tracking
  const int f = h->m.o.downsample_cameras ? 2 : 1;
  for (int i = 0; i < ncam; i++) {
    const uvio_hp_camera_t &c = h->m.o.cams[cam_ids[i]];
    im[i].w = f * c.width;
    im[i].h = f * c.height;
    im[i].d.resize((size_t)im[i].w * im[i].h);
    for (int y = 0; y < im[i].h; y++)
      std::memcpy(&im[i].d[(size_t)y * im[i].w], imgs[i] + (size_t)y * strides[i], im[i].w);
    if (masks && masks[i]) {
      mk[i] = im[i];
      for (int y = 0; y < im[i].h; y++)
        std::memcpy(&mk[i].d[(size_t)y * im[i].w], masks[i] + (size_t)y * strides[i], im[i].w);
    }
    if (f == 2) {
      im[i] = pyr_down(im[i]);
      if (masks && masks[i]) mk[i] = pyr_down(mk[i]);
    }
  }
  return h->m.feed_camera(t, camids, im, mk);
}
int orc_feed_uwb(orc_handle *h, double t, int n, const uint64_t *anchor_ids, const double *ranges) {
  std::vector<std::pair<size_t, double>> r;
  for (int i = 0; i < n; i++) r.push_back({(size_t)anchor_ids[i], ranges[i]});
  return h->m.feed_uwb(t, r);
}
int orc_init_anchors(orc_handle *h, int n, const uvio_hp_anchor_t *a) {
  std::vector<uvio_hp_anchor_t> v(a, a + n);
  return h->m.init_anchors(v);
}
// StaticInitializer::initialize alone on an IMU window (CPU tests of its branches): 1 initialized (state16 =
// q p v bg ba, *t the state time), 0 not
int orc_static_initialize(const uvio_hp_options_t *opts, int n, const double *t, const double *wm, const double *am,
                          int wait_for_jerk, double *t_init, double state16[16]) {
  InertialInitializer ini(*opts);
  for (int i = 0; i < n; i++) {
    ImuData d;
    d.t = t[i];
    for (int k = 0; k < 3; k++) d.wm[k] = wm[3 * i + k], d.am[k] = am[3 * i + k];
    ini.imu_data.push_back(d);
  }
  Mat cov, x;
  if (!ini.static_initialize(t_init, cov, x, wait_for_jerk != 0)) return 0;
  for (int k = 0; k < 16; k++) state16[k] = x[k];
  return 1;
}
int orc_initialized(orc_handle *h, int *out) {
  *out = h->m.is_initialized ? 1 : 0;
  return 0;
}
int orc_get_imu_state(orc_handle *h, double *t, double out[16]) {
  *t = h->m.state.timestamp;
  for (int k = 0; k < 16; k++) out[k] = h->m.state.imu->val[k];
  return 0;
}
int orc_get_cov_dim(orc_handle *h, int *n) {
  *n = h->m.state.Cov.r;
  return 0;
}
int orc_get_cov(orc_handle *h, double *out, int ld) {
  const Mat &C = h->m.state.Cov;
  for (int i = 0; i < C.r; i++)
    for (int j = 0; j < C.c; j++) out[(size_t)i * ld + j] = C(i, j);
  return 0;
}
int orc_get_state_vector(orc_handle *h, double *out, int cap, int *len, int *meta, int meta_cap, int *nvars) {
  int k = 0, nv = 0;
  for (auto &v : h->m.state.variables) {
    if (meta && 3 * nv + 2 < meta_cap) {
      meta[3 * nv] = v->kind;
      meta[3 * nv + 1] = v->id;
      meta[3 * nv + 2] = v->size;
    }
    for (int i = 0; i < v->val.r; i++) {
      if (k < cap) out[k] = v->val[i];
      k++;
    }
    nv++;
  }
  *len = k;
  if (nvars) *nvars = nv;
  return k <= cap ? 0 : UVIO_HP_E_CAPACITY;
}
int orc_get_fej_vector(orc_handle *h, double *out, int cap, int *len) {
  int k = 0;
  for (auto &v : h->m.state.variables)
    for (int i = 0; i < v->fej.r; i++, k++)
      if (k < cap) out[k] = v->fej[i];
  *len = k;
  return k <= cap ? 0 : UVIO_HP_E_CAPACITY;
}
// lock-step parity: overwrite the mean, the FEJ values and the covariance with another
// implementation's (same variable layout required)
int orc_set_state(orc_handle *h, const double *val, const double *fej, int len, const double *P, int n) {
  int k = 0;
  for (auto &v : h->m.state.variables) k += v->val.r;
  if (k != len || n != h->m.state.Cov.r) return UVIO_HP_E_ARG;
  k = 0;
  for (auto &v : h->m.state.variables)
    for (int i = 0; i < v->val.r; i++, k++) {
      v->val[i] = val[k];
      v->fej[i] = fej[k];
    }
  std::memcpy(h->m.state.Cov.d.data(), P, sizeof(double) * n * n);
  // the camera models mirror the intrinsics after every update (StateHelper.cpp:190-195)
  if (h->m.state.opt.do_calib_camera_intrinsics)
    for (auto &c : h->m.state.cam_intrinsics)
      for (int i = 0; i < 8; i++) h->m.state.cams.at(c.first).v[i] = c.second->val[i];
  return 0;
}
int orc_get_timing(orc_handle *h, uvio_hp_timing_t *out) {
  *out = h->m.timing;
  return 0;
}
int orc_get_clone_times(orc_handle *h, double *out, int cap, int *n) {
  int k = 0;
  for (auto &c : h->m.state.clones) {
    if (k < cap) out[k] = c.first;
    k++;
  }
  *n = k;
  return 0;
}

// VioManager::get_active_tracks (retriangulate_active_tracks outputs)
int orc_get_active_tracks(orc_handle *h, double *t, uint64_t *ids, double *posinG, double *uvd, int *uvd_valid, int cap,
                          int *n) {
  const auto &P = h->m.active_tracks_posinG;
  const auto &U = h->m.active_tracks_uvd;
  *t = h->m.active_tracks_time;
  // tracks with a uvd but no position cannot exist (uvd is derived from the position)
  *n = (int)P.size();
  if ((int)P.size() > cap) return UVIO_HP_E_CAPACITY;
  int k = 0;
  for (const auto &kv : P) {
    ids[k] = (uint64_t)kv.first;
    for (int j = 0; j < 3; j++) posinG[3 * k + j] = kv.second[j];
    auto u = U.find(kv.first);
    uvd_valid[k] = u != U.end();
    for (int j = 0; j < 3; j++) uvd[3 * k + j] = (u != U.end()) ? u->second[j] : 0.0;
    k++;
  }
  return 0;
}

// ---- updater-level entries (include/uvio_hp.h "Updater-level boundary"), the reference's own calls ----
// Features from the flat arrays, measurements appended in order (FeatureDatabase::update_feature,
// FeatureDatabase.cpp:59-98); kept[i] = 1 when feature i is still in feature_vec after the updater
// (used by the update), to_delete[i] = Feature::to_delete.
static std::vector<FeatP> orc_features(int nfeat, const uint64_t *ids, const int *off, const uvio_hp_feat_meas_t *m) {
  std::vector<FeatP> fv;
  for (int i = 0; i < nfeat; i++) {
    auto f = std::make_shared<Feature>();
    f->featid = (size_t)ids[i];
    for (int k = off[i]; k < off[i + 1]; k++) {
      const size_t c = (size_t)m[k].cam;
      f->uvs[c].push_back({m[k].u, m[k].v});
      f->uvs_norm[c].push_back({m[k].un, m[k].vn});
      f->timestamps[c].push_back(m[k].t);
    }
    fv.push_back(f);
  }
  return fv;
}
static void orc_outcome(const std::vector<FeatP> &in, const std::vector<FeatP> &after, int *kept, int *to_delete) {
  for (size_t i = 0; i < in.size(); i++) {
    kept[i] = 0;
    for (auto &f : after)
      if (f == in[i]) kept[i] = 1;
    to_delete[i] = in[i]->to_delete ? 1 : 0;
  }
}
int orc_updater(orc_handle *h, int which, int nfeat, const uint64_t *ids, const int *off, const uvio_hp_feat_meas_t *m,
                int *kept, int *to_delete) {
  std::vector<FeatP> fv = orc_features(nfeat, ids, off, m);
  const std::vector<FeatP> in = fv;
  int rc = 0;
  if (which == 0)
    rc = h->m.msckf.update(h->m.state, fv, &h->m.last_msckf);
  else if (which == 1)
    rc = h->m.slam.update(h->m.state, fv);
  else
    rc = h->m.slam.delayed_init(h->m.state, fv);
  orc_outcome(in, fv, kept, to_delete);
  return rc;
}
int orc_propagate_and_clone(orc_handle *h, double t) {
  int st = 0;
  if (!h->m.prop.propagate_and_clone(h->m.state, t, &st)) return st ? st : UVIO_HP_E_NUMERIC;
  return 0;
}
int orc_slam_change_anchors(orc_handle *h) {
  int r = h->m.slam.change_anchors(h->m.state);
  return r < 0 ? r : 0;
}
int orc_marginalize_slam(orc_handle *h) {
  StateHelper::marginalize_slam(h->m.state);
  return 0;
}
int orc_marginalize_old_clone(orc_handle *h) {
  StateHelper::marginalize_old_clone(h->m.state);
  return 0;
}
int orc_uwb_update_single(orc_handle *h, double t, uint64_t anchor_id, double range, int *applied) {
  const int r = h->m.uwb.update_single(h->m.state, t, (size_t)anchor_id, range);
  if (r < 0) return r;
  *applied = r;
  return 0;
}

// StateHelper::EKFUpdate on a standalone covariance (variables = one Vec of size N)
int orc_ekf_update(double *P, int N, const int *H_index, int n, const double *H, int r, const double *res, double sigma2,
                   double *dx_out) {
  uvio_hp_options_t o;
  std::memset(&o, 0, sizeof(o));
  o.num_cameras = 0;
  State s(o);
  s.variables.clear();
  auto big = make_vec(N);
  big->id = 0;
  s.variables.push_back(big);
  s.Cov = Mat(N, N);
  std::memcpy(s.Cov.d.data(), P, sizeof(double) * N * N);
  // one size-1 reference per H column (H_order of scalar slices)
  std::vector<VarP> slices;
  std::vector<Ref> order;
  for (int j = 0; j < n; j++) order.push_back(Ref{big.get(), H_index[j], 1});
  Mat Hm(r, n), rm(r, 1);
  std::memcpy(Hm.d.data(), H, sizeof(double) * r * n);
  std::memcpy(rm.d.data(), res, sizeof(double) * r);
  Mat before = big->val;
  bool ok = StateHelper::EKFUpdate(s, order, Hm, rm, sigma2);
  std::memcpy(P, s.Cov.d.data(), sizeof(double) * N * N);
  for (int i = 0; i < N; i++) dx_out[i] = big->val[i] - before[i];
  return ok ? 0 : UVIO_HP_E_NUMERIC;
}

// UpdaterMSCKF.cpp:274-286: measurement_compress_inplace then EKFUpdate on a standalone covariance
int orc_msckf_compressed_update(double *P, int N, const int *H_index, int n, const double *H, int m, const double *res,
                                double sigma2, double *dx_out) {
  Mat Hm(m, n), rm(m, 1);
  std::memcpy(Hm.d.data(), H, sizeof(double) * m * n);
  std::memcpy(rm.d.data(), res, sizeof(double) * m);
  UpdaterHelper::measurement_compress_inplace(Hm, rm);
  if (Hm.r == 0) {
    for (int i = 0; i < N; i++) dx_out[i] = 0.0;
    return 0;
  }
  return orc_ekf_update(P, N, H_index, n, Hm.d.data(), Hm.r, rm.d.data(), sigma2, dx_out);
}

// UpdaterHelper::measurement_compress_inplace on [H | res]: returns R (n+1 x n+1) of the Givens
// sweep applied to the augmented matrix (the reference applies it to H and res jointly).
int orc_compress(const double *A, int m, int n, double *R_out) {
  Mat H(m, n + 1);
  std::memcpy(H.d.data(), A, sizeof(double) * m * (n + 1));
  Givens G;
  int nc = n + 1;
  for (int c = 0; c < nc; c++) {
    for (int row = m - 1; row > c; row--) {
      G.make(H(row - 1, c), H(row, c));
      for (int j = c; j < nc; j++) G.apply(H(row - 1, j), H(row, j));
    }
  }
  for (int i = 0; i < nc; i++)
    for (int j = 0; j < nc; j++) R_out[i * nc + j] = (i < m && j >= i) ? H(i, j) : 0.0;
  return 0;
}

double orc_chi2_quantile95(int dof) { return chi2_quantile95(dof); }

// threads of the restated OpenCV calls (num_opencv_threads; 1 = serial)
int orc_set_threads(int n) {
  set_cv_threads(n);
  return cv_threads();
}

// per-feature results of every updater call of the last frame (include/uvio_hp.h uvio_hp_debug_frame_feats)
int orc_debug_frame_feats(orc_handle *h, int *kind, uint64_t *ids, double *pG, int *status, double *chi2, int cap,
                          int *n) {
  int k = 0;
  for (const auto &kd : h->m.fdbg.feats) {
    if (k < cap) {
      kind[k] = kd.first;
      ids[k] = kd.second.id;
      for (int j = 0; j < 3; j++) pG[3 * k + j] = kd.second.p_FinG[j];
      status[k] = kd.second.status;
      chi2[k] = kd.second.chi2;
    }
    k++;
  }
  *n = k;
  return 0;
}

// lock-step steering (updater.h FrameDebug): the device's per-feature results of the frame the oracle
// processes next; on = 0 turns steering off
int orc_set_steer(orc_handle *h, int on, int n, const int *kind, const uint64_t *ids, const double *pG,
                  const int *status, const double *chi2) {
  auto &d = h->m.fdbg;
  d.steer = on != 0;
  d.targets.clear();
  for (int i = 0; i < n; i++)
    d.targets[{kind[i], (size_t)ids[i]}] = SteerTarget{status[i], {pG[3 * i], pG[3 * i + 1], pG[3 * i + 2]}, chi2[i]};
  return 0;
}

// the steering log since creation: per event kind, feature id, stage, cast index, margin, disagreement
// before / after, found, candidates tried
int orc_get_steer_log(orc_handle *h, int *kind, uint64_t *ids, int *stage, int64_t *index, double *margin,
                      double *before, double *after, int *found, int *cands, int cap, int *n) {
  int k = 0;
  for (const auto &e : h->m.fdbg.log) {
    if (k < cap) {
      kind[k] = e.kind;
      ids[k] = e.featid;
      stage[k] = e.stage;
      index[k] = e.index;
      margin[k] = e.margin;
      before[k] = e.before;
      after[k] = e.after;
      found[k] = e.found;
      cands[k] = e.candidates;
    }
    k++;
  }
  *n = k;
  return 0;
}

// per-feature results of the last MSCKF update (debug / parity tests)
int orc_debug_last_msckf(orc_handle *h, uint64_t *ids, double *pG, int *status, double *chi2, int cap, int *n) {
  const auto &v = h->m.last_msckf.feats;
  int k = 0;
  for (const auto &d : v) {
    if (k < cap) {
      ids[k] = d.id;
      for (int j = 0; j < 3; j++) pG[3 * k + j] = d.p_FinG[j];
      status[k] = d.status;
      chi2[k] = d.chi2;
    }
    k++;
  }
  *n = k;
  return 0;
}

// TrackKLT state after the last camera feed (parity tests)
int orc_get_tracks(orc_handle *h, int cam, uint64_t *ids, float *uv, int cap, int *n) {
  auto &tr = h->m.tracker;
  auto it = tr.pts_last.find((size_t)cam);
  *n = 0;
  if (it == tr.pts_last.end()) return 0;
  const auto &pts = it->second;
  const auto &id = tr.ids_last[(size_t)cam];
  *n = (int)pts.size();
  if ((int)pts.size() > cap) return UVIO_HP_E_CAPACITY;
  for (size_t i = 0; i < pts.size(); i++) {
    if (ids) ids[i] = (uint64_t)id[i];
    if (uv) {
      uv[2 * i] = pts[i].x;
      uv[2 * i + 1] = pts[i].y;
    }
  }
  return 0;
}
int orc_get_pyramid(orc_handle *h, int cam, int level, int *w, int *hgt, uint8_t *img, int16_t *der, size_t cap) {
  auto &tr = h->m.tracker;
  auto it = tr.pyr_last.find((size_t)cam);
  if (it == tr.pyr_last.end() || level < 0 || level >= it->second.levels()) return UVIO_HP_E_STATE;
  const GrayImg &g = it->second.img[level];
  *w = g.w;
  *hgt = g.h;
  size_t px = (size_t)g.w * g.h;
  if (!img && !der) return 0;
  if (px > cap) return UVIO_HP_E_CAPACITY;
  if (img) std::memcpy(img, g.d.data(), px);
  if (der) std::memcpy(der, it->second.deriv[level].data(), px * 2 * sizeof(int16_t));
  return 0;
}

// ---- the tracker's OpenCV restatements one by one (tests/test_oracle_tracker.py pins them with
// property tests: SURVEY.md Appendix A; no OpenCV exists in this image) ----
static GrayImg gray(const uint8_t *src, int w, int h) {
  GrayImg g;
  g.w = w;
  g.h = h;
  g.d.assign(src, src + (size_t)w * h);
  return g;
}
int orc_equalize_hist(const uint8_t *src, int w, int h, uint8_t *dst) {
  GrayImg o = equalize_hist(gray(src, w, h));
  std::memcpy(dst, o.d.data(), o.d.size());
  return 0;
}
// dst: ((w+1)/2) x ((h+1)/2)
int orc_pyr_down(const uint8_t *src, int w, int h, uint8_t *dst) {
  GrayImg o = pyr_down(gray(src, w, h));
  std::memcpy(dst, o.d.data(), o.d.size());
  return 0;
}
// der: w x h x 2 (dx, dy)
int orc_scharr(const uint8_t *src, int w, int h, int16_t *der) {
  std::vector<int16_t> d = scharr_deriv(gray(src, w, h));
  std::memcpy(der, d.data(), d.size() * sizeof(int16_t));
  return 0;
}
// number of levels buildOpticalFlowPyramid keeps (level 0 included)
int orc_pyramid_levels(int w, int h, int win, int max_level) {
  std::vector<uint8_t> z((size_t)w * h, 0);
  return build_pyramid(gray(z.data(), w, h), win, max_level).levels();
}
// FAST on the ROI (x0, y0, rw, rh): out (x, y, response) in ROI coordinates, raster order
int orc_fast(const uint8_t *src, int w, int h, int x0, int y0, int rw, int rh, int thr, float *out, int cap, int *n) {
  std::vector<KeyPt> kp = fast_roi(gray(src, w, h), x0, y0, rw, rh, thr);
  *n = (int)kp.size();
  for (int i = 0; i < (int)kp.size() && i < cap; i++) {
    out[3 * i] = kp[i].x;
    out[3 * i + 1] = kp[i].y;
    out[3 * i + 2] = kp[i].response;
  }
  return (int)kp.size() <= cap ? 0 : UVIO_HP_E_CAPACITY;
}
// Grider_GRID.h:128 on one cell: n responses in cv::FAST's raster order -> order[i] = the raster index of the
// i-th keypoint after std::sort(compare_response) (mode 0, the reference), std::stable_sort (mode 1, the tie
// order rounds 1-5 used) or std::partial_sort(first, last, last) (mode 2, introsort's depth-limit heap path).
int orc_grid_order(const float *resp, int n, int mode, int *order) {
  std::vector<KeyPt> kp(n);
  for (int i = 0; i < n; i++) kp[i] = KeyPt{(float)i, 0.f, resp[i]};
  auto cmp = [](const KeyPt &a, const KeyPt &b) { return a.response > b.response; };
  if (mode == 0)
    grid_sort(kp);
  else if (mode == 1)
    std::stable_sort(kp.begin(), kp.end(), cmp);
  else if (mode == 2)
    std::partial_sort(kp.begin(), kp.end(), kp.end(), cmp);
  else
    return UVIO_HP_E_ARG;
  for (int i = 0; i < n; i++) order[i] = (int)kp[i].x;
  return 0;
}
// cornerSubPix in place on n points (x, y)
int orc_corner_subpix(const uint8_t *src, int w, int h, float *pts, int n, int win, int max_iters, double eps) {
  std::vector<KeyPt> kp(n);
  for (int i = 0; i < n; i++) kp[i] = KeyPt{pts[2 * i], pts[2 * i + 1], 0.f};
  corner_subpix(gray(src, w, h), kp, win, max_iters, eps);
  for (int i = 0; i < n; i++) pts[2 * i] = kp[i].x, pts[2 * i + 1] = kp[i].y;
  return 0;
}
// calcOpticalFlowPyrLK between two images (pyramids built here); p1 holds the initial guess on entry
int orc_lk(const uint8_t *prev, const uint8_t *next, int w, int h, int win, int max_level, int max_iters, float eps,
           const float *p0, float *p1, uint8_t *status, int n) {
  Pyramid a = build_pyramid(gray(prev, w, h), win, max_level), b = build_pyramid(gray(next, w, h), win, max_level);
  std::vector<KeyPt> k0(n), k1(n);
  for (int i = 0; i < n; i++) {
    k0[i] = KeyPt{p0[2 * i], p0[2 * i + 1], 0.f};
    k1[i] = KeyPt{p1[2 * i], p1[2 * i + 1], 0.f};
  }
  std::vector<uint8_t> st;
  lk_track(a, b, k0, k1, st, win, max_level, max_iters, eps);
  for (int i = 0; i < n; i++) {
    p1[2 * i] = k1[i].x;
    p1[2 * i + 1] = k1[i].y;
    status[i] = st[i];
  }
  return 0;
}
// findFundamentalMat(FM_RANSAC, thr, conf) inlier mask on n correspondences
int orc_ransac_mask(const float *x0, const float *y0, const float *x1, const float *y1, int n, double thr, double conf,
                    int max_iters, uint8_t *mask) {
  std::vector<uint8_t> m;
  ransac_fundamental_mask(std::vector<float>(x0, x0 + n), std::vector<float>(y0, y0 + n), std::vector<float>(x1, x1 + n),
                          std::vector<float>(y1, y1 + n), thr, conf, max_iters, m);
  std::memcpy(mask, m.data(), (size_t)n);
  return 0;
}
// 7-point fundamental matrices (<= 3, row-major 3x3 each); returns their count
int orc_fundamental_7pt(const double *x0, const double *y0, const double *x1, const double *y1, double *F) {
  return fundamental_7pt(x0, y0, x1, y1, F);
}

// Camera model entry points for fixture / finite-difference tests
int orc_camera_distort(const uvio_hp_camera_t *c, int n, const double *xy, double *uv, double *dz_dzn, double *dz_dzeta) {
  Camera cam;
  cam.model = c->model;
  cam.w = c->width;
  cam.h = c->height;
  for (int k = 0; k < 8; k++) cam.v[k] = c->intrinsics[k];
  for (int i = 0; i < n; i++) {
    double u, v;
    cam.distort_d(xy[2 * i], xy[2 * i + 1], u, v);
    uv[2 * i] = u;
    uv[2 * i + 1] = v;
    Mat a, b;
    cam.distort_jacobian(xy[2 * i], xy[2 * i + 1], a, b);
    if (dz_dzn) std::memcpy(dz_dzn + 4 * i, a.d.data(), 4 * sizeof(double));
    if (dz_dzeta) std::memcpy(dz_dzeta + 16 * i, b.d.data(), 16 * sizeof(double));
  }
  return 0;
}
int orc_camera_undistort(const uvio_hp_camera_t *c, int n, const float *uv, float *xy) {
  Camera cam;
  cam.model = c->model;
  for (int k = 0; k < 8; k++) cam.v[k] = c->intrinsics[k];
  for (int i = 0; i < n; i++) cam.undistort_f(uv[2 * i], uv[2 * i + 1], xy[2 * i], xy[2 * i + 1]);
  return 0;
}

}  // extern "C"
