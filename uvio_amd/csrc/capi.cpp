// extern "C" boundary of libuvio_hp.so (declared in include/uvio_hp.h).  Every entry converts
// exceptions into status codes: the library never exits the process.
#include <cstring>
#include <string>

#include "engine.h"

using namespace uvhp;

struct uvio_hp {
  Engine *e = nullptr;
  std::string err;
  // set by a fatal error of a state-changing call (the reference std::exit's on these: negative covariance
  // diagonal, StateHelper.cpp:112,181; a device or internal error likewise leaves the frame half applied, e.g.
  // measurements already trimmed from the feature database): every later state-changing call is refused
  std::string fatal;
};

// an exception that is not an HpError is a host-side logic error (e.g. std::out_of_range from a map
// lookup): reported as UVIO_HP_E_INTERNAL with the reference routine the engine was in
static std::string internal_error(const uvio_hp *h, const std::exception &ex) {
  std::string m = std::string("internal error: ") + ex.what();
  if (h && h->e && h->e->stage()[0]) m += std::string(" (in ") + h->e->stage() + ")";
  return m;
}

#define HP_GUARD(h, body)                                    \
  try {                                                      \
    if ((h) && (h)->e) HP_HIP(hipSetDevice((h)->e->device())); \
    body                                                     \
  } catch (const HpError &ex) {                              \
    if (h) (h)->err = ex.what();                             \
    return ex.code;                                          \
  } catch (const std::exception &ex) {                       \
    if (h) (h)->err = internal_error(h, ex);                 \
    return UVIO_HP_E_INTERNAL;                               \
  }

// a state-changing entry: refused after a fatal error; a fatal result stops the estimator
static bool is_fatal(int rc) { return rc == UVIO_HP_E_NUMERIC || rc == UVIO_HP_E_DEVICE || rc == UVIO_HP_E_INTERNAL; }
#define HP_FEED(h, call)                                                                         \
  if (!(h)->fatal.empty()) {                                                                     \
    (h)->err = "estimator stopped by an earlier fatal error (" + (h)->fatal + ")";             \
    return UVIO_HP_E_STATE;                                                                      \
  }                                                                                              \
  {                                                                                              \
    const int rc_ = [&]() -> int { HP_GUARD(h, return (call);) }();                              \
    if (is_fatal(rc_)) (h)->fatal = (h)->err;                                                    \
    return rc_;                                                                                  \
  }

extern "C" {

int uvio_hp_options_default(uvio_hp_options_t *opts) {
  if (!opts) return UVIO_HP_E_ARG;
  options_default(opts);
  return 0;
}

int uvio_hp_options_load(const char *path, uvio_hp_options_t *opts) {
  if (!path || !opts) return UVIO_HP_E_ARG;
  std::string err;
  return options_load(path, opts, &err);
}

static thread_local std::string g_create_err = "";  // why the last uvio_hp_create on this thread failed

int uvio_hp_create(const uvio_hp_options_t *opts, int device, uvio_hp_t **out) {
  if (!opts || !out) return UVIO_HP_E_ARG;
  *out = nullptr;
  uvio_hp_t *h = new uvio_hp_t();
  try {
    h->e = new Engine(*opts, device);
  } catch (const HpError &ex) {
    int c = ex.code;
    g_create_err = ex.what();
    delete h;
    return c;
  } catch (const std::exception &ex) {
    g_create_err = ex.what();
    delete h;
    return UVIO_HP_E_DEVICE;
  }
  *out = h;
  return 0;
}

int uvio_hp_destroy(uvio_hp_t *h) {
  if (!h) return UVIO_HP_E_ARG;
  delete h->e;
  delete h;
  return 0;
}

const char *uvio_hp_last_error(const uvio_hp_t *h) { return h ? h->err.c_str() : g_create_err.c_str(); }

int uvio_hp_initialize_with_gt(uvio_hp_t *h, const double x[17]) {
  if (!h || !x) return UVIO_HP_E_ARG;
  HP_GUARD(h, h->e->initialize_with_gt(x); return 0;)
}

int uvio_hp_feed_imu(uvio_hp_t *h, double t, const double wm[3], const double am[3]) {
  if (!h || !wm || !am) return UVIO_HP_E_ARG;
  HP_GUARD(h, h->e->feed_imu(t, wm, am); return 0;)
}

int uvio_hp_feed_imu_batch(uvio_hp_t *h, int n, const double *t, const double *wm, const double *am) {
  if (!h || n < 0 || (n > 0 && (!t || !wm || !am))) return UVIO_HP_E_ARG;
  HP_GUARD(h, for (int i = 0; i < n; i++) h->e->feed_imu(t[i], wm + 3 * i, am + 3 * i); return 0;)
}

int uvio_hp_feed_simulation(uvio_hp_t *h, double t, int ncam, const int *cam_ids, const int *counts, const uint64_t *ids,
                            const float *uv) {
  if (!h || ncam <= 0 || !cam_ids || !counts) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->feed_simulation(t, ncam, cam_ids, counts, ids, uv))
}

int uvio_hp_feed_camera(uvio_hp_t *h, double t, int ncam, const int *cam_ids, const uint8_t *const *imgs,
                        const int *strides, const uint8_t *const *masks) {
  if (!h || ncam <= 0 || !cam_ids || !imgs || !strides) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->feed_camera(t, ncam, cam_ids, imgs, strides, masks, false))
}

int uvio_hp_feed_camera_device(uvio_hp_t *h, double t, int ncam, const int *cam_ids, const uint8_t *const *imgs,
                               const int *strides, const uint8_t *const *masks) {
  if (!h || ncam <= 0 || !cam_ids || !imgs || !strides) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->feed_camera(t, ncam, cam_ids, imgs, strides, masks, true))
}

int uvio_hp_get_tracks(uvio_hp_t *h, int cam, uint64_t *ids, float *uv, int cap, int *n) {
  if (!h || !n) return UVIO_HP_E_ARG;
  HP_GUARD(h, {
    std::vector<uvhp::KeyPt> pts;
    std::vector<size_t> id;
    if (h->e->tracker()) h->e->tracker()->last_tracks(cam, pts, id);
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
  })
}

int uvio_hp_get_pyramid(uvio_hp_t *h, int cam, int level, int *w, int *hgt, uint8_t *img, int16_t *der, size_t cap) {
  if (!h || !w || !hgt) return UVIO_HP_E_ARG;
  HP_GUARD(h, {
    std::vector<uint8_t> im;
    std::vector<int16_t> d;
    if (!h->e->tracker() || !h->e->tracker()->last_pyramid(cam, level, w, hgt, img ? &im : nullptr, der ? &d : nullptr))
      return UVIO_HP_E_STATE;
    size_t px = (size_t)*w * *hgt;
    if ((img || der) && px > cap) return UVIO_HP_E_CAPACITY;
    if (img) std::memcpy(img, im.data(), px);
    if (der) std::memcpy(der, d.data(), px * 2 * sizeof(int16_t));
    return 0;
  })
}

int uvio_hp_feed_uwb(uvio_hp_t *h, double t, int n, const uint64_t *ids, const double *ranges) {
  if (!h || n < 0) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->feed_uwb(t, n, ids, ranges))
}

int uvio_hp_init_anchors(uvio_hp_t *h, int n, const uvio_hp_anchor_t *a) {
  if (!h || n < 0) return UVIO_HP_E_ARG;
  HP_GUARD(h, return h->e->init_anchors(n, a);)
}

int uvio_hp_initialized(const uvio_hp_t *h, int *out) {
  if (!h || !out) return UVIO_HP_E_ARG;
  *out = h->e->initialized() ? 1 : 0;
  return 0;
}

int uvio_hp_get_imu_state(uvio_hp_t *h, double *t, double out[16]) {
  if (!h || !t || !out) return UVIO_HP_E_ARG;
  *t = h->e->timestamp();
  std::memcpy(out, h->e->imu().val, sizeof(double) * 16);
  return 0;
}

int uvio_hp_get_cov_dim(uvio_hp_t *h, int *n) {
  if (!h || !n) return UVIO_HP_E_ARG;
  *n = h->e->cov_dim();
  return 0;
}

int uvio_hp_get_cov(uvio_hp_t *h, double *out, int ld) {
  if (!h || !out || ld < h->e->cov_dim()) return UVIO_HP_E_ARG;
  HP_GUARD(h, h->e->get_cov(out, ld); return 0;)
}

int uvio_hp_get_state_vector(uvio_hp_t *h, double *out, int cap, int *len, int *meta, int meta_cap, int *nvars) {
  if (!h || !out || !len) return UVIO_HP_E_ARG;
  int k = h->e->state_vector(out, cap, meta, meta_cap, nvars);
  *len = k;
  return k <= cap ? 0 : UVIO_HP_E_CAPACITY;
}

int uvio_hp_get_fej_vector(uvio_hp_t *h, double *out, int cap, int *len) {
  if (!h || !out || !len) return UVIO_HP_E_ARG;
  int k = h->e->state_vector(out, cap, nullptr, 0, nullptr, true);
  *len = k;
  return k <= cap ? 0 : UVIO_HP_E_CAPACITY;
}

int uvio_hp_get_timing(uvio_hp_t *h, uvio_hp_timing_t *out) {
  if (!h || !out) return UVIO_HP_E_ARG;
  *out = h->e->timing();
  return 0;
}

int uvio_hp_get_active_tracks(uvio_hp_t *h, double *t, uint64_t *ids, double *posinG, double *uvd, int *uvd_valid,
                              int cap, int *n) {
  if (!h || !t || !n || (cap > 0 && (!ids || !posinG || !uvd || !uvd_valid))) return UVIO_HP_E_ARG;
  HP_GUARD(h, {
    *n = h->e->get_active_tracks(t, ids, posinG, uvd, uvd_valid, cap);
    return *n <= cap ? 0 : UVIO_HP_E_CAPACITY;
  })
}

int uvio_hp_set_kernel_timing(uvio_hp_t *h, int on) {
  if (!h) return UVIO_HP_E_ARG;
  if (on < 0) return UVIO_HP_E_ARG;
  h->e->set_kernel_timing(on);
  return 0;
}

int uvio_hp_get_kernel_stats(uvio_hp_t *h, int flush, uvio_hp_kstat_t *out, int cap, int *n) {
  if (!h || !n || (cap > 0 && !out)) return UVIO_HP_E_ARG;
  HP_GUARD(h, h->e->kernel_stats(flush != 0, out, cap, n); return 0;)
}

int uvio_hp_get_clone_times(uvio_hp_t *h, double *out, int cap, int *n) {
  if (!h || !n) return UVIO_HP_E_ARG;
  auto t = h->e->clone_times();
  for (int i = 0; i < (int)t.size() && i < cap; i++) out[i] = t[i];
  *n = (int)t.size();
  return 0;
}

// ---- Updater-level boundary (include/uvio_hp.h) ----
int uvio_hp_set_state(uvio_hp_t *h, const double *val, const double *fej, int len, const double *P, int N, int ld) {
  if (!h || !val || !fej || !P || len <= 0 || N <= 0) return UVIO_HP_E_ARG;
  HP_GUARD(h, { return h->e->api_set_state(val, fej, len, P, N, ld); })
}
int uvio_hp_propagate_and_clone(uvio_hp_t *h, double t) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_propagate_and_clone(t))
}
int uvio_hp_msckf_update(uvio_hp_t *h, int nfeat, const uint64_t *featids, const int *meas_off,
                         const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_update(Engine::API_MSCKF, nfeat, featids, meas_off, meas, out))
}
int uvio_hp_slam_update(uvio_hp_t *h, int nfeat, const uint64_t *featids, const int *meas_off,
                        const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_update(Engine::API_SLAM, nfeat, featids, meas_off, meas, out))
}
int uvio_hp_slam_delayed_init(uvio_hp_t *h, int nfeat, const uint64_t *featids, const int *meas_off,
                              const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_update(Engine::API_DELAYED, nfeat, featids, meas_off, meas, out))
}
int uvio_hp_slam_change_anchors(uvio_hp_t *h) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_change_anchors())
}
int uvio_hp_marginalize_slam(uvio_hp_t *h) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_marginalize_slam())
}
int uvio_hp_marginalize_old_clone(uvio_hp_t *h) {
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_marginalize_old_clone())
}
int uvio_hp_uwb_update_single(uvio_hp_t *h, double t, uint64_t anchor_id, double range, int *applied) {
  (void)t;  // the reference's Jacobian does not read the measurement time (UVioUpdaterHelper.cpp:147-241)
  if (!h) return UVIO_HP_E_ARG;
  HP_FEED(h, h->e->api_uwb_update_single(anchor_id, range, applied))
}

int uvio_hp_debug_last_msckf(uvio_hp_t *h, uint64_t *ids, double *pG, int *status, double *chi2, int cap, int *n) {
  if (!h || !n) return UVIO_HP_E_ARG;
  const auto &v = h->e->last_msckf_;
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

int uvio_hp_debug_frame_feats(uvio_hp_t *h, int *kind, uint64_t *ids, double *pG, int *status, double *chi2, int cap,
                              int *n) {
  if (!h || !n) return UVIO_HP_E_ARG;
  int k = 0;
  for (const auto &kd : h->e->frame_feats_) {
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

int uvio_hp_shard_unique_id(uint8_t id[128]) {
  if (!id) return UVIO_HP_E_ARG;
  std::string err;
  int rc = rccl_unique_id(id, &err);
  if (rc) g_create_err = err;
  return rc;
}

int uvio_hp_shard_init_rccl(uvio_hp_t *h, int rank, int world, const uint8_t id[128], int min_features) {
  if (!h || !id) return UVIO_HP_E_ARG;
  HP_GUARD(h, h->e->shard_init_rccl(rank, world, id, min_features); return 0;)
}

int uvio_hp_shard_init_host(uvio_hp_t *h, int rank, int world, uvio_hp_allreduce_fn fn, void *user,
                            int min_features) {
  if (!h || !fn) return UVIO_HP_E_ARG;
  HP_GUARD(h, h->e->shard_init_host(rank, world, fn, user, min_features); return 0;)
}

int uvio_hp_shard_partition(const int *rows, int n, int world, int *bounds) {
  if (!rows || !bounds || n < 0 || world < 1) return UVIO_HP_E_ARG;
  shard_partition(rows, n, world, bounds);
  return 0;
}

int uvio_hp_ekf_update(double *P, int N, const int *H_index, int n, const double *H, int r, const double *res,
                       double sigma2, double *dx_out) {
  try {
    return Engine::ekf_update_standalone(P, N, H_index, n, H, r, res, sigma2, dx_out);
  } catch (const HpError &ex) {
    return ex.code;
  } catch (...) {
    return UVIO_HP_E_DEVICE;
  }
}

int uvio_hp_msckf_compressed_update(double *P, int N, const int *H_index, int n, const double *H, int m,
                                    const double *res, double sigma2, double *dx_out) {
  try {
    return Engine::ekf_update_standalone(P, N, H_index, n, H, m, res, sigma2, dx_out, true);
  } catch (const HpError &ex) {
    return ex.code;
  } catch (...) {
    return UVIO_HP_E_DEVICE;
  }
}

int uvio_hp_compress(const double *A, int m, int n, double *R_out) {
  try {
    return Engine::compress_standalone(A, m, n, R_out);
  } catch (const HpError &ex) {
    return ex.code;
  } catch (...) {
    return UVIO_HP_E_DEVICE;
  }
}

int uvio_hp_undistort(int model, const double cam[8], int n, const float *uv, float *uvn, uint8_t *ambiguous) {
  try {
    return Engine::undistort_standalone(model, cam, n, uv, uvn, ambiguous);
  } catch (const HpError &ex) {
    return ex.code;
  } catch (...) {
    return UVIO_HP_E_DEVICE;
  }
}

int uvio_hp_debug_grid_order(const uint8_t *resp, const int *off, int ncell, int kmax, int depth, int *arrangement,
                             int *top) {
  try {
    return Engine::grid_order_standalone(resp, off, ncell, kmax, depth, arrangement, top);
  } catch (const HpError &ex) {
    return ex.code;
  } catch (...) {
    return UVIO_HP_E_DEVICE;
  }
}

int uvio_hp_debug_grid_stats(uvio_hp_t *h, uint64_t *cells, uint64_t *introsort_cells) {
  if (!h) return UVIO_HP_E_ARG;
  unsigned long long c = 0;
  unsigned long long i = 0;
  HP_GUARD(h, if (h->e->tracker()) h->e->tracker()->grid_stats(&c, &i);)
  if (cells) *cells = c;
  if (introsort_cells) *introsort_cells = i;
  return 0;
}

}  // extern "C"
