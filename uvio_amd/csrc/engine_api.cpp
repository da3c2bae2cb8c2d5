// Updater-level entry points of the C ABI (include/uvio_hp.h "Updater-level boundary"):
// single updater calls on the engine's current state with caller-provided features, mirroring
// UpdaterMSCKF::update (UpdaterMSCKF.h:68), UpdaterSLAM::update / delayed_init / change_anchors
// (UpdaterSLAM.h:70-87), UpdaterUWB::update_single (UpdaterUWB.h:55), Propagator::propagate_and_clone
// (Propagator.h:110) and StateHelper::marginalize_* (StateHelper.h:224-230).  The same device paths run as
// inside the VioManager frame; only the feature bookkeeping comes from the caller.
#include <unordered_map>

#include "engine.h"

namespace uvhp {

// ov_core::Feature records from the flat arrays: a camera's track is created at its first measurement
// (Feature::track inserts at the front, the map order of the reference's per-camera unordered_maps)
static std::vector<FeatP> make_features(int nfeat, const uint64_t *ids, const int *off, const uvio_hp_feat_meas_t *m,
                                        int ncam) {
  std::vector<FeatP> fv;
  fv.reserve(nfeat);
  for (int i = 0; i < nfeat; i++) {
    if (off[i + 1] < off[i]) throw HpError(UVIO_HP_E_ARG, "meas_off must be non-decreasing");
    auto f = std::make_shared<Feature>();
    f->featid = (size_t)ids[i];
    for (int k = off[i]; k < off[i + 1]; k++) {
      if (m[k].cam < 0 || m[k].cam >= ncam) throw HpError(UVIO_HP_E_ARG, "measurement camera id out of range");
      f->track((size_t)m[k].cam).m.push_back(FeatMeas{m[k].u, m[k].v, m[k].un, m[k].vn, m[k].t});
    }
    fv.push_back(f);
  }
  return fv;
}

int Engine::api_set_state(const double *val, const double *fej, int len, const double *P, int N, int ld) {
  stage_ = "set_state";
  int k = 0;
  for (auto &v : vars_) k += v->vlen;
  if (k != len || N != N_ || ld < N) throw HpError(UVIO_HP_E_ARG, "state snapshot does not match the state layout");
  k = 0;
  for (auto &v : vars_)
    for (int i = 0; i < v->vlen; i++, k++) {
      v->val[i] = val[k];
      v->fej[i] = fej[k];
    }
  if (o_.do_calib_camera_intrinsics)
    for (auto &c : calib_intr_)
      for (int i = 0; i < 8; i++) cams_[c.first].v[i] = c.second->val[i];
  HP_HIP(hipMemcpy2DAsync(d_.P, sizeof(double) * d_.ldp, P, sizeof(double) * ld, sizeof(double) * N, N,
                          hipMemcpyHostToDevice, d_.stream));
  ++p_epoch_;
  dev_sync();
  return 0;
}

int Engine::api_propagate_and_clone(double t) {
  if (!is_initialized_) throw HpError(UVIO_HP_E_STATE, "propagate_and_clone before initialization");
  if (timestamp_ > t) return UVIO_HP_E_ORDER;
  if (timestamp_ == t) return 0;
  return propagate_and_clone(t);
}

int Engine::api_update(int which, int nfeat, const uint64_t *featids, const int *meas_off,
                       const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out) {
  if (!is_initialized_) throw HpError(UVIO_HP_E_STATE, "updater call before initialization");
  if (nfeat < 0 || (nfeat > 0 && (!featids || !meas_off || !meas || !out))) return UVIO_HP_E_ARG;
  std::vector<FeatP> fv = make_features(nfeat, featids, meas_off, meas, o_.num_cameras);
  const std::vector<FeatP> in = fv;
  if (which == API_SLAM)
    for (auto &f : fv)
      if (slam_.find(f->featid) == slam_.end()) throw HpError(UVIO_HP_E_ARG, "UpdaterSLAM::update: feature is not a SLAM landmark");
  int rc = 0;
  last_upd_.clear();
  if (which == API_MSCKF)
    rc = msckf_update(fv);
  else if (which == API_SLAM)
    rc = slam_update(fv);
  else
    rc = slam_delayed_init(fv);
  if (rc) return rc;
  const std::vector<FeatDebug> &res = (which == API_MSCKF) ? last_msckf_ : last_upd_;
  std::unordered_map<size_t, const FeatDebug *> by_id;
  for (auto &d : res) by_id[d.id] = &d;
  for (int i = 0; i < nfeat; i++) {
    uvio_hp_feat_result_t &o = out[i];
    o.featid = in[i]->featid;
    o.to_delete = in[i]->to_delete ? 1 : 0;
    auto it = by_id.find(in[i]->featid);
    if (it == by_id.end()) {  // cleaned away before the batch (too few measurements in the clone window)
      o.status = 1;
      o.chi2 = 0.0;
      for (int k = 0; k < 3; k++) o.p_FinG[k] = 0.0;
    } else {
      o.status = it->second->status;
      o.chi2 = it->second->chi2;
      for (int k = 0; k < 3; k++) o.p_FinG[k] = it->second->p_FinG[k];
    }
  }
  return 0;
}

int Engine::api_change_anchors() {
  if (!is_initialized_) throw HpError(UVIO_HP_E_STATE, "change_anchors before initialization");
  return slam_change_anchors();
}

int Engine::api_marginalize_slam() {
  if (!is_initialized_) throw HpError(UVIO_HP_E_STATE, "marginalize_slam before initialization");
  marginalize_slam();
  return 0;
}

int Engine::api_marginalize_old_clone() {
  if (!is_initialized_) throw HpError(UVIO_HP_E_STATE, "marginalize_old_clone before initialization");
  marginalize_old_clone();
  return 0;
}

int Engine::api_uwb_update_single(uint64_t anchor_id, double range, int *applied) {
  if (!is_initialized_) throw HpError(UVIO_HP_E_STATE, "UWB update before initialization");
  const int a = uwb_update_single((size_t)anchor_id, range);
  if (applied) *applied = a;
  return 0;
}

}  // namespace uvhp
