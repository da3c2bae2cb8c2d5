// Engine: VioManager::retriangulate_active_tracks (VioManagerHelper.cpp:190-388) on the device, and the
// VioManager::get_active_tracks getter (VioManager.h:114) that reads its results back on demand.
//
// The reference runs it inside the timed "re-tri & marg" bucket (VioManager.cpp:555-558) for messages whose
// first camera is cam0.  It changes neither the state nor the feature database: its outputs are the current
// tracks' positions (active_tracks_posinG) and their depth in camera 0 (active_tracks_uvd), which stay in HBM
// until a caller asks for them; the per-track running triangulation systems (active_feat_linsys_*) persist in
// a featid-keyed hash table on the device (kernels_feat.hip, k_retri_*).
// Since nothing reads those outputs before get_active_tracks, the frame only takes its inputs at the
// reference's point (the clone and camera poses, the SLAM landmarks, the camera models, the observations) and
// retri_flush runs the undistortion, the uploads and the launches later, on the auxiliary stream: while the
// host waits for the next frame's update chain (engine_chain.cpp), at the next simulated feed (which refills
// the observations), at the next retriangulation if no chain ran, or when get_active_tracks asks.  The same
// inputs give the same results; the frame's critical path loses the undistortion and the launches.
#include <algorithm>
#include <cstring>

#include "engine.h"

namespace uvhp {

void Engine::retri_alloc(int nobs, int nslam) {
  const int ns = std::max(nslam, 1);
  int need = 1024;
  while (need < 2 * std::max(nobs, 1)) need *= 2;
  // buffers the auxiliary stream may still read are replaced only after it has drained
  if (nobs > rt_.obs_cap || need > rt_.cap || ns > rt_.slam_cap) HP_HIP(hipStreamSynchronize(d_.aux));
  if (nobs > rt_.obs_cap) {
    const int oc = std::max(nobs, 2 * rt_.obs_cap);
    if (rt_.d_obs) HP_HIP(hipFree(rt_.d_obs));
    if (rt_.h_obs) HP_HIP(hipHostFree(rt_.h_obs));
    if (rt_.scratch) HP_HIP(hipFree(rt_.scratch));
    HP_HIP(hipMalloc(&rt_.d_obs, sizeof(DRetriObs) * oc));
    HP_HIP(hipHostMalloc(&rt_.h_obs, sizeof(DRetriObs) * oc, hipHostMallocDefault));
    HP_HIP(hipMalloc(&rt_.scratch, sizeof(double) * 17 * oc));
    rt_.obs_cap = oc;
  }
  if (need > rt_.cap) {
    // grow the hash tables; last frame's systems move to the new capacity (re-inserted on the host: the
    // table only grows a few times per run)
    std::vector<unsigned long long> keys;
    std::vector<DRetriEntry> ent;
    if (rt_.cap > 0) {
      dev_sync();
      keys.resize(rt_.cap);
      ent.resize(rt_.cap);
      HP_HIP(hipMemcpy(keys.data(), rt_.keys[rt_.cur], sizeof(unsigned long long) * rt_.cap, hipMemcpyDeviceToHost));
      HP_HIP(hipMemcpy(ent.data(), rt_.ent[rt_.cur], sizeof(DRetriEntry) * rt_.cap, hipMemcpyDeviceToHost));
    }
    for (int g = 0; g < 2; g++) {
      if (rt_.keys[g]) HP_HIP(hipFree(rt_.keys[g]));
      if (rt_.ent[g]) HP_HIP(hipFree(rt_.ent[g]));
      HP_HIP(hipMalloc(&rt_.keys[g], sizeof(unsigned long long) * need));
      HP_HIP(hipMalloc(&rt_.ent[g], sizeof(DRetriEntry) * need));
      HP_HIP(hipMemset(rt_.keys[g], 0xFF, sizeof(unsigned long long) * need));
    }
    if (!keys.empty()) {
      std::vector<unsigned long long> nk(need, kRetriEmpty);
      std::vector<DRetriEntry> ne(need);
      for (size_t i = 0; i < keys.size(); i++) {
        if (keys[i] == kRetriEmpty) continue;
        unsigned long long k = keys[i];
        k ^= k >> 33;
        k *= 0xff51afd7ed558ccdull;
        k ^= k >> 33;
        unsigned h = (unsigned)(k & (unsigned long long)(need - 1));
        while (nk[h] != kRetriEmpty) h = (h + 1) & (need - 1);
        nk[h] = keys[i];
        ne[h] = ent[i];
      }
      HP_HIP(hipMemcpy(rt_.keys[rt_.cur], nk.data(), sizeof(unsigned long long) * need, hipMemcpyHostToDevice));
      HP_HIP(hipMemcpy(rt_.ent[rt_.cur], ne.data(), sizeof(DRetriEntry) * need, hipMemcpyHostToDevice));
    }
    rt_.cap = need;
  }
  if (ns > rt_.slam_cap) {
    if (rt_.d_slam) HP_HIP(hipFree(rt_.d_slam));
    if (rt_.h_slam) HP_HIP(hipHostFree(rt_.h_slam));
    HP_HIP(hipMalloc(&rt_.d_slam, sizeof(DRetriSlam) * 2 * ns));
    HP_HIP(hipHostMalloc(&rt_.h_slam, sizeof(DRetriSlam) * 2 * ns, hipHostMallocDefault));
    rt_.slam_cap = 2 * ns;
  }
}

// the frame's observations in the reference's loop order (cameras in message order, each camera's tracks
// in get_last_obs order); SLAM landmarks' positions in the global frame (VioManagerHelper.cpp:302-318)
void Engine::retriangulate_active_tracks(double t, const std::vector<int> &camids) {
  stage_ = "VioManager::retriangulate_active_tracks";
  if (camids.empty() || camids[0] != 0) return;
  auto cit = clones_.find(t);
  if (cit == clones_.end()) throw HpError(UVIO_HP_E_STATE, "retriangulate_active_tracks: no clone at the frame time");
  retri_flush();  // not reached with a job pending: every feed flushes first (the simulated feed before refilling frame_obs_)
  // observations: the simulated feed keeps its own (frame_obs_); the KLT tracker's last tracks otherwise
  if (tracker_) {
    frame_obs_.clear();
    std::vector<KeyPt> pts;
    std::vector<size_t> ids;
    for (int cam : camids) {
      tracker_->last_tracks(cam, pts, ids);
      for (size_t i = 0; i < pts.size(); i++) {
        DRetriObs o{};
        o.featid = ids[i];
        o.u = pts[i].x;
        o.v = pts[i].y;
        o.cam = cam;
        frame_obs_.push_back(o);
      }
    }
  }
  RetriJob &job = rt_.pend_job;
  job = RetriJob{};
  // current clone, per-camera poses (R_GtoCi = R_ItoC R_GtoI, p_CiinG = p_IinG - R_GtoCi^T p_IinC)
  const VarP &clone = cit->second;
  double R_GtoI[9];
  quat_2_Rot(clone->val, R_GtoI);
  for (int c = 0; c < o_.num_cameras; c++) {
    double R_ItoC[9], t3[3];
    quat_2_Rot(calib_pose_.at(c)->val, R_ItoC);
    m3_mul(R_ItoC, R_GtoI, job.R_GtoC[c]);
    m3t_vec(job.R_GtoC[c], calib_pose_.at(c)->val + 4, t3);
    for (int k = 0; k < 3; k++) job.p_CinG[c][k] = clone->val[4 + k] - t3[k];
  }
  quat_2_Rot(calib_pose_.at(0)->val, job.R_ItoC0);
  for (int k = 0; k < 3; k++) job.p_IinC0[k] = calib_pose_.at(0)->val[4 + k], job.p_IinG[k] = clone->val[4 + k];
  std::memcpy(job.R_GtoI, R_GtoI, sizeof(R_GtoI));
  job.w0 = cams_[0].w;
  job.h0 = cams_[0].h;
  job.max_cond = o_.fi_max_cond_number;
  job.min_dist = o_.fi_min_dist;
  job.max_dist = o_.fi_max_dist;
  // SLAM landmarks (the state estimate takes priority over the triangulation)
  std::vector<DRetriSlam> &sl = rt_.pend_sl;
  sl.clear();
  for (auto &kv : slam_) {
    const VarP &lm = kv.second;
    DRetriSlam d{};
    d.featid = lm->featid;
    double p[3];
    lm->xyz(false, p);
    if (lm->rep == 2 || lm->rep == 3 || lm->rep == 4 || lm->rep == 5) {
      double Ric[9], Rgi[9], d0[3], t1[3], t2[3];
      quat_2_Rot(calib_pose_.at(lm->anchor_cam)->val, Ric);
      const VarP &anc = clones_.at(lm->anchor_time);
      quat_2_Rot(anc->val, Rgi);
      for (int k = 0; k < 3; k++) d0[k] = p[k] - calib_pose_.at(lm->anchor_cam)->val[4 + k];
      m3t_vec(Ric, d0, t1);
      m3t_vec(Rgi, t1, t2);
      for (int k = 0; k < 3; k++) p[k] = t2[k] + anc->val[4 + k];
    }
    for (int k = 0; k < 3; k++) d.pos[k] = p[k];
    sl.push_back(d);
  }
  // undistort_cv with the camera models as of now for the tracker's points, and for the simulated feed's when
  // this frame's updates may have moved the intrinsics since the feed undistorted the same pixels
  // (StateHelper.cpp:190-195)
  rt_.pend_undist = tracker_ || o_.do_calib_camera_intrinsics;
  if (rt_.pend_undist)
    for (int c = 0; c < o_.num_cameras; c++) rt_.pend_cams[c] = cams_[c];
  rt_.pend_t = t;
  rt_.pend = true;
}

// the pending job: the undistortion (on the pool, straight into the pinned upload buffer), the uploads and the
// launches (k_retri_*); the results replace the previous frame's
void Engine::retri_flush() {
  if (!rt_.pend) return;
  rt_.pend = false;
  const int nobs = (int)frame_obs_.size();
  {
    HPROF("retri.wait_copy");
    if (rt_.copy_pending) HP_HIP(hipEventSynchronize(rt_.copied));  // the previous uploads read h_obs / h_slam
    rt_.copy_pending = false;
  }
  RetriJob &job = rt_.pend_job;
  const std::vector<DRetriSlam> &sl = rt_.pend_sl;
  retri_alloc(nobs, (int)sl.size());
  {
    HPROF("retri.undist");
    DRetriObs *h = rt_.h_obs;
    const bool undist = rt_.pend_undist;
    const CamParams *cams = rt_.pend_cams;
    pool_.parallel_for(frame_obs_.size(), undist ? 512 : 8192, [&](size_t b, size_t e) {
      if (!undist) {
        std::memcpy(h + b, frame_obs_.data() + b, sizeof(DRetriObs) * (e - b));
        return;
      }
      for (size_t k = b; k < e; k++) {
        DRetriObs o = frame_obs_[k];
        cam_undistort_f(cams[o.cam], o.u, o.v, o.un, o.vn);
        h[k] = o;
      }
    });
  }
  job.nobs = nobs;
  job.cap = rt_.cap;
  job.obs = rt_.d_obs;
  job.scratch = rt_.scratch;
  job.keys_old = rt_.keys[rt_.cur];
  job.ent_old = rt_.ent[rt_.cur];
  job.keys_new = rt_.keys[1 - rt_.cur];
  job.ent_new = rt_.ent[1 - rt_.cur];
  job.nslam = (int)sl.size();
  job.slam = rt_.d_slam;
  // both uploads from pinned buffers that only this job writes (the last one's copies have run: copied)
  if (!sl.empty()) std::memcpy(rt_.h_slam, sl.data(), sizeof(DRetriSlam) * sl.size());
  if (nobs) HP_HIP(hipMemcpyAsync(rt_.d_obs, rt_.h_obs, sizeof(DRetriObs) * nobs, hipMemcpyHostToDevice, d_.aux));
  if (!sl.empty())
    HP_HIP(hipMemcpyAsync(rt_.d_slam, rt_.h_slam, sizeof(DRetriSlam) * sl.size(), hipMemcpyHostToDevice, d_.aux));
  if (nobs || !sl.empty()) {
    HP_HIP(hipEventRecord(rt_.copied, d_.aux));
    rt_.copy_pending = true;
  }
  launch_retriangulate(d_.aux, job);
  rt_.cur = 1 - rt_.cur;
  rt_.nslam = job.nslam;
  rt_.time = rt_.pend_t;
  rt_.valid = true;
}

// VioManager::get_active_tracks (VioManager.h:114)
int Engine::get_active_tracks(double *t, uint64_t *ids, double *posinG, double *uvd, int *uvd_valid, int cap) {
  retri_flush();
  *t = rt_.valid ? rt_.time : -1;
  if (!rt_.valid) return 0;
  dev_sync();
  HP_HIP(hipStreamSynchronize(d_.aux));
  std::vector<unsigned long long> keys(rt_.cap);
  std::vector<DRetriEntry> ent(rt_.cap);
  std::vector<DRetriSlam> sl(rt_.nslam);
  HP_HIP(hipMemcpy(keys.data(), rt_.keys[rt_.cur], sizeof(unsigned long long) * rt_.cap, hipMemcpyDeviceToHost));
  HP_HIP(hipMemcpy(ent.data(), rt_.ent[rt_.cur], sizeof(DRetriEntry) * rt_.cap, hipMemcpyDeviceToHost));
  if (rt_.nslam) HP_HIP(hipMemcpy(sl.data(), rt_.d_slam, sizeof(DRetriSlam) * rt_.nslam, hipMemcpyDeviceToHost));
  int n = 0;
  auto put = [&](unsigned long long id, const double *p, const double *d, int ok) {
    if (n < cap) {
      ids[n] = id;
      for (int k = 0; k < 3; k++) posinG[3 * n + k] = p[k], uvd[3 * n + k] = ok ? d[k] : 0.0;
      uvd_valid[n] = ok;
    }
    n++;
  };
  for (int i = 0; i < rt_.cap; i++)
    if (keys[i] != kRetriEmpty && ent[i].last_pass >= 0) put(keys[i], ent[i].pos, ent[i].uvd, ent[i].uvd_valid);
  for (auto &s : sl) put(s.featid, s.pos, s.uvd, s.uvd_valid);
  return n;
}

}  // namespace uvhp
