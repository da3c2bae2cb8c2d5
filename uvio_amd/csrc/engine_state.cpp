// Engine: state layout, device buffers and covariance operations.
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "engine.h"

namespace uvhp {

// ---- Type::update family ----
void Var::update(const double *dx) {
  if (kind == V_IMU || kind == V_POSE || kind == V_QUAT) {
    quat_boxplus(val, dx);
    for (int i = 3; i < size; i++) val[i + 1] += dx[i];
  } else {
    for (int i = 0; i < size; i++) val[i] += dx[i];
  }
}

// Landmark::get_xyz (Landmark.cpp:26-63); representation ids of LandmarkRepresentation.h:38
void Var::xyz(bool getfej, double *o) const {
  const double *p = getfej ? fej : val;
  switch (rep) {
    case 0:
    case 2:
      o[0] = p[0]; o[1] = p[1]; o[2] = p[2];
      break;
    case 1:
    case 3:
      o[0] = (1 / p[2]) * cos(p[0]) * sin(p[1]);
      o[1] = (1 / p[2]) * sin(p[0]) * sin(p[1]);
      o[2] = (1 / p[2]) * cos(p[1]);
      break;
    case 4:
      // reference quirk (Landmark.cpp:47-52): the fej value is ignored for this representation
      o[0] = (1 / val[2]) * val[0];
      o[1] = (1 / val[2]) * val[1];
      o[2] = 1 / val[2];
      break;
    default:
      o[0] = o[1] = o[2] = 0;
  }
}
void Var::set_xyz(const double *p, bool isfej) {
  double *d = isfej ? fej : val;
  switch (rep) {
    case 0:
    case 2:
      d[0] = p[0]; d[1] = p[1]; d[2] = p[2];
      break;
    case 1:
    case 3: {
      double g_rho = 1 / sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
      d[0] = atan2(p[1], p[0]);
      d[1] = acos(g_rho * p[2]);
      d[2] = g_rho;
      break;
    }
    case 4:
      d[0] = p[0] / p[2];
      d[1] = p[1] / p[2];
      d[2] = 1 / p[2];
      break;
    default:
      break;
  }
}

// ---- Feature (Feature.cpp:26-111) ----
void MeasList::keep_if_valid(const std::vector<double> &valid) {
  size_t w = b;
  for (size_t i = b; i < v.size(); i++)
    if (std::binary_search(valid.begin(), valid.end(), v[i].t)) v[w++] = v[i];
  v.resize(w);
  if (v.size() == b) clear();
  recache();
}
// Feature::clean_old_measurements (Feature.cpp:37-60): keep the measurements at the given (sorted) times
void Feature::clean_old_measurements(const std::vector<double> &valid) {
  for (auto &c : tracks) c.m.keep_if_valid(valid);
}
// Feature::clean_older_measurements (Feature.cpp:85-104): drop every measurement at or before t.  A camera's
// measurements of an in-order stream form a prefix, found by binary search (MeasList::drop_through).
void Feature::clean_older_measurements(double t) {
  for (auto &c : tracks) c.m.drop_through(t);
}

static VarP mk(VKind k, int size, int vlen) { return std::make_shared<Var>(k, size, vlen); }

// State::State (State.cpp:28-166) + UVioManager ctor (UVioManager.cpp:26-58)
Engine::Engine(const uvio_hp_options_t &o, int device) : o_(o), device_(device) {
  if (o_.num_cameras < 1 || o_.num_cameras > UVIO_HP_MAX_CAMS) throw HpError(UVIO_HP_E_ARG, "num_cameras out of range");
  g_track_reserve.store(std::max(8, o_.max_clone_size + 4), std::memory_order_relaxed);
  // configurations the reference accepts but this build does not implement fail here, loudly
  if (!o_.use_klt) throw HpError(UVIO_HP_E_CONFIG, "use_klt: false (TrackDescriptor / ORB) is not implemented");
  if (o_.use_aruco) throw HpError(UVIO_HP_E_CONFIG, "use_aruco: true (TrackAruco) is not implemented");
  if (o_.feat_rep_msckf != 0 && o_.feat_rep_msckf != 4)
    throw HpError(UVIO_HP_E_CONFIG, "feat_rep_msckf: only GLOBAL_3D / ANCHORED_MSCKF_INVERSE_DEPTH are implemented");
  if (o_.feat_rep_slam != 0 && o_.feat_rep_slam != 2 && o_.feat_rep_slam != 4)
    throw HpError(UVIO_HP_E_CONFIG, "feat_rep_slam: only GLOBAL_3D / ANCHORED_3D / ANCHORED_MSCKF_INVERSE_DEPTH are implemented");
  currid_ = 4 * (size_t)o_.max_aruco_features + 1;  // TrackBase::currid (TrackBase.cpp:34)
  int cur = 0;
  imu_ = mk(V_IMU, 15, 16);
  imu_->val[3] = imu_->fej[3] = 1;
  imu_->id = cur;
  vars_.push_back(imu_);
  cur += 15;
  dw_ = mk(V_VEC, 6, 6);
  da_ = mk(V_VEC, 6, 6);
  tg_ = mk(V_VEC, 9, 9);
  qg_ = mk(V_QUAT, 3, 4);
  qa_ = mk(V_QUAT, 3, 4);
  for (int k = 0; k < 6; k++) dw_->val[k] = dw_->fej[k] = o_.imu_dw[k], da_->val[k] = da_->fej[k] = o_.imu_da[k];
  for (int k = 0; k < 9; k++) tg_->val[k] = tg_->fej[k] = o_.imu_tg[k];
  for (int k = 0; k < 4; k++) qg_->val[k] = qg_->fej[k] = o_.q_GYROtoIMU[k], qa_->val[k] = qa_->fej[k] = o_.q_ACCtoIMU[k];
  if (o_.do_calib_imu_intrinsics) {
    for (auto &v : {dw_, da_}) {
      v->id = cur;
      vars_.push_back(v);
      cur += v->size;
    }
    if (o_.do_calib_imu_g_sensitivity) {
      tg_->id = cur;
      vars_.push_back(tg_);
      cur += 9;
    }
    VarP q = (o_.imu_model == 0) ? qg_ : qa_;
    q->id = cur;
    vars_.push_back(q);
    cur += 3;
  }
  calib_dt_ = mk(V_VEC, 1, 1);
  calib_dt_->val[0] = calib_dt_->fej[0] = o_.calib_camimu_dt;
  if (o_.do_calib_camera_timeoffset) {
    calib_dt_->id = cur;
    vars_.push_back(calib_dt_);
    cur += 1;
  }
  for (int i = 0; i < o_.num_cameras; i++) {
    VarP pose = mk(V_POSE, 6, 7), intr = mk(V_VEC, 8, 8);
    const uvio_hp_camera_t &c = o_.cams[i];
    for (int k = 0; k < 4; k++) pose->val[k] = pose->fej[k] = c.q_ItoC[k];
    for (int k = 0; k < 3; k++) pose->val[4 + k] = pose->fej[4 + k] = c.p_IinC[k];
    for (int k = 0; k < 8; k++) intr->val[k] = intr->fej[k] = c.intrinsics[k];
    calib_pose_.insert({(size_t)i, pose});
    calib_intr_.insert({(size_t)i, intr});
    cams_[i].model = c.model;
    cams_[i].w = c.width;
    cams_[i].h = c.height;
    for (int k = 0; k < 8; k++) cams_[i].v[k] = c.intrinsics[k];
    if (o_.do_calib_camera_pose) {
      pose->id = cur;
      vars_.push_back(pose);
      cur += 6;
    }
    if (o_.do_calib_camera_intrinsics) {
      intr->id = cur;
      vars_.push_back(intr);
      cur += 8;
    }
  }
  N_ = cur;
  chi2_table_ = std::vector<double>(1000, 0.0);
  alloc_device();
  // initial covariance (State.cpp:133-165): built once on the host, then resident on the device
  std::vector<double> Ph((size_t)N_ * N_, 0.0);
  for (int i = 0; i < N_; i++) Ph[(size_t)i * N_ + i] = 1e-6;
  auto setd = [&](int id, int n, double v) {
    for (int k = 0; k < n; k++) Ph[(size_t)(id + k) * N_ + id + k] = v;
  };
  if (o_.do_calib_imu_intrinsics) {
    setd(dw_->id, 6, 0.005 * 0.005);
    setd(da_->id, 6, 0.008 * 0.008);
    if (o_.do_calib_imu_g_sensitivity) setd(tg_->id, 9, 0.005 * 0.005);
    setd((o_.imu_model == 0 ? qg_ : qa_)->id, 3, 0.005 * 0.005);
  }
  if (o_.do_calib_camera_timeoffset) setd(calib_dt_->id, 1, 0.01 * 0.01);
  for (int i = 0; i < o_.num_cameras; i++) {
    if (o_.do_calib_camera_pose) {
      setd(calib_pose_.at(i)->id, 3, 0.005 * 0.005);
      setd(calib_pose_.at(i)->id + 3, 3, 0.015 * 0.015);
    }
    if (o_.do_calib_camera_intrinsics) {
      setd(calib_intr_.at(i)->id, 4, 1.0);
      setd(calib_intr_.at(i)->id + 4, 4, 0.005 * 0.005);
    }
  }
  upload_P_full(Ph, N_);
  if (o_.record_timing_information) {
    // VioManager.cpp:105-122: the old file is replaced, its directory created
    std::string path(o_.record_timing_filepath);
    std::remove(path.c_str());
    for (size_t k = 1; k < path.size(); k++)
      if (path[k] == '/') mkdir(path.substr(0, k).c_str(), 0755);
    timing_csv_ = std::fopen(path.c_str(), "a");
    if (!timing_csv_) throw HpError(UVIO_HP_E_CONFIG, "record_timing_filepath: cannot open " + path);
    std::fprintf(timing_csv_, "# timestamp (sec),tracking,propagation,msckf update,");
    if (o_.max_slam_features > 0) std::fprintf(timing_csv_, "slam update,slam delayed,");
    std::fprintf(timing_csv_, "re-tri & marg,total\n");
  }
  // uvio
  p_IinU_ = mk(V_VEC, 3, 3);
  for (int k = 0; k < 3; k++) p_IinU_->val[k] = p_IinU_->fej[k] = o_.p_IinU[k];
  if (o_.use_uwb) {
    if (o_.do_calib_uwb_extrinsics) {
      std::vector<double> HR(9, 0.0), HL(9, 0.0), R(9, 0.0), res(3, 0.0);
      for (int k = 0; k < 3; k++) HL[4 * k] = 1.0, R[4 * k] = o_.prior_uwb_imu_cov;
      initialize_invertible_host(p_IinU_, {{imu_->id, 3}}, HR, HL, R, res);
      for (int k = 0; k < 3; k++) p_IinU_->val[k] = p_IinU_->fej[k] = o_.p_IinU[k];
    }
    if (o_.n_anchors > 0) init_anchors(o_.n_anchors, o_.anchors);
  }
}

Engine::~Engine() {
  if (timing_csv_) std::fclose(timing_csv_);
  hipSetDevice(device_);
  if (shard_.nccl) rccl_comm_destroy(shard_.nccl);
  tracker_.reset();
  void *rptrs[] = {rt_.keys[0], rt_.keys[1], rt_.ent[0], rt_.ent[1], rt_.d_obs, rt_.d_slam, rt_.scratch};
  for (void *p : rptrs)
    if (p) hipFree(p);
  if (rt_.h_obs) hipHostFree(rt_.h_obs);
  if (rt_.h_slam) hipHostFree(rt_.h_slam);
  if (rt_.copied) hipEventDestroy(rt_.copied);
  void *ptrs[] = {d_.P, d_.P2, d_.T, d_.Phi, d_.Q, d_.dnc, d_.iold, d_.feats, d_.meas, d_.vars, d_.clones, d_.cams,
                  d_.chi2, d_.H, d_.Tall, d_.partials, d_.R, d_.hidx, d_.ekf.M, d_.ekf.W, d_.ekf.S, d_.ekf.y,
                  d_.ekf.Dinv, d_.stg_d, d_.acc, d_.shard, d_.hidx_pre, d_.chain, d_.frame, d_.chi2S, d_.uwb_reg,
                  d_.uwb_h};
  for (void *p : ptrs)
    if (p) hipFree(p);
  if (d_.pin) hipHostFree(d_.pin);
  if (d_.shard_host) hipHostFree(d_.shard_host);
  if (d_.stg_h) hipHostFree(d_.stg_h);
  if (d_.hidx_pre_h) hipHostFree(d_.hidx_pre_h);
  if (d_.chain_host) hipHostFree(d_.chain_host);
  if (d_.uwb_host) hipHostFree(d_.uwb_host);
  for (auto &e : d_.ev_pre)
    if (e) hipEventDestroy(e);
  if (d_.ev_aux_in) hipEventDestroy(d_.ev_aux_in);
  if (d_.ev_aux_out) hipEventDestroy(d_.ev_aux_out);
  if (d_.aux) hipStreamDestroy(d_.aux);
  if (d_.ev_copy) hipEventDestroy(d_.ev_copy);
  if (d_.copy) hipStreamDestroy(d_.copy);
  if (d_.ev0) hipEventDestroy(d_.ev0);
  if (d_.ev1) hipEventDestroy(d_.ev1);
  if (d_.stream) hipStreamDestroy(d_.stream);
}

template <typename T>
static void dalloc(T **p, size_t n) {
  HP_HIP(hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T)));
}

// Capacities from the config (DESIGN.md "Data layout"): P is sized for the largest state the
// config can reach (IMU + intrinsics + dt + cams + (max_clones+1) clones + max_slam landmarks +
// anchors + p_IinU), so appends / deletions never reallocate.
void Engine::alloc_device() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device_)
    throw HpError(UVIO_HP_E_DEVICE, "no HIP device " + std::to_string(device_));
  HP_HIP(hipSetDevice(device_));
  HP_HIP(hipStreamCreateWithFlags(&d_.stream, hipStreamNonBlocking));
  HP_HIP(hipEventCreate(&d_.ev0));
  HP_HIP(hipEventCreate(&d_.ev1));
  HP_HIP(hipStreamCreateWithFlags(&d_.aux, hipStreamNonBlocking));
  HP_HIP(hipEventCreateWithFlags(&d_.ev_aux_in, hipEventDisableTiming));
  HP_HIP(hipEventCreateWithFlags(&d_.ev_aux_out, hipEventDisableTiming));
  HP_HIP(hipStreamCreateWithFlags(&d_.copy, hipStreamNonBlocking));
  HP_HIP(hipEventCreateWithFlags(&d_.ev_copy, hipEventDisableTiming));
  kprof_.stream = d_.stream;
  HP_HIP(hipEventCreateWithFlags(&rt_.copied, hipEventDisableTiming));
  d_.ekf.kp = &kprof_;
  int C = o_.max_clone_size + 2;
  int K = o_.num_cameras;
  int cap = N_ + 6 * C + 3 * std::max(o_.max_slam_features, 0) + 5 * UVIO_HP_MAX_ANCHORS + 3 + 8;
  cap = (cap + 7) / 8 * 8;
  d_.ldp = cap;
  dalloc(&d_.P, (size_t)cap * cap);
  dalloc(&d_.P2, (size_t)cap * cap);
  dalloc(&d_.T, (size_t)cap * 64);
  dalloc(&d_.Phi, 64 * 64);
  dalloc(&d_.Q, 64 * 64);
  dalloc(&d_.dnc, 8);
  dalloc(&d_.iold, 256);
  // update batch capacities
  int maxf = std::max(o_.max_msckf_in_update, 1);
  maxf = std::min(maxf, 4096);
  maxf = std::max(maxf, std::max(o_.max_slam_in_update, o_.max_slam_features));
  maxf = std::min(std::max(maxf, 64), 8192);
  d_.max_feat = maxf;
  int meas_per_feat = std::min(C * K, kMaxMeasPerFeat);
  d_.max_meas_total = maxf * meas_per_feat;
  d_.max_vars_total = maxf * kMaxVarsPerFeat;
  d_.max_rows = maxf * 2 * meas_per_feat;
  d_.max_ncol = cap + 1;
  d_.ldh = (d_.max_ncol + 7) / 8 * 8;
  dalloc(&d_.feats, maxf);
  dalloc(&d_.meas, d_.max_meas_total);
  dalloc(&d_.vars, d_.max_vars_total);
  dalloc(&d_.clones, C + 4);
  dalloc(&d_.cams, UVIO_HP_MAX_CAMS);
  dalloc(&d_.chi2, 1000);
  dalloc(&d_.H, (size_t)d_.max_rows * d_.ldh);
  dalloc(&d_.Tall, (size_t)d_.max_rows * d_.ldh);
  int maxch = std::max((d_.max_rows + 511) / 512 + 1, gram_num_chunks(2048) + 1);  // 512- or 64-row chunks
  dalloc(&d_.partials, (size_t)maxch * d_.max_ncol * d_.max_ncol);
  dalloc(&d_.R, (size_t)2 * d_.max_ncol * d_.ldh);
  dalloc(&d_.hidx, d_.max_ncol + d_.max_rows);
  dalloc(&d_.hidx_pre, (size_t)DeviceBufs::kPreSlots * d_.max_ncol);
  HP_HIP(hipHostMalloc((void **)&d_.hidx_pre_h, sizeof(int) * DeviceBufs::kPreSlots * std::max(d_.max_ncol, 1),
                       hipHostMallocDefault));
  for (auto &e : d_.ev_pre) HP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  int rmax = std::max(d_.max_ncol, kMaxEkfRows);
  dalloc(&d_.ekf.M, (size_t)cap * rmax);
  dalloc(&d_.ekf.W, (size_t)cap * rmax);
  dalloc(&d_.ekf.S, (size_t)5 * rmax * rmax);
  dalloc(&d_.ekf.y, rmax);
  dalloc(&d_.ekf.M3, (size_t)cap * 3);
  dalloc(&d_.ekf.Dinv, (size_t)(rmax / 16 + 1) * 256);
  d_.dx_bytes = sizeof(double) * (cap + 16);
  // one frame chain holds the MSCKF batch, the SLAM chunks and the delayed initialization's two passes
  d_.fout_cap = maxf + 3 * std::max(o_.max_slam_features, 0) + 64;
  d_.chain_k = std::max(o_.max_slam_features, 1) + std::max(o_.max_slam_features, 1) / std::max(o_.max_slam_in_update, 1) + 4;
  d_.chain_stride = (size_t)cap + 16;
  // [chain regions (reversed) | dx block (neg, dx) | fout] on the device and mirrored in pinned memory
  const size_t reg_bytes = sizeof(double) * d_.chain_k * d_.chain_stride;
  const size_t res_bytes = reg_bytes + d_.dx_bytes + sizeof(DFeatOut) * d_.fout_cap;
  HP_HIP(hipMalloc((void **)&d_.chain, res_bytes));
  HP_HIP(hipMemset(d_.chain, 0, res_bytes));
  d_.dxneg = (double *)((char *)d_.chain + reg_bytes);
  d_.fout = (DFeatOut *)((char *)d_.dxneg + d_.dx_bytes);
  dalloc(&d_.acc, 4);
  dalloc(&d_.shard, (size_t)d_.max_ncol * d_.max_ncol + 2);
  d_.ekf.neg = (int *)d_.dxneg;
  d_.ekf.dx = d_.dxneg + 1;
  HP_HIP(hipHostMalloc((void **)&d_.chain_host, res_bytes + sizeof(double) * 16 + 64, hipHostMallocDefault));
  // chi2 table: boost::math::quantile(chi_squared(dof), 0.95) for dof 1..999 (UpdaterMSCKF.cpp:52-55)
  for (int i = 1; i < 1000; i++) chi2_table_[i] = chi2_quantile95(i);
  HP_HIP(hipMemcpy(d_.chi2, chi2_table_.data(), 1000 * sizeof(double), hipMemcpyHostToDevice));
  // pinned staging: batch upload + small downloads
  d_.pin_bytes = sizeof(DFeat) * maxf + sizeof(DMeas) * d_.max_meas_total + sizeof(DVar) * d_.max_vars_total +
                 sizeof(DClone) * (C + 4) + sizeof(DCam) * UVIO_HP_MAX_CAMS + sizeof(int) * (d_.max_ncol + d_.max_rows) +
                 sizeof(double) * (cap + 16) + sizeof(DFeatOut) * d_.fout_cap + sizeof(double) * 16 + 4096;
  HP_HIP(hipHostMalloc(&d_.pin, d_.pin_bytes, hipHostMallocDefault));
  char *pb = (char *)d_.chain_host + reg_bytes;
  d_.neg_host = (int *)pb;  // same layout as dxneg
  d_.dx_host = (double *)(pb + sizeof(double));
  d_.fout_host = (DFeatOut *)(pb + d_.dx_bytes);
  d_.aux_host = (double *)(pb + d_.dx_bytes + sizeof(DFeatOut) * d_.fout_cap);
  d_.frame_bytes = sizeof(DClone) * (C + 4) + sizeof(DCam) * UVIO_HP_MAX_CAMS + sizeof(DPoseVal) * (C + 4 + UVIO_HP_MAX_CAMS) +
                   sizeof(double) * cap + 1024;
  dalloc(&d_.frame, d_.frame_bytes);
  // upload staging (batch tables, Phi / Q, column maps)
  d_.stg_cap = d_.pin_bytes + 2 * 64 * 64 * sizeof(double) + 64 * 1024;
  // test hook: a smaller ring recycles every few batches (tests/test_gpu_configs.py staging test)
  if (const char *e = std::getenv("UVIO_HP_STAGE_BYTES")) d_.stg_cap = std::min(d_.stg_cap, (size_t)std::atoll(e));
  if (const char *e = std::getenv("UVIO_HP_NO_PREDETECT")) predetect_on_ = e[0] != '1';
  HP_HIP(hipHostMalloc(&d_.stg_h, d_.stg_cap, hipHostMallocDefault));
  HP_HIP(hipMalloc(&d_.stg_d, d_.stg_cap));
  d_.uwb_stride = (size_t)d_.ldp + 4;
  dalloc(&d_.uwb_reg, kUwbMaxRanges * d_.uwb_stride);
  dalloc(&d_.uwb_h, kUwbMaxRanges * 16);
  HP_HIP(hipHostMalloc((void **)&d_.uwb_host, sizeof(double) * kUwbMaxRanges * d_.uwb_stride, hipHostMallocDefault));
}

void Engine::upload_P_full(const std::vector<double> &Ph, int N) {
  HP_HIP(hipMemcpy2DAsync(d_.P, sizeof(double) * d_.ldp, Ph.data(), sizeof(double) * N, sizeof(double) * N, N,
                          hipMemcpyHostToDevice, d_.stream));
  ++p_epoch_;
  dev_sync();
}
void Engine::download_P(std::vector<double> &Ph) {
  Ph.assign((size_t)N_ * N_, 0.0);
  if (N_ == 0) return;
  HP_HIP(hipMemcpy2DAsync(Ph.data(), sizeof(double) * N_, d_.P, sizeof(double) * d_.ldp, sizeof(double) * N_, N_,
                          hipMemcpyDeviceToHost, d_.stream));
  dev_sync();
}
void Engine::get_cov(double *out, int ld) {
  HP_HIP(hipMemcpy2DAsync(out, sizeof(double) * ld, d_.P, sizeof(double) * d_.ldp, sizeof(double) * N_, N_,
                          hipMemcpyDeviceToHost, d_.stream));
  dev_sync();
}

// A ring: tables are appended after the last flushed one and the ring restarts only when full (after
// a stream sync), so a staged table stays valid on the device until many later launch groups.
void *Engine::stage_bytes(const void *src, size_t bytes) {
  const size_t need = (bytes + 255) / 256 * 256;
  if (need > d_.stg_cap) throw HpError(UVIO_HP_E_CAPACITY, "upload staging exhausted");
  if (d_.stg_used + need > d_.stg_cap) {
    stage_flush();
    dev_sync();
    d_.stg_used = d_.stg_flushed = 0;
    d_.stg_epoch++;
    timing_.stage_restarts++;
  }
  if (bytes) std::memcpy(d_.stg_h + d_.stg_used, src, bytes);
  void *dev = d_.stg_d + d_.stg_used;
  d_.stg_used += need;
  return dev;
}

void *Engine::stage_reserve(size_t bytes, void **host) {
  const size_t need = (bytes + 255) / 256 * 256;
  if (need > d_.stg_cap) throw HpError(UVIO_HP_E_CAPACITY, "upload staging exhausted");
  if (d_.stg_used + need > d_.stg_cap) {
    stage_flush();
    dev_sync();
    d_.stg_used = d_.stg_flushed = 0;
    d_.stg_epoch++;
    timing_.stage_restarts++;
  }
  *host = d_.stg_h + d_.stg_used;
  void *dev = d_.stg_d + d_.stg_used;
  d_.stg_used += need;
  return dev;
}

// With kernels still queued on the main stream the upload goes out on the copy stream and the main stream waits
// on its event: enqueued on the main stream the transfer started only after every kernel queued before it (the
// chain's SLAM tables behind the MSCKF update), and its ~15-20 us from start to completion showed as an idle
// gap before the next launch.  On an idle main stream the copy goes there directly (the cross-stream wait only
// adds latency then).  The ring region is not read by anything queued earlier (reused only after a restart,
// which syncs).  The one exception is a copy queued on the main stream after a restart that still reads the
// previous epoch's bytes (the chain's blob, engine_chain.cpp): its caller passes on_main, so the upload of the
// new epoch, which may overwrite those bytes, is ordered behind the copy.
void Engine::stage_flush(bool on_main) {
  if (d_.stg_used == d_.stg_flushed) return;
  const bool idle = on_main || hipStreamQuery(d_.stream) == hipSuccess;
  HP_HIP(hipMemcpyAsync(d_.stg_d + d_.stg_flushed, d_.stg_h + d_.stg_flushed, d_.stg_used - d_.stg_flushed,
                        hipMemcpyHostToDevice, idle ? d_.stream : d_.copy));
  if (!idle) {
    HP_HIP(hipEventRecord(d_.ev_copy, d_.copy));
    HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_copy, 0));
  }
  d_.stg_flushed = d_.stg_used;
}

void Engine::dev_sync() {
  if (d_.fout_pending) {  // feature results of a batch whose update did not read back (yet)
    HP_HIP(hipMemcpyAsync(d_.fout_host, d_.fout, sizeof(DFeatOut) * d_.fout_pending, hipMemcpyDeviceToHost,
                          d_.stream));
    d_.fout_pending = 0;
  }
  auto t0 = std::chrono::steady_clock::now();
  spin_sync(d_.stream);
  timing_.sync_wait += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  timing_.device_syncs++;
  if (kprof_.on) kprof_.harvest(true);
}

// cumulative per-class kernel statistics since the timing was switched on (flush: wait for the device
// so every recorded launch is counted)
void Engine::kernel_stats(bool flush, uvio_hp_kstat_t *out, int cap, int *n) {
  static const struct {
    const char *name, *kernels;
    int bound;
  } info[KC_COUNT] = {
      {"feature", "k_feature", 1},
      {"chi2", "k_gather_pcan,k_gemm_HPg,k_gemm_HPg_tiled,k_chi2_S,k_chi2_S2,k_chi2", 1},
      {"gram", "k_gram,k_gram_mfma", 1},
      {"ekf_update", "k_ekf_MS,k_ekf_fact,k_ekf_WP,k_gram_reduce,k_info_cholP,k_gemm_mfma,k_info_cholZ,k_trinv16,"
                     "k_trsm_lt,k_info_P,k_di_M,k_di_S,k_info_split1,k_info_split_schur,k_info_split3,k_info_split_out",
       1},
      {"ldl", "k_ekf_fact", 1},
      {"lk", "k_lk", 0},
      {"pyramid", "k_hist_multi,k_pyr_pair", 0},
      {"fast", "k_fast_score,k_fast_select", 0},
      {"subpix", "k_subpix", 0},
  };
  // the tracker's detection stream (predetect on the worker thread) keeps its own event pairs
  const KProf *pre = nullptr;
  if (flush) {
    HP_HIP(hipStreamSynchronize(d_.stream));
    kprof_.harvest(true);
    if (tracker_) pre = &tracker_->pre_prof();
    // LK bytes are counted on the device by both streams' timed launches (LkSlots::bytes), never credited
    if (tracker_) kprof_.bytes[KC_LK] = (double)tracker_->lk_bytes();
  }
  *n = KC_COUNT;
  for (int k = 0; k < KC_COUNT && k < cap; k++) {
    uvio_hp_kstat_t &o = out[k];
    std::memset(&o, 0, sizeof(o));
    std::snprintf(o.name, sizeof(o.name), "%s", info[k].name);
    std::snprintf(o.kernels, sizeof(o.kernels), "%s", info[k].kernels);
    o.bound = info[k].bound;
    o.launches = kprof_.launches[k] + (pre ? pre->launches[k] : 0);
    o.seconds = kprof_.secs[k] + (pre ? pre->secs[k] : 0.0);
    o.flops = kprof_.flops[k] + (pre ? pre->flops[k] : 0.0);
    o.bytes = kprof_.bytes[k] + (pre ? pre->bytes[k] : 0.0);
  }
}

// regions 0 .. nreg-1 of the frame chain, the dx block and the first fo per-feature results: one contiguous span
// of the results block (DeviceBufs::region_dev), one copy
void Engine::chain_results_copy(int nreg, int fo) {
  if (nreg <= 0 && fo <= 0) return;
  const char *d0 = (const char *)d_.region_dev(std::max(nreg, 0) - 1);
  const char *d1 = (const char *)(d_.fout + std::max(fo, 0));
  char *h0 = (char *)d_.region_host(std::max(nreg, 0) - 1);
  HP_HIP(hipMemcpyAsync(h0, d0, (size_t)(d1 - d0), hipMemcpyDeviceToHost, d_.stream));
}

void Engine::read_dx(const char *who) {
  // [neg | dx (N) | chi2, accepted of a delayed-init chi2 gate (EkfScratch::chi2_gate)]
  HPROF("read_dx");
  // [count | dx], and the pending batch results behind them in the same copy
  const size_t bytes = d_.fout_pending ? d_.dx_bytes + sizeof(DFeatOut) * d_.fout_pending
                                       : sizeof(double) * (3 + (size_t)N_);
  d_.fout_pending = 0;
  HP_HIP(hipMemcpyAsync(d_.neg_host, d_.dxneg, bytes, hipMemcpyDeviceToHost, d_.stream));
  dev_sync();
  if (*d_.neg_host > 0) throw HpError(UVIO_HP_E_NUMERIC, std::string(who) + ": negative covariance diagonal");
}

// StateHelper::EKFPropagation on the device (StateHelper.cpp:36-114).  The new block is rows
// s0 .. s0+p-1, or the rows listed in `rows` (several variables at once, block-row Phi).
void Engine::cov_propagate(int s0, int p, const std::vector<int> &iold, const std::vector<double> &Phi,
                           const std::vector<double> &Q, const std::vector<int> *rows) {
  int q = (int)iold.size();
  if (p > 64 || q > 256) throw HpError(UVIO_HP_E_CAPACITY, "propagation block too large");
  const double *dPhi = stage(Phi.data(), (size_t)p * q);
  const double *dQ = stage(Q.data(), (size_t)p * p);
  const int *diold = stage(iold.data(), (size_t)q);
  const int *drows = rows ? stage(rows->data(), rows->size()) : nullptr;
  stage_flush();
  launch_cov_propagate(d_.stream, d_.P, d_.ldp, N_, s0, p, diold, q, dPhi, dQ, d_.T, drows);
  ++p_epoch_;
}

void Engine::check_neg_diag(const char *who) {
  HP_HIP(hipMemsetAsync(d_.ekf.neg, 0, sizeof(int), d_.stream));
  launch_check_diag(d_.stream, d_.P, d_.ldp, N_, d_.ekf.neg);
  HP_HIP(hipMemcpyAsync(d_.neg_host, d_.ekf.neg, sizeof(int), hipMemcpyDeviceToHost, d_.stream));
  dev_sync();
  if (*d_.neg_host > 0) throw HpError(UVIO_HP_E_NUMERIC, std::string(who) + ": negative covariance diagonal");
}

// cov_propagate of the IMU block (contiguous rows s0 ..) followed by clone_imu_pose, as ONE launch when the
// propagation is small (launch_prop_clone); false when it did nothing (the caller takes the two-step path)
bool Engine::cov_propagate_clone(int s0, int p, const std::vector<int> &iold, const std::vector<double> &Phi,
                                 const std::vector<double> &Q, bool do_dt, const double *ddnc) {
  const int q = (int)iold.size();
  if (p > 32 || q > 32 || N_ + 6 > d_.ldp || N_ * p > 8 * 1024 || std::getenv("UVIO_HP_NO_PROP_FUSE"))
    return false;  // (launch_prop_clone's bounds)
  const double *dPhi = stage(Phi.data(), (size_t)p * q);
  const double *dQ = stage(Q.data(), (size_t)p * p);
  const int *diold = stage(iold.data(), (size_t)q);
  stage_flush();
  if (!launch_prop_clone(d_.stream, d_.P, d_.ldp, N_, s0, p, diold, q, dPhi, dQ, d_.T, imu_->id,
                         do_dt ? calib_dt_->id : 0, do_dt ? ddnc : d_.dnc, do_dt ? 1 : 0))
    throw HpError(UVIO_HP_E_CAPACITY, "fused propagation refused after the size check");
  ++p_epoch_;
  return true;
}

// StateHelper::clone(imu->pose()) + augment_clone (StateHelper.cpp:341-391, 579-616)
VarP Engine::clone_imu_pose(const double *dnc, bool do_dt, const double *staged) {
  if (N_ + 6 > d_.ldp) throw HpError(UVIO_HP_E_CAPACITY, "covariance capacity exceeded");
  const double *ddnc = d_.dnc;
  if (do_dt) {
    ddnc = staged;  // already on the device (staged and flushed by the caller)
    if (!ddnc) {
      ddnc = stage(dnc, 6);
      stage_flush();
    }
  }
  launch_clone(d_.stream, d_.P, d_.ldp, N_, imu_->id, do_dt ? calib_dt_->id : 0, ddnc, do_dt ? 1 : 0);
  ++p_epoch_;
  return add_clone_var();
}

// the clone's host variable (its covariance rows / columns N_ .. N_+5 are written on the device)
VarP Engine::add_clone_var() {
  VarP pose = mk(V_POSE, 6, 7);
  for (int k = 0; k < 7; k++) pose->val[k] = imu_->val[k], pose->fej[k] = imu_->fej[k];
  pose->id = N_;
  N_ += 6;
  vars_.push_back(pose);
  return pose;
}

// StateHelper::marginalize (StateHelper.cpp:271-339)
void Engine::marginalize(const VarP &m) {
  int m0 = m->id, ms = m->size;
  launch_marginalize(d_.stream, d_.P, d_.P2, d_.ldp, N_, m0, ms);
  std::swap(d_.P, d_.P2);
  ++p_epoch_;
  std::vector<VarP> keep;
  for (auto &v : vars_)
    if (v != m) {
      if (v->id > m0) v->id -= ms;
      keep.push_back(v);
    }
  vars_ = keep;
  m->id = -1;
  N_ -= ms;
}

void Engine::marginalize_many(const std::vector<VarP> &ms) {
  if (ms.empty()) return;
  if (ms.size() == 1) {
    marginalize(ms[0]);
    return;
  }
  std::vector<uint8_t> gone((size_t)N_, 0);
  for (const auto &m : ms)
    for (int k = 0; k < m->size; k++) gone[(size_t)(m->id + k)] = 1;
  std::vector<int> src, before((size_t)N_ + 1, 0);
  src.reserve((size_t)N_);
  for (int i = 0; i < N_; i++) {
    before[(size_t)i + 1] = before[(size_t)i] + gone[(size_t)i];
    if (!gone[(size_t)i]) src.push_back(i);
  }
  const int Nn = (int)src.size();
  const int *dsrc = stage(src.data(), src.size());
  stage_flush();
  launch_marginalize_multi(d_.stream, d_.P, d_.P2, d_.ldp, Nn, dsrc);
  std::swap(d_.P, d_.P2);
  ++p_epoch_;
  std::vector<VarP> keep;
  keep.reserve(vars_.size());
  for (auto &v : vars_)
    if (!gone[(size_t)v->id]) {  // (variables are disjoint intervals: a removed start index is one of ms)
      v->id -= before[(size_t)v->id];
      keep.push_back(v);
    }
  vars_ = keep;
  for (const auto &m : ms) m->id = -1;
  N_ = Nn;
}

// algorithmic FP64 FLOPs of one EKFUpdate with r rows over n columns of an N-dim state (SURVEY.md §8(d)
// F_ekf: M = P H^T, S, its factor, K, P - K M^T, dx) and the bytes it must move at least (P read and
// written once, H and the residual read)
double ekf_flops(double N, double n, double r) {
  return 2 * N * n * r + 2 * r * n * n + 2 * r * r * n + r * r * r + 2 * N * r * r + N * N * r + 2 * N * r;
}
double ekf_bytes(double N, double n, double r) { return 8.0 * (2 * N * N + r * (n + 1) + N); }

void Engine::apply_dx(const double *dx) {
  for (auto &v : vars_) v->update(dx + v->id);
  if (o_.do_calib_camera_intrinsics)
    for (auto &c : calib_intr_)
      for (int k = 0; k < 8; k++) cams_[c.first].v[k] = c.second->val[k];
}

// EKF update of P on the device with rows H (r x n, ld) / residual; dx applied to the host mean
void Engine::ekf_update_rows(const double *Hdev, int ldh, int r, int n, const std::vector<int> &hidx,
                             const double *resdev, int res_stride, double sigma2, const int *hidx_dev,
                             const std::function<bool()> &apply, const int *gate, const double *Tdev) {
  if (r <= 0) {
    if (apply) apply();
    return;
  }
  if (r > kMaxEkfRows) throw HpError(UVIO_HP_E_CAPACITY, "direct EKF update with more than 255 rows");
  if (!hidx_dev) {
    hidx_dev = stage(hidx.data(), (size_t)n);
    stage_flush();
  }
  d_.ekf.gate = gate;
  {
    HPROF("ekf_rows.launch");
    KScope ks(&kprof_, KC_EKF);
    d_.ekf.Tall = Tdev;
    d_.ekf.ldt = ldh;
    launch_ekf_update(d_.stream, d_.P, d_.ldp, N_, Hdev, ldh, r, n, hidx_dev, resdev, res_stride, sigma2, d_.ekf);
    d_.ekf.Tall = nullptr;
    ++p_epoch_;
  }
  kprof_.credit(KC_EKF, ekf_flops(N_, n, r), ekf_bytes(N_, n, r));
  read_dx("EKFUpdate");
  if (!apply || apply()) apply_dx(d_.dx_host);
}

// EKF update from the Gram partials of a stacked batch (compressed path, m > n)
void Engine::ekf_update_info(int nch, int n, const std::vector<int> &hidx, double sigma2,
                             const std::function<bool()> &apply, const int *gate, const double *partials) {
  // the prefactor of these columns is in flight and P is unchanged since it was enqueued
  const bool inflight = d_.pre_N >= 0;
  const bool pre = inflight && d_.pre_N == N_ && d_.pre_hidx == hidx && d_.pre_epoch == p_epoch_;
  d_.pre_hidx.clear();
  d_.pre_N = -1;
  d_.ekf.gate = gate;
  const double *G = partials ? partials : d_.partials;
  if (pre) {
    HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_aux_out, 0));
    KScope ks(&kprof_, KC_EKF);
    launch_ekf_info_post(d_.stream, d_.P, d_.ldp, N_, G, nch, n, sigma2, d_.R, d_.ekf);
  } else {
    // a stale prefactor still writes the factor scratch on the side stream: order the full update after it
    if (inflight) HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_aux_out, 0));
    const int *dh = stage(hidx.data(), (size_t)n);
    stage_flush();
    KScope ks(&kprof_, KC_EKF);
    launch_ekf_info(d_.stream, d_.P, d_.ldp, N_, G, nch, n, dh, sigma2, d_.R, d_.ekf);
  }
  ++p_epoch_;
  // the timed launches: without the side-stream prefactor (Cholesky of P_II, n^3 / 3, and V, N n^2) when it ran
  const double fl = ekf_flops(N_, n, n) - (pre ? (double)n * n * n / 3.0 + (double)N_ * n * n : 0.0);
  kprof_.credit(KC_EKF, fl, ekf_bytes(N_, n, n));
  read_dx("EKFUpdate");
  if (!apply || apply()) apply_dx(d_.dx_host);
}

// The information-form update's prefactor (launch_ekf_info_pre: P_II = L L^T, V = P[:,I] L^-T) for the
// columns hidx of the state as it is now, on the side stream, behind everything enqueued so far; the
// next ekf_update_info on the same columns and state size waits for it instead of factoring again.  Between
// the two calls only kernels that read P may be enqueued (the feature group, chi2 gate and Gram do).
void Engine::info_prefactor(const std::vector<int> &hidx) {
  const int n = (int)hidx.size();
  if (n < 1 || n > d_.max_ncol) return;
  const int slot = d_.pre_slot;
  d_.pre_slot = (d_.pre_slot + 1) % DeviceBufs::kPreSlots;
  int *hh = d_.hidx_pre_h + (size_t)slot * d_.max_ncol, *hd = d_.hidx_pre + (size_t)slot * d_.max_ncol;
  HP_HIP(hipEventSynchronize(d_.ev_pre[slot]));  // this slot's copy, kPreSlots prefactors ago, has run
  std::memcpy(hh, hidx.data(), sizeof(int) * n);
  HP_HIP(hipEventRecord(d_.ev_aux_in, d_.stream));
  HP_HIP(hipStreamWaitEvent(d_.aux, d_.ev_aux_in, 0));
  HP_HIP(hipMemcpyAsync(hd, hh, sizeof(int) * n, hipMemcpyHostToDevice, d_.aux));
  HP_HIP(hipEventRecord(d_.ev_pre[slot], d_.aux));
  launch_ekf_info_pre(d_.aux, d_.P, d_.ldp, N_, n, hd, d_.ekf);
  HP_HIP(hipEventRecord(d_.ev_aux_out, d_.aux));
  d_.pre_hidx = hidx;
  d_.pre_N = N_;
  d_.pre_epoch = p_epoch_;
}

// StateHelper::set_initial_covariance (StateHelper.cpp:199-223).  Start-up only (initialize_with_gt,
// anchor init): P is read back, the blocks are written, and P is re-uploaded.
void Engine::set_initial_covariance(const std::vector<double> &cov, const std::vector<VarP> &order) {
  std::vector<double> Ph;
  download_P(Ph);
  int ii = 0;
  for (auto &a : order) {
    int kk = 0;
    for (auto &b : order) {
      for (int i = 0; i < a->size; i++)
        for (int j = 0; j < b->size; j++) {
          int ncov = 0;
          for (auto &c : order) ncov += c->size;
          Ph[(size_t)(a->id + i) * N_ + b->id + j] = cov[(size_t)(ii + i) * ncov + kk + j];
        }
      kk += b->size;
    }
    ii += a->size;
  }
  for (int i = 0; i < N_; i++)
    for (int j = 0; j < i; j++) Ph[(size_t)i * N_ + j] = Ph[(size_t)j * N_ + i];
  upload_P_full(Ph, N_);
}

// StateHelper::initialize_invertible (StateHelper.cpp:484-577) — start-up only (UWB extrinsic /
// anchor initialization in the UVioManager ctor, UVioManager.cpp:33-55, 221-247).
void Engine::initialize_invertible_host(const VarP &v, const std::vector<std::pair<int, int>> &H_order,
                                        const std::vector<double> &H_R, const std::vector<double> &H_L,
                                        const std::vector<double> &R, const std::vector<double> &res) {
  int r = (int)res.size(), sz = v->size;
  int nh = 0;
  for (auto &h : H_order) nh += h.second;
  std::vector<int> idx;
  for (auto &h : H_order)
    for (int k = 0; k < h.second; k++) idx.push_back(h.first + k);
  std::vector<double> Ph;
  download_P(Ph);
  int N = N_;
  // M_a = P[:, idx] H_R^T (N x r)
  std::vector<double> Ma((size_t)N * r, 0.0);
  for (int i = 0; i < N; i++)
    for (int a = 0; a < r; a++) {
      double s = 0;
      for (int k = 0; k < nh; k++) s += Ph[(size_t)i * N + idx[k]] * H_R[a * nh + k];
      Ma[(size_t)i * r + a] = s;
    }
  // M = H_R P_small H_R^T + R
  std::vector<double> M((size_t)r * r);
  for (int a = 0; a < r; a++)
    for (int b = 0; b < r; b++) {
      double s = 0;
      for (int k = 0; k < nh; k++) s += H_R[a * nh + k] * Ma[(size_t)idx[k] * r + b];
      M[a * r + b] = s + R[a * r + b];
    }
  // H_L^-1 (small, Gauss-Jordan)
  std::vector<double> A = H_L, Inv((size_t)sz * sz, 0.0);
  for (int i = 0; i < sz; i++) Inv[i * sz + i] = 1;
  for (int c = 0; c < sz; c++) {
    int piv = c;
    for (int i = c + 1; i < sz; i++)
      if (std::fabs(A[i * sz + c]) > std::fabs(A[piv * sz + c])) piv = i;
    for (int j = 0; j < sz; j++) std::swap(A[c * sz + j], A[piv * sz + j]), std::swap(Inv[c * sz + j], Inv[piv * sz + j]);
    double d = A[c * sz + c];
    for (int j = 0; j < sz; j++) A[c * sz + j] /= d, Inv[c * sz + j] /= d;
    for (int i = 0; i < sz; i++)
      if (i != c) {
        double f = A[i * sz + c];
        for (int j = 0; j < sz; j++) A[i * sz + j] -= f * A[c * sz + j], Inv[i * sz + j] -= f * Inv[c * sz + j];
      }
  }
  int Nn = N + sz;
  std::vector<double> Pn((size_t)Nn * Nn, 0.0);
  for (int i = 0; i < N; i++) std::memcpy(&Pn[(size_t)i * Nn], &Ph[(size_t)i * N], sizeof(double) * N);
  for (int i = 0; i < N; i++)
    for (int a = 0; a < sz; a++) {
      double s = 0;
      for (int b = 0; b < r; b++) s += Ma[(size_t)i * r + b] * Inv[a * sz + b];
      Pn[(size_t)i * Nn + N + a] = -s;
      Pn[(size_t)(N + a) * Nn + i] = -s;
    }
  for (int a = 0; a < sz; a++)
    for (int b = 0; b < sz; b++) {
      double s = 0;
      for (int c = 0; c < r; c++)
        for (int e = 0; e < r; e++) s += Inv[a * sz + c] * M[c * r + e] * Inv[b * sz + e];
      Pn[(size_t)(N + a) * Nn + N + b] = s;
    }
  std::vector<double> dxv(sz, 0.0);
  for (int a = 0; a < sz; a++)
    for (int b = 0; b < r; b++) dxv[a] += Inv[a * sz + b] * res[b];
  v->update(dxv.data());
  v->id = N;
  vars_.push_back(v);
  N_ = Nn;
  upload_P_full(Pn, Nn);
}

int Engine::state_vector(double *out, int cap, int *meta, int meta_cap, int *nvars, bool fej) {
  int k = 0, nv = 0;
  for (auto &v : vars_) {
    if (meta && 3 * nv + 2 < meta_cap) {
      meta[3 * nv] = v->kind;
      meta[3 * nv + 1] = v->id;
      meta[3 * nv + 2] = v->size;
    }
    for (int i = 0; i < v->vlen; i++) {
      if (k < cap) out[k] = fej ? v->fej[i] : v->val[i];
      k++;
    }
    nv++;
  }
  if (nvars) *nvars = nv;
  return k;
}

std::vector<double> Engine::clone_times() const {
  std::vector<double> t;
  for (auto &c : clones_) t.push_back(c.first);
  return t;
}

}  // namespace uvhp

namespace uvhp {

// Standalone StateHelper::EKFUpdate on a caller-provided covariance (kernel-level parity entry):
// the same device kernels the manager uses, on temporary device buffers.
int Engine::ekf_update_standalone(double *P, int N, const int *H_index, int n, const double *H, int r,
                                  const double *res, double sigma2, double *dx_out, bool compress) {
  if (!P || N <= 0 || n <= 0 || r <= 0 || !H || !res || !H_index || !dx_out) return UVIO_HP_E_ARG;
  for (int j = 0; j < n; j++)
    if (H_index[j] < 0 || H_index[j] >= N) return UVIO_HP_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return UVIO_HP_E_DEVICE;
  hipStream_t s;
  HP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int ldh = n + 1;
  bool info = compress && r > n;
  if (!info && r > kMaxEkfRows) return UVIO_HP_E_CAPACITY;
  int rw = std::max(r, n + 1);
  int nch = gram_num_chunks(r);
  double *dP, *dH, *dM, *dW, *dS, *dy, *ddx, *dDinv, *dPart = nullptr, *dG = nullptr;
  int *dI, *dneg;
  dalloc(&dP, (size_t)N * N);
  dalloc(&dH, (size_t)r * ldh);
  dalloc(&dM, (size_t)N * rw);
  dalloc(&dW, (size_t)N * rw);
  dalloc(&dS, (size_t)5 * rw * rw);
  dalloc(&dy, rw);
  dalloc(&dDinv, (size_t)(rw / 16 + 1) * 256);
  if (info) {
    dalloc(&dPart, (size_t)nch * ldh * ldh);
    dalloc(&dG, (size_t)ldh * ldh);
  }
  dalloc(&ddx, N);
  dalloc(&dI, n);
  dalloc(&dneg, 2 + n);
  std::vector<double> Ha((size_t)r * ldh);
  for (int i = 0; i < r; i++) {
    std::memcpy(&Ha[(size_t)i * ldh], H + (size_t)i * n, sizeof(double) * n);
    Ha[(size_t)i * ldh + n] = res[i];
  }
  HP_HIP(hipMemcpyAsync(dP, P, sizeof(double) * N * N, hipMemcpyHostToDevice, s));
  HP_HIP(hipMemcpyAsync(dH, Ha.data(), sizeof(double) * Ha.size(), hipMemcpyHostToDevice, s));
  HP_HIP(hipMemcpyAsync(dI, H_index, sizeof(int) * n, hipMemcpyHostToDevice, s));
  HP_HIP(hipMemsetAsync(dneg, 0, sizeof(int), s));
  EkfScratch sc{dM, dW, dS, dy, ddx, dneg, dDinv};
  if (info) {
    int nc2 = 0;
    launch_gram(s, dH, r, ldh, ldh, dPart, &nc2);
    launch_ekf_info(s, dP, N, N, dPart, nc2, n, dI, sigma2, dG, sc);
  } else {
    launch_ekf_update(s, dP, N, N, dH, ldh, r, n, dI, dH + n, ldh, sigma2, sc);
  }
  int neg = 0;
  HP_HIP(hipMemcpyAsync(P, dP, sizeof(double) * N * N, hipMemcpyDeviceToHost, s));
  HP_HIP(hipMemcpyAsync(dx_out, ddx, sizeof(double) * N, hipMemcpyDeviceToHost, s));
  HP_HIP(hipMemcpyAsync(&neg, dneg, sizeof(int), hipMemcpyDeviceToHost, s));
  HP_HIP(hipStreamSynchronize(s));
  void *ptrs[] = {dP, dH, dM, dW, dS, dy, ddx, dDinv, dI, dneg, dPart, dG};
  for (void *p : ptrs)
    if (p) hipFree(p);
  hipStreamDestroy(s);
  return neg > 0 ? UVIO_HP_E_NUMERIC : 0;
}

// Standalone measurement compression: R factor of [H | res] (m x (n+1)) via the Gram + Cholesky kernels
int Engine::compress_standalone(const double *A, int m, int n, double *R_out) {
  if (!A || m <= 0 || n <= 0 || !R_out) return UVIO_HP_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return UVIO_HP_E_DEVICE;
  hipStream_t s;
  HP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int ncol = n + 1;
  int nch = gram_num_chunks(m);
  double *dA, *dPart, *dR;
  dalloc(&dA, (size_t)m * ncol);
  dalloc(&dPart, (size_t)nch * ncol * ncol);
  dalloc(&dR, (size_t)2 * ncol * ncol);
  HP_HIP(hipMemcpyAsync(dA, A, sizeof(double) * m * ncol, hipMemcpyHostToDevice, s));
  int nc2 = 0;
  launch_gram(s, dA, m, ncol, ncol, dPart, &nc2);
  launch_gram_reduce_chol(s, dPart, nc2, ncol, dR, ncol);
  HP_HIP(hipMemcpyAsync(R_out, dR, sizeof(double) * ncol * ncol, hipMemcpyDeviceToHost, s));
  HP_HIP(hipStreamSynchronize(s));
  hipFree(dA);
  hipFree(dPart);
  hipFree(dR);
  hipStreamDestroy(s);
  return 0;
}


// CamBase::undistort_f (ov_core/src/cam/CamBase.h:89, CamRadtan.h:99 / CamEqui.h:108) over n points on the
// device; the points whose float result could depend on the equidistant model's tan (cam_undistort_f's flag)
// are recomputed here with the host's libm, so uvn is the host's result for every point.
int Engine::undistort_standalone(int model, const double cam[8], int n, const float *uv, float *uvn, uint8_t *amb) {
  if ((model != 0 && model != 1) || !cam || n < 0 || (n > 0 && (!uv || !uvn))) return UVIO_HP_E_ARG;
  if (n == 0) return 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return UVIO_HP_E_DEVICE;
  CamParams c{};
  c.model = model;
  for (int k = 0; k < 8; k++) c.v[k] = cam[k];
  hipStream_t s;
  HP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *d_uv, *d_uvn;
  uint8_t *d_amb;
  HP_HIP(hipMalloc(&d_uv, sizeof(float) * 2 * (size_t)n));
  HP_HIP(hipMalloc(&d_uvn, sizeof(float) * 2 * (size_t)n));
  HP_HIP(hipMalloc(&d_amb, (size_t)n));
  std::vector<uint8_t> h_amb(n);
  HP_HIP(hipMemcpyAsync(d_uv, uv, sizeof(float) * 2 * (size_t)n, hipMemcpyHostToDevice, s));
  launch_undistort_points(s, c, n, d_uv, d_uvn, d_amb);
  HP_HIP(hipMemcpyAsync(uvn, d_uvn, sizeof(float) * 2 * (size_t)n, hipMemcpyDeviceToHost, s));
  HP_HIP(hipMemcpyAsync(h_amb.data(), d_amb, (size_t)n, hipMemcpyDeviceToHost, s));
  HP_HIP(hipStreamSynchronize(s));
  hipFree(d_uv);
  hipFree(d_uvn);
  hipFree(d_amb);
  hipStreamDestroy(s);
  for (int i = 0; i < n; i++) {
    if (h_amb[i]) cam_undistort_f(c, uv[2 * i], uv[2 * i + 1], uvn[2 * i], uvn[2 * i + 1]);
    if (amb) amb[i] = h_amb[i];
  }
  return 0;
}

int Engine::grid_order_standalone(const uint8_t *resp, const int *off, int ncell, int kmax, int depth,
                                  int *arrangement, int *top) {
  if (ncell < 0 || !off || kmax < 0 || kmax > 64 || (kmax > 0 && !top)) return UVIO_HP_E_ARG;
  if (ncell == 0) return 0;
  int nmax = 0;
  for (int c = 0; c < ncell; c++) {
    if (off[c + 1] < off[c]) return UVIO_HP_E_ARG;
    nmax = std::max(nmax, off[c + 1] - off[c]);
  }
  const int total = off[ncell];
  if (total > 0 && (!resp || !arrangement)) return UVIO_HP_E_ARG;
  if (nmax > 16384) return UVIO_HP_E_CAPACITY;  // 8 bytes of LDS per candidate
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return UVIO_HP_E_DEVICE;
  hipStream_t s;
  HP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint8_t *d_resp = nullptr;
  int *d_off = nullptr, *d_arr = nullptr, *d_top = nullptr;
  const size_t ntop = (size_t)ncell * (size_t)std::max(kmax, 1);
  HP_HIP(hipMalloc(&d_resp, std::max(total, 1)));
  HP_HIP(hipMalloc(&d_off, sizeof(int) * (size_t)(ncell + 1)));
  HP_HIP(hipMalloc(&d_arr, sizeof(int) * (size_t)std::max(total, 1)));
  HP_HIP(hipMalloc(&d_top, sizeof(int) * ntop));
  if (total > 0) HP_HIP(hipMemcpyAsync(d_resp, resp, (size_t)total, hipMemcpyHostToDevice, s));
  HP_HIP(hipMemcpyAsync(d_off, off, sizeof(int) * (size_t)(ncell + 1), hipMemcpyHostToDevice, s));
  if (kmax > 0) HP_HIP(hipMemcpyAsync(d_top, top, sizeof(int) * ntop, hipMemcpyHostToDevice, s));
  launch_grid_order_probe(s, d_resp, d_off, ncell, nmax, kmax, depth, d_arr, d_top);
  HP_HIP(hipGetLastError());
  if (total > 0) HP_HIP(hipMemcpyAsync(arrangement, d_arr, sizeof(int) * (size_t)total, hipMemcpyDeviceToHost, s));
  if (kmax > 0) HP_HIP(hipMemcpyAsync(top, d_top, sizeof(int) * ntop, hipMemcpyDeviceToHost, s));
  HP_HIP(hipStreamSynchronize(s));
  hipFree(d_resp);
  hipFree(d_off);
  hipFree(d_arr);
  hipFree(d_top);
  hipStreamDestroy(s);
  return 0;
}

}  // namespace uvhp
