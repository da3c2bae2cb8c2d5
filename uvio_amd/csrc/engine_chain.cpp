// The frame's update as one device chain (VioManager.cpp:498-547: UpdaterMSCKF::update, UpdaterSLAM::update in
// chunks of max_slam_in_update, UpdaterSLAM::delayed_init).
//
// Each reference updater linearizes at the state the previous one left: the SLAM chunk after the MSCKF update,
// the next chunk after it, every delayed initialization after the one before.  Here the host builds every
// batch's tables up front from the frame's selection and enqueues all of it on the library stream; the state
// the linearizations read lives on the device for the length of the chain:
//   * the clone / camera tables (DClone, DCam) with the JPL pose values behind them (DPoseVal) and an additive
//     mirror of the mean indexed by covariance id (the SLAM landmarks' values), all in one dedicated buffer;
//   * after every update k_chain_apply moves them by the update's dx with the host's own formulas
//     (Var::update, quat_2_Rot; the same FP64 operations in the same order), gated by the update's acceptance;
//   * the delayed initialization's batch triangulation feeds its per-candidate linearization on the device
//     (DBatchParams::tri_in), each candidate's landmark goes into a fixed slot N0 + 3 j whose rows are zeroed
//     when the candidate is rejected (zero rows of P make zero rows of every later M and K), and the host
//     compacts the zeroed slots away afterwards in one gather.
// Every update writes its dx into its own region of d_.chain; after ONE wait the host replays the updaters in
// order on its mean (per-feature results, dx, landmark creation, fail counts), exactly the sequence the
// reference applies.  The batches' decisions (accepted rows, chi2, LM status) never need the host in between.
#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "engine.h"
#include "hprof.h"

namespace uvhp {

using clk = std::chrono::steady_clock;
static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

void Engine::marginalize_slots(std::vector<int> slots) {
  if (slots.empty()) return;
  std::sort(slots.begin(), slots.end());
  std::vector<int> src;
  src.reserve(N_);
  size_t k = 0;
  for (int i = 0; i < N_; i++) {
    while (k < slots.size() && i >= slots[k] + 3) k++;
    if (k < slots.size() && i >= slots[k] && i < slots[k] + 3) continue;
    src.push_back(i);
  }
  const int Nn = (int)src.size();
  const int *dsrc = stage(src.data(), src.size());
  stage_flush();
  launch_compact(d_.stream, d_.P, d_.P2, d_.ldp, Nn, dsrc);
  std::swap(d_.P, d_.P2);
  ++p_epoch_;
  for (auto &v : vars_) {
    int shift = 0;
    for (int s : slots)
      if (v->id > s) shift += 3;
    v->id -= shift;
  }
  N_ = Nn;
}

// one enqueued batch of the chain and what its replay needs
struct Engine::ChainItem {
  int kind = 0;  // 0 MSCKF, 1 SLAM chunk, 2 delayed-init triangulation, 3 delayed-init candidates
  Engine::Batch b;
  std::vector<FeatP> fv;
  // feature-sharded MSCKF batch (RCCL): fv is this rank's chunk of fv_all, the Gram is all-reduced in the chain
  bool sharded = false;
  std::vector<FeatP> fv_all;
  int region = -1;  // d_.chain region of its update (-1: none enqueued)
  int m = 0;        // stacked rows
  // the batch's staged tables (device addresses after the flush)
  bool staged = false;
  const DFeat *t_feats = nullptr;
  const DMeas *t_meas = nullptr;
  const DVar *t_vars = nullptr;
  const int *t_hidx = nullptr;
};

int Engine::update_frame(std::vector<FeatP> &up, std::vector<FeatP> &slam_upd, std::vector<FeatP> &delayed) {
  stage_ = "update chain";
  last_msckf_.clear();
  last_upd_.clear();
  std::vector<double> clonetimes;
  for (auto &c : clones_) clonetimes.push_back(c.first);
  // ---- 0) each updater's measurement cleaning (UpdaterMSCKF.cpp:69-86, UpdaterSLAM.cpp:68-84 / 262-283);
  // the clone set does not change during the updates, so all three lists are cleaned up front.  The SLAM
  // list is split into its max_slam_in_update chunks first (VioManager.cpp:533-545) and each chunk is
  // cleaned on its own, as UpdaterSLAM::update does: a feature left without measurements shrinks its chunk,
  // it does not pull the next chunk's features forward
  {
    std::vector<uint8_t> few(up.size());
    pool_.parallel_for(up.size(), 64, [&](size_t b0, size_t e0) {
      for (size_t i = b0; i < e0; i++) {
        up[i]->clean_old_measurements(clonetimes);
        few[i] = up[i]->count() < 2;
      }
    });
    std::vector<FeatP> keep;
    keep.reserve(up.size());
    for (size_t i = 0; i < up.size(); i++) {
      if (few[i])
        up[i]->to_delete = true;
      else
        keep.push_back(std::move(up[i]));
    }
    up.swap(keep);
  }
  std::vector<std::vector<FeatP>> slam_chunks;
  {
    const size_t chunk = (size_t)std::max(o_.max_slam_in_update, 1);
    std::vector<FeatP> all;
    for (size_t c0 = 0; c0 < slam_upd.size(); c0 += chunk) {
      std::vector<FeatP> keep;
      for (size_t i = c0; i < std::min(slam_upd.size(), c0 + chunk); i++) {
        FeatP &f = slam_upd[i];
        f->clean_old_measurements(clonetimes);
        if (f->count() < 1)
          f->to_delete = true;
        else
          keep.push_back(f);
      }
      all.insert(all.end(), keep.begin(), keep.end());
      if (!keep.empty()) slam_chunks.push_back(std::move(keep));
    }
    slam_upd.swap(all);
  }
  {
    std::vector<FeatP> keep;
    for (auto &f : delayed) {
      f->clean_old_measurements(clonetimes);
      if (f->count() < 2)
        f->to_delete = true;
      else
        keep.push_back(f);
    }
    delayed.swap(keep);
  }
  if (up.empty() && slam_upd.empty() && delayed.empty()) return 0;
  if (!up.empty() && o_.feat_rep_msckf != 0 && o_.feat_rep_msckf != 4)
    throw HpError(UVIO_HP_E_CONFIG, "feat_rep_msckf: only GLOBAL_3D / ANCHORED_MSCKF_INVERSE_DEPTH are implemented");
  const int rep_slam = o_.feat_rep_slam;
  if (!delayed.empty() && rep_slam != 0 && rep_slam != 2 && rep_slam != 4)
    throw HpError(UVIO_HP_E_CONFIG, "feat_rep_slam: representation not implemented");
  for (auto &f : slam_upd) {
    const VarP &lm = slam_.at(f->featid);
    if (lm->rep != 0 && lm->rep != 2 && lm->rep != 4)
      throw HpError(UVIO_HP_E_CONFIG, "feat_rep_slam: representation not implemented");
  }
  const int N0 = N_;
  const int K = (int)delayed.size();
  if (N0 + 3 * K > d_.ldp) throw HpError(UVIO_HP_E_CAPACITY, "covariance capacity exceeded");

  // ---- 1) host side first: the frame state blob and every batch's tables (the large MSCKF batches write
  // theirs straight into the staging ring while they are built)
  double t_build[3] = {0, 0, 0}, t_launch[3] = {0, 0, 0};
  auto tm0 = clk::now();
  Batch base;
  build_clone_cam_tables(base, false);
  const int ncl = (int)base.clones.size(), ncam = (int)base.cams.size();
  std::vector<char> blob;
  size_t o_cam, o_cv, o_camv, o_xv;
  {
    HPROF("chain.state");
    std::vector<DPoseVal> cv(ncl), camv(ncam);
    int s = 0;
    for (auto &c : clones_) {
      for (int k = 0; k < 4; k++) cv[s].q[k] = c.second->val[k];
      for (int k = 0; k < 3; k++) cv[s].p[k] = c.second->val[4 + k];
      cv[s].pid = c.second->id;
      s++;
    }
    for (int c = 0; c < ncam; c++) {
      const VarP &pose = calib_pose_.at(c);
      for (int k = 0; k < 4; k++) camv[c].q[k] = pose->val[k];
      for (int k = 0; k < 3; k++) camv[c].p[k] = pose->val[4 + k];
      camv[c].pid = pose->id;
    }
    std::vector<double> xv((size_t)d_.ldp, 0.0);
    for (auto &kv : slam_)
      for (int k = 0; k < kv.second->size; k++) xv[(size_t)kv.second->id + k] = kv.second->val[k];
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    o_cam = al(sizeof(DClone) * ncl);
    o_cv = o_cam + al(sizeof(DCam) * ncam);
    o_camv = o_cv + al(sizeof(DPoseVal) * ncl);
    o_xv = o_camv + al(sizeof(DPoseVal) * ncam);
    const size_t bytes = o_xv + sizeof(double) * xv.size();
    if (bytes > d_.frame_bytes) throw HpError(UVIO_HP_E_CAPACITY, "update chain state exceeds its buffer");
    blob.assign(bytes, 0);
    std::memcpy(blob.data(), base.clones.data(), sizeof(DClone) * ncl);
    std::memcpy(blob.data() + o_cam, base.cams.data(), sizeof(DCam) * ncam);
    std::memcpy(blob.data() + o_cv, cv.data(), sizeof(DPoseVal) * ncl);
    std::memcpy(blob.data() + o_camv, camv.data(), sizeof(DPoseVal) * ncam);
    std::memcpy(blob.data() + o_xv, xv.data(), sizeof(double) * xv.size());
  }
  // the blob goes into the ring ahead of the MSCKF tables and is copied to its own buffer once on the device
  // (the ring may restart while later batches are staged)
  const char *blob_staged = stage(blob.data(), blob.size());
  const long long blob_epoch = d_.stg_epoch;
  std::vector<std::unique_ptr<ChainItem>> items;
  ChainItem *msk = nullptr, *tri = nullptr, *cand = nullptr;
  std::vector<ChainItem *> slam_items;
  auto stage_item = [&](ChainItem &it) {
    Batch &b = it.b;
    it.t_feats = stage(b.feats.data(), b.feats.size());
    it.t_meas = b.meas_dev ? b.meas_dev : stage(b.meas.data(), b.meas.size());
    it.t_vars = b.vars_dev ? b.vars_dev : stage(b.vars.data(), b.vars.size());
    it.t_hidx = stage(b.hidx.data(), b.hidx.size());
    b.hidx_dev = it.t_hidx;
    it.staged = true;
  };
  // the bytes a group of batches adds to the ring: staged together (one copy) when they fit behind what it
  // holds, else each right before its launches (enqueue_batch)
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  auto stage_group = [&](const std::vector<ChainItem *> &g) {
    size_t need = 0;
    for (ChainItem *it : g) {
      const Batch &b = it->b;
      need += al(sizeof(DFeat) * b.feats.size()) + al(sizeof(int) * b.hidx.size());
      if (!b.meas_dev) need += al(sizeof(DMeas) * b.meas.size());
      if (!b.vars_dev) need += al(sizeof(DVar) * b.vars.size());
    }
    if (d_.stg_used + need > d_.stg_cap) return;
    for (ChainItem *it : g) stage_item(*it);
  };
  // ---- 1a) UpdaterMSCKF's batch: built, staged with the blob, and launched before the rest is built (the host
  // builds the SLAM / delayed-initialization batches while the device runs the MSCKF update)
  if (!up.empty()) {
    HPROF("chain.msckf.build");
    auto it = std::make_unique<ChainItem>();
    it->kind = 0;
    size_t lo = 0, hi = up.size();
    if (shard_.enabled && (int)up.size() >= shard_.min_features) {
      // UpdaterMSCKF::update split across the ranks inside the chain (shard.cpp: the same partition, pack and
      // all-reduce as msckf_update_sharded; over RCCL the all-reduce is enqueued on the chain's stream)
      std::vector<int> rows(up.size()), bounds(shard_.world + 1);
      for (size_t i = 0; i < up.size(); i++) rows[i] = 2 * up[i]->count() - 3;
      shard_partition(rows.data(), (int)up.size(), shard_.world, bounds.data());
      lo = (size_t)bounds[shard_.rank];
      hi = (size_t)bounds[shard_.rank + 1];
      it->sharded = true;
      it->fv_all = up;
      it->fv.assign(up.begin() + lo, up.begin() + hi);
    } else {
      it->fv = up;
    }
    {
      HPROF("chain.msckf.build.tables");
      build_clone_cam_tables(it->b, false);
    }
    {
      HPROF("chain.msckf.build.add");
      add_features_to_batch(it->b, up, lo, hi, 0, o_.feat_rep_msckf);
    }
    msk = it.get();
    items.push_back(std::move(it));
    HPROF("chain.msckf.build.stage");
    stage_group({msk});
  }
  char *const frame = d_.frame;
  {
    HPROF("chain.stage");
    if (d_.stg_epoch != blob_epoch) {
      // the ring restarted after the blob was staged: it is on the device (the restart flushed it and waited);
      // copied out before anything staged since then is flushed over it -- the flush goes on the same stream,
      // behind the copy (on the copy stream it could overwrite the blob's old bytes before the copy reads them)
      HP_HIP(hipMemcpyAsync(frame, blob_staged, blob.size(), hipMemcpyDeviceToDevice, d_.stream));
      stage_flush(true);
      timing_.chain_blob_old_epoch = 1;
    } else {
      stage_flush();
      HP_HIP(hipMemcpyAsync(frame, blob_staged, blob.size(), hipMemcpyDeviceToDevice, d_.stream));
    }
  }
  t_build[0] = secs(tm0, clk::now());
  DClone *fr_cl = (DClone *)frame;
  DCam *fr_cam = (DCam *)(frame + o_cam);
  DPoseVal *fr_cv = (DPoseVal *)(frame + o_cv), *fr_camv = (DPoseVal *)(frame + o_camv);
  double *fr_xv = (double *)(frame + o_xv);

  int fo = 0, nreg = 0;
  const size_t st = d_.chain_stride;
  auto new_region = [&]() {
    if (nreg >= d_.chain_k) throw HpError(UVIO_HP_E_CAPACITY, "update chain: too many updates in one frame");
    return nreg++;
  };
  auto region = [&](int r) { return d_.region_dev(r); };
  // a batch's feature kernel (+ the chi2 group); results at d_.fout + b.fout_off
  auto enqueue_batch = [&](ChainItem &it, int mode, double s2, double mult, bool chi2, const DFeatOut *tri_in) {
    Batch &b = it.b;
    const int nf = (int)b.feats.size();
    if (nf > d_.max_feat || (int)b.n_meas() > d_.max_meas_total || (int)b.n_vars() > d_.max_vars_total ||
        b.rows > d_.max_rows || b.n_canon + 1 > d_.max_ncol)
      throw HpError(UVIO_HP_E_CAPACITY, "update batch exceeds device capacity");
    if (fo + nf > d_.fout_cap) throw HpError(UVIO_HP_E_CAPACITY, "update chain: per-feature results exceed capacity");
    int max_meas = 0, max_nf = 0;
    for (auto &F : b.feats) {
      max_meas = std::max(max_meas, F.nmeas);
      max_nf = std::max(max_nf, F.nf);
    }
    if (max_meas > kMaxMeasPerFeat) throw HpError(UVIO_HP_E_CAPACITY, "too many measurements per feature");
    b.fout_off = fo;
    fo += nf;
    if (!it.staged) {
      stage_item(it);
      stage_flush();
    }
    if (b.meas_dev && b.stg_epoch != d_.stg_epoch && d_.stg_used > (size_t)((const char *)b.meas_dev - d_.stg_d))
      throw HpError(UVIO_HP_E_CAPACITY, "upload staging ring restarted inside one launch group (UVIO_HP_STAGE_BYTES too small)");
    b.chi2 = chi2;
    DBatchParams bp = batch_params(b, s2, mult);
    bp.xv = fr_xv;
    bp.tri_in = tri_in;
    const char *tsdump = std::getenv("UVIO_HP_FEAT_TS");  // debug only: per-feature phase cycle counts
    if (tsdump) {                                          // 8 k_feature + 4 k_chi2 stamps per feature
      HP_HIP(hipMalloc(&bp.dbg_ts, sizeof(long long) * 16 * nf));
      HP_HIP(hipMemsetAsync(bp.dbg_ts, 0, sizeof(long long) * 16 * nf, d_.stream));
    }
    {
      KScope ks(&kprof_, KC_FEATURE);
      launch_feature_linearize(d_.stream, bp, it.t_feats, it.t_meas, it.t_vars, fr_cl, fr_cam, d_.P, d_.chi2, d_.H,
                               d_.fout + b.fout_off, max_meas, max_nf);
    }
    if (chi2) {
      int max_rows_f = 0;
      for (auto &F : b.feats) max_rows_f = std::max(max_rows_f, (mode == 0) ? 2 * F.nmeas - 3 : 2 * F.nmeas);
      KScope ks(&kprof_, KC_CHI2);
      launch_chi2_batch(d_.stream, bp, it.t_feats, d_.P, it.t_hidx, d_.H, b.rows, d_.Tall, d_.chi2, d_.fout + b.fout_off,
                        max_rows_f, d_.acc, d_.R, &d_.chi2S, &d_.chi2S_cap);
    }
    if (tsdump) {  // synchronous copy-back: debug runs only (the chain loses its overlap)
      std::vector<long long> h(16 * (size_t)nf);
      HP_HIP(hipStreamSynchronize(d_.stream));
      HP_HIP(hipMemcpy(h.data(), bp.dbg_ts, sizeof(long long) * h.size(), hipMemcpyDeviceToHost));
      HP_HIP(hipFree(bp.dbg_ts));
      if (FILE *fp = std::fopen(tsdump, "ab")) {
        for (int i = 0; i < nf; i++) {
          long long rec[16] = {mode, nf, b.feats[i].nmeas, b.feats[i].nf};
          for (int k = 0; k < 12; k++) rec[4 + k] = h[16 * (size_t)i + k];
          std::fwrite(rec, sizeof(long long), 16, fp);
        }
        std::fclose(fp);
      }
    }
    it.m = b.rows;
  };
  // the EKF update of a batch's stacked rows (direct, or information form on their Gram), gated by the batch's
  // accepted count, dx into a fresh region; then the state tables move by it
  auto enqueue_update = [&](ChainItem &it, double s2) {
    Batch &b = it.b;
    const int m = b.rows, n = b.n_canon, ncol = n + 1;
    it.region = new_region();
    EkfScratch sc = d_.ekf;
    sc.dx = region(it.region);
    sc.gate = d_.acc;
    if (m > n || m > kMaxEkfRows) {
      int nch = 0;
      gram(m, ncol, &nch);
      const bool inflight = d_.pre_N >= 0;
      const bool pre = inflight && d_.pre_N == N_ && d_.pre_hidx == b.hidx && d_.pre_epoch == p_epoch_;
      d_.pre_hidx.clear();
      d_.pre_N = -1;
      if (pre) {
        HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_aux_out, 0));
        KScope ks(&kprof_, KC_EKF);
        launch_ekf_info_post(d_.stream, d_.P, d_.ldp, N_, d_.partials, nch, n, s2, d_.R, sc);
      } else {
        if (inflight) HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_aux_out, 0));
        KScope ks(&kprof_, KC_EKF);
        launch_ekf_info(d_.stream, d_.P, d_.ldp, N_, d_.partials, nch, n, b.hidx_dev, s2, d_.R, sc);
      }
      const double fl = ekf_flops(N_, n, n) - (pre ? (double)n * n * n / 3.0 + (double)N_ * n * n : 0.0);
      kprof_.credit(KC_EKF, fl, ekf_bytes(N_, n, n));
    } else {
      sc.Tall = d_.Tall;
      sc.ldt = d_.ldh;
      KScope ks(&kprof_, KC_EKF);
      launch_ekf_update(d_.stream, d_.P, d_.ldp, N_, d_.H, d_.ldh, m, n, b.hidx_dev, d_.H + n, d_.ldh, s2, sc);
      kprof_.credit(KC_EKF, ekf_flops(N_, n, m), ekf_bytes(N_, n, m));
    }
    ++p_epoch_;
    launch_chain_apply(d_.stream, nullptr, d_.acc, sc.neg, sc.dx, fr_cl, fr_cv, ncl, fr_cam, fr_camv, ncam,
                       o_.do_calib_camera_pose, o_.do_calib_camera_intrinsics, fr_xv, N_, d_.P, d_.ldp, N_, -1,
                       sc.dx + N_ + 8);
  };

  // the sharded MSCKF update: this rank's Gram packed with its accepted count and rows, all-reduced over the ranks
  // (every rank enqueues it, rows or not: it is a collective), then the information-form update of the summed
  // Gram on every rank; the totals [accepted, rows] go to the region (N + 10, N + 11) for the replay
  auto enqueue_sharded_update = [&](ChainItem &it, double s2) {
    Batch &b = it.b;
    const int m = b.rows, n = b.n_canon, ncol = n + 1;
    it.region = new_region();
    EkfScratch sc = d_.ekf;
    sc.dx = region(it.region);
    sc.gate = d_.acc;
    int nch = 0;
    if (m > 0) gram(m, ncol, &nch);
    launch_shard_pack(d_.stream, d_.partials, nch, ncol, d_.fout + b.fout_off, (int)b.feats.size(), d_.acc, d_.shard);
    shard_allreduce(d_.shard, (size_t)ncol * ncol + 2);
    launch_shard_unpack(d_.stream, d_.shard, ncol, d_.acc);
    HP_HIP(hipMemcpyAsync(sc.dx + N_ + 10, d_.shard + (size_t)ncol * ncol, 2 * sizeof(double), hipMemcpyDeviceToDevice,
                          d_.stream));
    const bool inflight = d_.pre_N >= 0;
    const bool pre = inflight && d_.pre_N == N_ && d_.pre_hidx == b.hidx && d_.pre_epoch == p_epoch_;
    d_.pre_hidx.clear();
    d_.pre_N = -1;
    if (pre) {
      HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_aux_out, 0));
      KScope ks(&kprof_, KC_EKF);
      launch_ekf_info_post(d_.stream, d_.P, d_.ldp, N_, d_.shard, 1, n, s2, d_.R, sc);
    } else {
      if (inflight) HP_HIP(hipStreamWaitEvent(d_.stream, d_.ev_aux_out, 0));
      KScope ks(&kprof_, KC_EKF);
      launch_ekf_info(d_.stream, d_.P, d_.ldp, N_, d_.shard, 1, n, b.hidx_dev, s2, d_.R, sc);
    }
    kprof_.credit(KC_EKF, ekf_flops(N_, n, n) - (pre ? (double)n * n * n / 3.0 + (double)N_ * n * n : 0.0),
                  ekf_bytes(N_, n, n));
    ++p_epoch_;
    launch_chain_apply(d_.stream, nullptr, d_.acc, sc.neg, sc.dx, fr_cl, fr_cv, ncl, fr_cam, fr_camv, ncam,
                       o_.do_calib_camera_pose, o_.do_calib_camera_intrinsics, fr_xv, N_, d_.P, d_.ldp, N_, -1,
                       sc.dx + N_ + 8);
  };

  // ---- 3) UpdaterMSCKF::update
  auto tl0 = clk::now();
  if (msk) {
    HPROF("chain.msckf");
    PrefactorJoin pj(this);
    if (msk->sharded || msk->b.rows > msk->b.n_canon || msk->b.rows > kMaxEkfRows) info_prefactor(msk->b.hidx);
    const double s2 = o_.msckf_sigma_pix * o_.msckf_sigma_pix;
    enqueue_batch(*msk, 0, s2, o_.msckf_chi2_multipler, true, nullptr);
    if (msk->sharded)
      enqueue_sharded_update(*msk, s2);
    else if (msk->m >= 1)
      enqueue_update(*msk, s2);
  }
  // ---- 1b) the SLAM chunks' and the delayed initialization's batches (host, while the MSCKF update runs)
  auto tb1 = clk::now();
  for (auto &ch : slam_chunks) {
    HPROF("chain.slam.build");
    auto it = std::make_unique<ChainItem>();
    it->kind = 1;
    it->fv = ch;
    Batch &b = it->b;
    build_clone_cam_tables(b, true);
    std::vector<int> lm_canon;
    for (auto &f : it->fv) {
      const VarP &lm = slam_.at(f->featid);
      lm_canon.push_back(b.n_canon);
      for (int k = 0; k < lm->size; k++) b.hidx.push_back(lm->id + k);
      b.n_canon += lm->size;
    }
    for (size_t i = 0; i < it->fv.size(); i++) {
      const VarP &lm = slam_.at(it->fv[i]->featid);
      add_feature(this, it->fv[i], 1, lm->rep, o_, b.cams, b.slot_of_time, b.clones, b.feats, b.meas, b.vars, b.rows,
                  lm.get(), lm_canon[i]);
    }
    slam_items.push_back(it.get());
    items.push_back(std::move(it));
  }
  auto tb2 = clk::now();
  if (K > 0) {
    HPROF("chain.delayed.build");
    auto ti = std::make_unique<ChainItem>();
    ti->kind = 2;
    ti->fv = delayed;
    build_clone_cam_tables(ti->b, false);
    for (auto &f : delayed)
      add_feature(this, f, 2, rep_slam, o_, ti->b.cams, ti->b.slot_of_time, ti->b.clones, ti->b.feats, ti->b.meas,
                  ti->b.vars, ti->b.rows, nullptr, -1);
    tri = ti.get();
    items.push_back(std::move(ti));
    auto ci = std::make_unique<ChainItem>();
    ci->kind = 3;
    ci->fv = delayed;
    Batch &b = ci->b;
    build_clone_cam_tables(b, false);
    for (auto &f : delayed)
      add_feature(this, f, 3, rep_slam, o_, b.cams, b.slot_of_time, b.clones, b.feats, b.meas, b.vars, b.rows, nullptr, -1);
    if (b.rows > d_.max_rows || b.n_canon + 1 > d_.max_ncol || (int)b.n_meas() > d_.max_meas_total ||
        (int)b.n_vars() > d_.max_vars_total)
      throw HpError(UVIO_HP_E_CAPACITY, "delayed-initialization chain exceeds device capacity");
    for (int j = 0; j < K; j++)
      if (b.feats[j].nmeas > kMaxMeasPerFeat) throw HpError(UVIO_HP_E_CAPACITY, "too many measurements per feature");
    cand = ci.get();
    items.push_back(std::move(ci));
  }
  {
    HPROF("chain.stage");
    std::vector<ChainItem *> g(slam_items);
    if (tri) g.push_back(tri);
    if (cand) g.push_back(cand);
    stage_group(g);
    stage_flush();
  }
  auto tb3 = clk::now();
  t_build[1] = secs(tb1, tb2);
  t_build[2] = secs(tb2, tb3);
  auto tl1 = clk::now();
  // ---- 4) UpdaterSLAM::update in chunks of max_slam_in_update (VioManager.cpp:533-545)
  {
    HPROF("chain.slam");
    const double s2 = o_.slam_sigma_pix * o_.slam_sigma_pix;
    for (ChainItem *it : slam_items) {
      PrefactorJoin pj(this);
      if (it->b.rows > it->b.n_canon || it->b.rows > kMaxEkfRows) info_prefactor(it->b.hidx);
      enqueue_batch(*it, 1, s2, o_.slam_chi2_multipler, true, nullptr);
      if (it->m >= 1) enqueue_update(*it, s2);
    }
  }
  auto tl2 = clk::now();
  // ---- 5) UpdaterSLAM::delayed_init: batch triangulation, then per candidate (fixed slot N0 + 3 j) the
  // linearization at the current state, initialize_invertible and the chi2-gated update of the other rows
  if (K > 0) {
    HPROF("chain.delayed");
    const double s2 = o_.slam_sigma_pix * o_.slam_sigma_pix;
    enqueue_batch(*tri, 2, s2, o_.slam_chi2_multipler, false, nullptr);
    Batch &b = cand->b;
    if (fo + K > d_.fout_cap) throw HpError(UVIO_HP_E_CAPACITY, "update chain: per-feature results exceed capacity");
    b.fout_off = fo;
    fo += K;
    if (!cand->staged) {
      stage_item(*cand);
      stage_flush();
    }
    b.chi2 = false;
    DBatchParams bp = batch_params(b, s2, o_.slam_chi2_multipler);
    bp.nfeat = 1;
    bp.gate_out = d_.acc;  // triangulation ok and linearized: gates initialize_invertible and the update
    bp.xv = fr_xv;
    const int n = b.n_canon;
    const DFeatOut *tri_out = d_.fout + tri->b.fout_off;
    DFeatOut *fo3 = d_.fout + b.fout_off;
    cand->region = nreg;
    for (int j = 0; j < K; j++) {
      const DFeat &F = b.feats[j];
      const int Ni = N0 + 3 * j, nup = 2 * F.nmeas - 3;
      bp.tri_in = tri_out + j;
      const char *tsdump = std::getenv("UVIO_HP_FEAT_TS");  // debug only: the candidate's phase cycle counts
      if (tsdump) {
        HP_HIP(hipMalloc(&bp.dbg_ts, sizeof(long long) * 16));
        HP_HIP(hipMemsetAsync(bp.dbg_ts, 0, sizeof(long long) * 16, d_.stream));
      }
      {
        KScope ks(&kprof_, KC_FEATURE);
        launch_feature_linearize(d_.stream, bp, cand->t_feats + j, cand->t_meas, cand->t_vars, fr_cl, fr_cam, d_.P,
                                 d_.chi2, d_.H, fo3 + j, F.nmeas, F.nf);
      }
      if (tsdump) {  // synchronous copy-back: debug runs only
        long long h[16];
        HP_HIP(hipStreamSynchronize(d_.stream));
        HP_HIP(hipMemcpy(h, bp.dbg_ts, sizeof(h), hipMemcpyDeviceToHost));
        HP_HIP(hipFree(bp.dbg_ts));
        bp.dbg_ts = nullptr;
        if (FILE *fp = std::fopen(tsdump, "ab")) {
          long long rec[16] = {3, 1, F.nmeas, F.nf};
          for (int k = 0; k < 12; k++) rec[4 + k] = h[k];
          std::fwrite(rec, sizeof(long long), 16, fp);
          std::fclose(fp);
        }
      }
      EkfScratch sc = d_.ekf;
      sc.dx = region(new_region());
      double *Hrow = d_.H + (size_t)F.row_off * d_.ldh;
      static const bool di_unfused = std::getenv("UVIO_HP_DI_UNFUSED") != nullptr;  // the eight-launch chain (A/B)
      if (nup > 0 && !di_unfused) {
        sc.chi2_gate = d_.acc;
        sc.chi2_thr = o_.slam_chi2_multipler * chi2_table_[std::min(2 * F.nmeas, 999)];
        sc.gate = nullptr;
        KScope ks(&kprof_, KC_EKF);
        launch_di_candidate(d_.stream, d_.P, d_.ldp, Ni, Hrow, d_.ldh, nup, n, cand->t_hidx, s2, sc, fo3 + j,
                            sc.dx + Ni + 5, fr_cl, fr_cv, ncl, fr_cam, fr_camv, ncam, o_.do_calib_camera_pose,
                            o_.do_calib_camera_intrinsics, sc.dx + Ni + 8);
        kprof_.credit(KC_EKF, ekf_flops(Ni + 3, n, nup), ekf_bytes(Ni + 3, n, nup));
        continue;
      }
      launch_init_invertible(d_.stream, d_.P, d_.ldp, Ni, Hrow, d_.ldh, n, cand->t_hidx, nullptr, s2, sc, fo3 + j, d_.acc,
                             sc.dx + Ni + 5);
      if (nup > 0) {
        sc.chi2_gate = d_.acc;
        sc.chi2_thr = o_.slam_chi2_multipler * chi2_table_[std::min(2 * F.nmeas, 999)];
        sc.gate = nullptr;
        KScope ks(&kprof_, KC_EKF);
        launch_ekf_update(d_.stream, d_.P, d_.ldp, Ni + 3, Hrow + 3 * (size_t)d_.ldh, d_.ldh, nup, n, cand->t_hidx,
                          Hrow + 3 * (size_t)d_.ldh + n, d_.ldh, s2, sc);
        kprof_.credit(KC_EKF, ekf_flops(Ni + 3, n, nup), ekf_bytes(Ni + 3, n, nup));
      }
      launch_chain_apply(d_.stream, fo3 + j, d_.acc, nup > 0 ? sc.neg : nullptr, nup > 0 ? sc.dx : nullptr, fr_cl, fr_cv,
                         ncl, fr_cam, fr_camv, ncam, o_.do_calib_camera_pose, o_.do_calib_camera_intrinsics, nullptr, 0,
                         d_.P, d_.ldp, Ni + 3, Ni, sc.dx + Ni + 8);
    }
    ++p_epoch_;
  }
  auto tl3 = clk::now();
  t_launch[0] = secs(tl0, tb1);
  t_launch[1] = secs(tl1, tl2);
  t_launch[2] = secs(tl2, tl3);
  // ---- 5) one readback: every update's region and every batch's per-feature results
  const auto tw = clk::now();
  {
    HPROF("chain.wait");
    chain_results_copy(nreg, fo);
    d_.fout_pending = 0;
    // the next frame's detection (Tracker::predetect) while the device runs this chain: it reads only this
    // frame's tracker results; on the tracker's detection stream and worker thread, joined by the next feed
    if (camera_frame_ && predetect_on_ && tracker_) {
      HPROF("chain.predetect");
      tracker_->predetect_async();
    }
    // the previous frame's retriangulation (engine_retri.cpp; its own stream, so this wait does not cover it)
    if (rt_.pend) {
      HPROF("chain.retri");
      retri_flush();
    }
    if (chain_overlap_) {
      HPROF("chain.overlap");
      auto f = std::move(chain_overlap_);
      chain_overlap_ = nullptr;
      f();
    }
    {
      HPROF("chain.stock");
      refill_feature_stock();
    }
    dev_sync();
  }
  auto tm3 = clk::now();
  // ---- 6) replay on the host mean, in the reference's order
  HPROF("chain.replay");
  auto neg_check = [&](const double *base, int N) {
    if (base[N + 9] > 0.5) throw HpError(UVIO_HP_E_NUMERIC, "EKFUpdate: negative covariance diagonal");
  };
  std::vector<DFeatOut> outs;
  for (auto &itp : items) {
    ChainItem &it = *itp;
    if (it.kind == 0) {
      finish_batch(it.b, 0, outs);
      for (auto &f : it.fv_all) f->to_delete = true;  // sharded: every rank's features leave the database
      int acc = 0, acc_rows = 0;
      for (size_t i = 0; i < outs.size(); i++) {
        last_msckf_.push_back(FeatDebug{it.fv[i]->featid, {outs[i].p_FinG[0], outs[i].p_FinG[1], outs[i].p_FinG[2]},
                                        outs[i].status == 2 ? 1 : outs[i].status, outs[i].chi2});
        frame_feats_.push_back({0, last_msckf_.back()});
        it.fv[i]->to_delete = true;
        for (int k = 0; k < 3; k++) it.fv[i]->p_FinG[k] = outs[i].p_FinG[k], it.fv[i]->p_FinA[k] = outs[i].p_FinA[k];
        if (outs[i].status == 0) acc++, acc_rows += outs[i].rows;
      }
      timing_.msckf_rows = acc_rows;
      timing_.msckf_cols = it.b.n_canon;
      if (it.region >= 0) {
        const double *base = d_.region_host(it.region);
        neg_check(base, N_);
        if (it.sharded) {  // the update's acceptance and rows are every rank's (the all-reduced totals)
          acc = base[N_ + 8] > 0.5 ? 1 : 0;
          timing_.msckf_rows = (int)(base[N_ + 11] + 0.5);
        }
        if (acc > 0) apply_dx(base);
      }
    } else if (it.kind == 1) {
      finish_batch(it.b, 1, outs);
      last_upd_.clear();
      int acc = 0;
      for (size_t i = 0; i < outs.size(); i++) {
        last_upd_.push_back(FeatDebug{it.fv[i]->featid, {0.0, 0.0, 0.0}, outs[i].status == 2 ? 1 : outs[i].status, outs[i].chi2});
        frame_feats_.push_back({1, last_upd_.back()});
        it.fv[i]->to_delete = true;
        if (outs[i].status == 3) slam_.at(it.fv[i]->featid)->fail_count++;
        if (outs[i].status == 0) acc++;
      }
      if (it.region >= 0) {
        const double *base = d_.region_host(it.region);
        neg_check(base, N_);
        if (acc > 0) apply_dx(base);
      }
    } else if (it.kind == 3) {
      std::vector<DFeatOut> touts;
      finish_batch(tri->b, 2, touts);
      finish_batch(it.b, 3, outs);
      last_upd_.clear();
      N_ = N0 + 3 * K;
      std::vector<int> dead;
      for (int j = 0; j < K; j++) {
        FeatP &f = it.fv[j];
        const int Ni = N0 + 3 * j, nup = 2 * it.b.feats[j].nmeas - 3;
        f->to_delete = true;
        if (touts[j].status == 1 || touts[j].status == 2) {
          last_upd_.push_back(FeatDebug{f->featid, {0.0, 0.0, 0.0}, touts[j].status, 0.0});
          frame_feats_.push_back({2, FeatDebug{f->featid, {0.0, 0.0, 0.0}, 1, 0.0}});
          dead.push_back(Ni);
          continue;
        }
        // anchor (host rule, identical to the kernel's) and the triangulated position
        f->anchor_cam_id = it.b.feats[j].anchor_cam;
        f->anchor_clone_timestamp = f->find((size_t)f->anchor_cam_id)->m.back().t;
        for (int k = 0; k < 3; k++) f->p_FinA[k] = touts[j].p_FinA[k], f->p_FinG[k] = touts[j].p_FinG[k];
        const double *base = d_.region_host(it.region + j);
        if (base[Ni + 9] > 0.5) throw HpError(UVIO_HP_E_NUMERIC, "EKFUpdate: negative covariance diagonal");
        const bool accepted = base[Ni + 8] > 0.5;
        last_upd_.push_back(FeatDebug{f->featid, {f->p_FinG[0], f->p_FinG[1], f->p_FinG[2]}, accepted ? 0 : 3,
                                      nup > 0 ? base[Ni + 3] : 0.0});
        frame_feats_.push_back({2, last_upd_.back()});
        if (!accepted) {
          dead.push_back(Ni);
          continue;
        }
        VarP lm = std::make_shared<Var>(V_LANDMARK, 3, 3);
        lm->featid = f->featid;
        lm->rep = rep_slam;
        lm->unique_cam = f->anchor_cam_id;
        lm->anchor_cam = f->anchor_cam_id;
        lm->anchor_time = f->anchor_clone_timestamp;
        const bool relr = (rep_slam == 2 || rep_slam == 4);
        lm->set_xyz(relr ? f->p_FinA : f->p_FinG, false);
        lm->set_xyz(relr ? f->p_FinA : f->p_FinG, true);
        lm->id = Ni;
        vars_.push_back(lm);
        double HLinv[9], dl[3];
        inv3_cofactor(outs[j].HfR, HLinv);  // the device's formula: identical H_Linv
        const double *resinit = base + Ni + 5;
        for (int a = 0; a < 3; a++)
          dl[a] = HLinv[3 * a] * resinit[0] + HLinv[3 * a + 1] * resinit[1] + HLinv[3 * a + 2] * resinit[2];
        lm->update(dl);
        if (nup > 0) apply_dx(base);
        slam_.insert({f->featid, lm});
      }
      marginalize_slots(dead);  // the rejected candidates' zeroed slots
    }
  }
  auto tm4 = clk::now();
  // each updater's host time: its tables + its launches; the one wait and the replay go with the last
  chain_times_[0] = t_build[0] + t_launch[0];
  chain_times_[1] = t_build[1] + t_launch[1];
  chain_times_[2] = t_build[2] + t_launch[2] + secs(tw, tm4);
  timing_.chain_wait = secs(tw, tm4);
  (void)tm3;
  return 0;
}

}  // namespace uvhp
