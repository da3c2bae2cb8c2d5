// Host orchestration of the MI355X hot path.  The host keeps the state *mean* and the variable
// bookkeeping (ids / sizes, like ov_type::Type::_id) and decides what to update; every operation on
// the covariance P runs on the device, where P stays resident for the whole run.
//
// Reference surfaces mirrored: ov_msckf::VioManager (VioManager.cpp:50-651),
// uvio::UVioManager (UVioManager.cpp:26-344), Propagator (Propagator.cpp:33-1015),
// StateHelper (StateHelper.cpp:36-645), UpdaterMSCKF/SLAM (UpdaterMSCKF.cpp, UpdaterSLAM.cpp),
// UpdaterUWB (UpdaterUWB.cpp), FeatureDatabase (FeatureDatabase.cpp).
#pragma once
#include <chrono>
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "hp_common.h"
#include "hprof.h"
#include "kernels.h"
#include "pool.h"
#include "tracker.h"

namespace uvhp {

enum VKind { V_IMU = 0, V_VEC = 1, V_QUAT = 2, V_POSE = 3, V_LANDMARK = 4, V_ANCHOR = 5 };

// ov_type::Type bookkeeping + value / first estimate
struct Var {
  VKind kind;
  int id = -1, size = 0, vlen = 0;
  double val[16] = {0}, fej[16] = {0};
  // landmark
  size_t featid = 0;
  int rep = 0, anchor_cam = -1, unique_cam = -1, fail_count = 0;
  double anchor_time = -1;
  bool should_marg = false;
  // uwb anchor
  uint64_t anchor_id = 0;
  bool fixed = false;
  Var(VKind k, int sz, int vl) : kind(k), size(sz), vlen(vl) {}
  void update(const double *dx);  // Type::update family (JPLQuat.h:114, IMU.h:78, Vec.h:55, ...)
  void xyz(bool fej_, double *out) const;          // Landmark::get_xyz (Landmark.cpp:26)
  void set_xyz(const double *p, bool fej_);        // Landmark::set_from_xyz (Landmark.cpp:65)
};
using VarP = std::shared_ptr<Var>;

// One camera's measurements of a feature (Feature::uvs / uvs_norm / timestamps of that camera,
// Feature.h:39-96), stored together
struct FeatMeas {
  float u, v, un, vn;
  double t;
};
// One camera's measurements in time order.  Trimming the oldest ones (FeatureDatabase::cleanup_measurements,
// every frame, over every feature of the database) only advances a start offset -- the storage is compacted
// once the dead prefix outgrows the live part -- so the per-frame cleanup touches no measurement data.
struct MeasList {
  std::vector<FeatMeas> v;
  size_t b = 0;         // first live entry
  bool sorted = true;   // live entries in non-decreasing time (every in-order stream); the time searches
                        // (contains / drop_through) fall back to the reference's linear scans otherwise
  double tf = 0, tl = 0;  // times of the first and the last live entry (valid when not empty): the selection
                          // scans over every feature decide from these without touching the storage
  using iterator = std::vector<FeatMeas>::iterator;
  using const_iterator = std::vector<FeatMeas>::const_iterator;
  size_t size() const { return v.size() - b; }
  bool empty() const { return v.size() == b; }
  FeatMeas &operator[](size_t i) { return v[b + i]; }
  const FeatMeas &operator[](size_t i) const { return v[b + i]; }
  FeatMeas &back() { return v.back(); }
  const FeatMeas &back() const { return v.back(); }
  const FeatMeas &front() const { return v[b]; }
  iterator begin() { return v.begin() + (std::ptrdiff_t)b; }
  iterator end() { return v.end(); }
  const_iterator begin() const { return v.begin() + (std::ptrdiff_t)b; }
  const_iterator end() const { return v.end(); }
  double last_t() const { return tl; }
  void push_back(const FeatMeas &x) {
    if (v.size() == b)
      tf = x.t;
    else if (x.t < tl)
      sorted = false;
    v.push_back(x);
    tl = x.t;
  }
  // a live entry at time t (FeatureDatabase::features_containing's std::find, FeatureDatabase.cpp:169-208)
  bool contains(double t) const {
    if (sorted) {
      if (empty() || t < tf || t > tl) return false;
      if (t == tf || t == tl) return true;
      auto it = std::lower_bound(begin(), end(), t, [](const FeatMeas &x, double tt) { return x.t < tt; });
      return it != end() && it->t == t;
    }
    for (auto it = begin(); it != end(); ++it)
      if (it->t == t) return true;
    return false;
  }
  // remove every live entry at or before t (Feature::clean_older_measurements, Feature.cpp:85-104)
  void drop_through(double t) {
    if (sorted) {
      auto it = std::upper_bound(begin(), end(), t, [](double tt, const FeatMeas &x) { return tt < x.t; });
      drop_front((size_t)(it - begin()));
      return;
    }
    size_t w = b;
    for (size_t i = b; i < v.size(); i++)
      if (!(v[i].t <= t)) v[w++] = v[i];
    v.resize(w);
    if (v.size() == b) clear();
    recache();
  }
  void recache() {
    if (v.size() > b) tf = v[b].t, tl = v.back().t;
  }
  void clear() {
    v.clear();
    b = 0;
    sorted = true;
  }
  iterator erase(iterator first, iterator last) {  // (callers may have rewritten entries through iterators)
    auto r = v.erase(first, last);
    recache();
    return r;
  }
  void drop_front(size_t k) {  // remove the k oldest live entries
    if (k == 0) return;
    b += k;
    if (b == v.size()) {
      clear();
    } else if (b > 32 && 2 * b > v.size()) {
      v.erase(v.begin(), v.begin() + (std::ptrdiff_t)b);
      b = 0;
    }
    recache();
  }
  void keep_if_valid(const std::vector<double> &valid);  // keep the entries whose time is in `valid` (sorted)
};
struct CamTrack {
  size_t cam;
  MeasList m;
};
// A feature's per-camera tracks, stored in the feature object (no separate allocation: a scan over every
// feature of the database touches one object per feature), in the reference's iteration order (below)
struct TrackSet {
  CamTrack t[UVIO_HP_MAX_CAMS];
  int n = 0;
  CamTrack *begin() { return t; }
  CamTrack *end() { return t + n; }
  const CamTrack *begin() const { return t; }
  const CamTrack *end() const { return t + n; }
  size_t size() const { return (size_t)n; }
  bool empty() const { return n == 0; }
  CamTrack &front() { return t[0]; }
  CamTrack &insert_front(size_t cam) {
    if (n >= UVIO_HP_MAX_CAMS) throw std::runtime_error("feature observed by more than UVIO_HP_MAX_CAMS cameras");
    // the first unused slot moves to the front: its storage may have been reserved ahead (Engine's feature stock)
    CamTrack spare = std::move(t[n]);
    for (int i = n; i > 0; i--) t[i] = std::move(t[i - 1]);
    t[0] = std::move(spare);
    t[0].cam = cam;
    t[0].m.clear();  // (keeps the capacity)
    n++;
    return t[0];
  }
};
// capacity a new track reserves: one measurement per clone of the window and a few spare (a capacity hint
// only, set from max_clone_size by the engine): the per-frame appends then do not reallocate as they grow
inline std::atomic<int> g_track_reserve{0};

struct Feature {
  size_t featid = 0;
  bool to_delete = false;
  bool held = false;     // read by this frame's update chain: trimmed after the chain, not during it
  size_t dense_idx = 0;  // slot in Engine::dense_
  // Per camera, in the iteration order of the reference's unordered_map<size_t, vector<...>> members:
  // with libstdc++ and at most UVIO_HP_MAX_CAMS small integer keys every key sits in its own bucket and
  // a new key is linked at the list front, so iteration runs in reverse first-insertion order
  // (tests/test_oracle.py pins this) -- a camera's first measurement inserts its track at the front.
  TrackSet tracks;
  int anchor_cam_id = -1;
  double anchor_clone_timestamp = -1;
  double p_FinA[3] = {0, 0, 0}, p_FinG[3] = {0, 0, 0};
  CamTrack &track(size_t cam) {
    for (auto &c : tracks)
      if (c.cam == cam) return c;
    CamTrack &c = tracks.insert_front(cam);
    if (const int r = g_track_reserve.load(std::memory_order_relaxed)) c.m.v.reserve((size_t)r);
    return c;
  }
  const CamTrack *find(size_t cam) const {
    for (auto &c : tracks)
      if (c.cam == cam) return &c;
    return nullptr;
  }
  void clean_old_measurements(const std::vector<double> &valid);  // valid: ascending
  void clean_older_measurements(double t);
  int count() const {
    int c = 0;
    for (auto &p : tracks) c += (int)p.m.size();
    return c;
  }
};
using FeatP = std::shared_ptr<Feature>;

// The feature database's map nodes come from bump-allocated 64 KB slabs (a slab is freed once its last node
// is): nodes inserted one after another sit next to each other, and since a new key of this workload lands
// in an empty bucket, which libstdc++ links at the front of its node list, the map's iteration order is
// mostly reverse insertion order -- the selection's walk over every feature (VioManager.cpp:366-392) then
// reads memory in a descending stream instead of one cache miss per node.  The iteration order itself
// depends only on the keys, the bucket policy and the operation sequence, not on where the nodes live.
class NodeSlabs {
 public:
  static constexpr size_t kSlab = size_t(1) << 16;
  NodeSlabs() = default;
  NodeSlabs(const NodeSlabs &) = delete;
  NodeSlabs &operator=(const NodeSlabs &) = delete;
  ~NodeSlabs() {
    if (cur_) std::free(cur_);
  }
  void *alloc(size_t sz) {
    sz = (sz + 15) & ~size_t(15);
    if (!cur_ || cur_->used + sz > kSlab) next_slab();
    void *p = reinterpret_cast<char *>(cur_) + cur_->used;
    cur_->used += sz;
    cur_->live++;
    return p;
  }
  void release(void *p) {
    Slab *s = reinterpret_cast<Slab *>(reinterpret_cast<uintptr_t>(p) & ~(kSlab - 1));
    if (--s->live == 0 && s != cur_) std::free(s);
  }

 private:
  struct Slab {
    size_t used, live;
  };
  static constexpr size_t kHeader = 64;
  Slab *cur_ = nullptr;
  void next_slab() {
    Slab *old = cur_;
    void *m = std::aligned_alloc(kSlab, kSlab);
    if (!m) throw std::bad_alloc();
    cur_ = static_cast<Slab *>(m);
    cur_->used = kHeader;
    cur_->live = 0;
    if (old && old->live == 0) std::free(old);
  }
};
// single-object allocations (the map's nodes) from the slabs, arrays (the bucket array) from operator new
template <class T>
struct SlabAlloc {
  using value_type = T;
  NodeSlabs *s;
  explicit SlabAlloc(NodeSlabs *s_) : s(s_) {}
  template <class U>
  SlabAlloc(const SlabAlloc<U> &o) : s(o.s) {}
  T *allocate(size_t n) {
    if (n == 1 && sizeof(T) <= 256) return static_cast<T *>(s->alloc(sizeof(T)));
    return std::allocator<T>().allocate(n);
  }
  void deallocate(T *p, size_t n) {
    if (n == 1 && sizeof(T) <= 256)
      s->release(p);
    else
      std::allocator<T>().deallocate(p, n);
  }
  template <class U>
  bool operator==(const SlabAlloc<U> &o) const { return s == o.s; }
  template <class U>
  bool operator!=(const SlabAlloc<U> &o) const { return s != o.s; }
};
// clone time -> slot of a batch's clone table (built in time order): a sorted array searched by bisection
// (add_feature looks up every measurement's clone twice; a std::map node chase per lookup was most of the
// MSCKF batch build at cfg4 / cfg5)
struct SlotTable {
  std::vector<double> t;
  void clear() { t.clear(); }
  void push(double x) { t.push_back(x); }  // ascending
  int find(double x) const {
    auto it = std::lower_bound(t.begin(), t.end(), x);
    return (it != t.end() && *it == x) ? (int)(it - t.begin()) : -1;
  }
  int at(double x) const {
    const int s = find(x);
    if (s < 0) throw std::out_of_range("measurement time is not a clone time");
    return s;
  }
};
using DbMap = std::unordered_map<size_t, FeatP, std::hash<size_t>, std::equal_to<size_t>,
                                 SlabAlloc<std::pair<const size_t, FeatP>>>;

// Feature-sharded MSCKF update across replicas.  Every rank holds the same filter; the
// features of an update are split into contiguous row-balanced chunks, each rank linearizes, gates and
// forms the Gram of its own chunk, the (n+1)^2 information blocks are all-reduced (RCCL on the library's
// stream, or a host callback), and every rank applies the identical information-form update.
struct ShardComm {
  bool enabled = false;
  int rank = 0, world = 1;
  int min_features = 1;              // updates with fewer features run unsharded on every rank
  void *nccl = nullptr;              // ncclComm_t (RCCL)
  uvio_hp_allreduce_fn host_fn = nullptr;
  void *host_user = nullptr;
};

// contiguous chunks of `rows` balanced by their sum: bounds[r] .. bounds[r+1] is rank r's range
void shard_partition(const int *rows, int n, int world, int *bounds);
// RCCL through dlopen (no link-time dependency; reuses the copy PyTorch already loaded, if any)
int rccl_unique_id(uint8_t id[128], std::string *err);
void *rccl_comm_init(int rank, int world, const uint8_t id[128]);
void rccl_allreduce_sum(void *comm, double *buf, size_t count, hipStream_t s);
void rccl_comm_destroy(void *comm);

struct ImuSample {
  double t, wm[3], am[3];
};

// Device-resident buffers (allocated once at create, sized from the config)
struct DeviceBufs {
  hipStream_t stream = nullptr;
  int ldp = 0;               // P capacity / leading dimension
  double *P = nullptr, *P2 = nullptr;
  double *T = nullptr;       // propagation scratch (ldp x 64)
  double *Phi = nullptr, *Q = nullptr, *dnc = nullptr;
  int *iold = nullptr;
  // update batch
  int max_feat = 0, max_meas_total = 0, max_vars_total = 0, max_rows = 0, ldh = 0, max_ncol = 0;
  DFeat *feats = nullptr;
  DMeas *meas = nullptr;
  DVar *vars = nullptr;
  DClone *clones = nullptr;
  DCam *cams = nullptr;
  DFeatOut *fout = nullptr;
  double *chi2 = nullptr;
  double *H = nullptr;       // H_all (max_rows x ldh)
  double *Tall = nullptr;    // H_all P_can (max_rows x ldh), chi2 gate
  double *chi2S = nullptr;   // per-feature S of the large chi2 gates (launch_chi2_batch grows it)
  size_t chi2S_cap = 0;      // doubles
  double *partials = nullptr;
  double *R = nullptr;       // compressed (ncol x ncol, + global Cholesky scratch)
  int *hidx = nullptr;
  EkfScratch ekf{};
  // pinned host staging
  void *pin = nullptr;
  size_t pin_bytes = 0;
  double *dx_host = nullptr;
  int *neg_host = nullptr;
  DFeatOut *fout_host = nullptr;
  double *aux_host = nullptr;  // 16 host-only landing slots (delayed-init residual, shard totals)
  int fout_pending = 0;        // feature results not yet copied: they ride along with the next readback
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // feature-kernel timing
  // upload staging ring: small host tables of one launch group are packed into pinned memory and sent
  // with ONE copy (stage / stage_flush); the kernels read the device copy directly
  char *stg_h = nullptr, *stg_d = nullptr;
  size_t stg_cap = 0, stg_used = 0, stg_flushed = 0;
  long long stg_epoch = 0;  // ring restarts so far (a reservation must not outlive one: run_batch checks)
  // [negative-diagonal count (8 B) | dx (cap + 15) | feature results (max features)], mirrored in pinned
  // memory at neg_host / dx_host / fout_host: an update's dx and its batch's results come back in ONE copy
  double *dxneg = nullptr;
  size_t dx_bytes = 0;  // bytes of [count | dx] (the offset of the feature results)
  // feature sharding: the all-reduced [G upper triangle (max_ncol^2) | accepted features | accepted rows]
  double *shard = nullptr, *shard_host = nullptr;
  int *acc = nullptr;       // accepted features of the last update batch (gates its P update)
  // information-form prefactor on a side stream (Engine::info_prefactor): P_II's factor and V while the
  // feature group runs; its column map in a dedicated device buffer (pinned mirror), the run it belongs to
  hipStream_t aux = nullptr;
  hipEvent_t ev_aux_in = nullptr, ev_aux_out = nullptr;
  // staging uploads run on their own stream (the DMA transfer overlaps the kernels already queued on `stream`,
  // which waits on ev_copy before its next launch)
  hipStream_t copy = nullptr;
  hipEvent_t ev_copy = nullptr;
  // the prefactor's column maps: kPreSlots pinned / device slots used in turn, each freed by its copy's event
  // (a slot is reused kPreSlots prefactors later, so the host never waits on the one just enqueued)
  static constexpr int kPreSlots = 8;
  int *hidx_pre = nullptr, *hidx_pre_h = nullptr;
  hipEvent_t ev_pre[kPreSlots] = {};
  int pre_slot = 0;
  std::vector<int> pre_hidx;  // columns of the pending prefactor (empty: none)
  int pre_N = -1;
  long long pre_epoch = -1;  // Engine::p_epoch_ when the prefactor was enqueued
  // delayed-initialization chain (Engine::slam_delayed_init): per candidate one region of chain_stride doubles
  // [dx (N) | chi2, accepted | init residual (3) | accepted, negative diagonals], chain_k candidates per chain,
  // mirrored in pinned memory
  // The frame chain's per-update regions sit right in front of dxneg (region r at dxneg - (r + 1) stride), and
  // chain_host mirrors [regions | dx block | fout] in pinned memory, so the chain's regions and every batch's
  // per-feature results come back in ONE copy (chain_results_copy)
  double *chain = nullptr, *chain_host = nullptr;  // the allocations: [chain_k regions][dx block][fout]
  int chain_k = 0;
  size_t chain_stride = 0;
  double *region_dev(int r) const { return dxneg - (size_t)(r + 1) * chain_stride; }
  const double *region_host(int r) const { return (const double *)neg_host - (size_t)(r + 1) * chain_stride; }
  int fout_cap = 0;            // per-feature result slots in fout / fout_host (one frame chain's batches)
  char *frame = nullptr;       // the frame chain's device state: clone / camera tables, pose values, mirror
  size_t frame_bytes = 0;
  // the chained UWB ranges of one message (Engine::uwb_update_message): per range a region [accepted, negative
  // diagonals, chi2, S | dx] of uwb_stride doubles (pinned mirror uwb_host) and its row h (16 doubles)
  double *uwb_reg = nullptr, *uwb_host = nullptr, *uwb_h = nullptr;
  size_t uwb_stride = 0;
};

// the per-feature measurement / variable tables of one feature in the reference iteration order (engine_update.cpp)
class Engine;
void add_feature(Engine *, const FeatP &f, int mode, int rep, const uvio_hp_options_t &o, const std::vector<DCam> &cams,
                 const SlotTable &slot_of_time, const std::vector<DClone> &clones, std::vector<DFeat> &feats,
                 std::vector<DMeas> &meas, std::vector<DVar> &vars, int &rows, const Var *landmark, int landmark_canon);
// algorithmic FP64 FLOPs / bytes of one EKFUpdate (engine_state.cpp)
double ekf_flops(double N, double n, double r);
double ekf_bytes(double N, double n, double r);

class Engine {
 public:
  explicit Engine(const uvio_hp_options_t &o, int device);
  ~Engine();

  void initialize_with_gt(const double x[17]);
  void feed_imu(double t, const double wm[3], const double am[3]);
  int feed_simulation(double t, int ncam, const int *cam_ids, const int *counts, const uint64_t *ids, const float *uv);
  int feed_camera(double t, int ncam, const int *cam_ids, const uint8_t *const *imgs, const int *strides,
                  const uint8_t *const *masks, bool device_imgs);
  int feed_uwb(double t, int n, const uint64_t *ids, const double *ranges);
  Tracker *tracker() { return tracker_.get(); }
  int init_anchors(int n, const uvio_hp_anchor_t *a);
  // HIP's current device is per host thread: every C-ABI entry binds the engine's device first, so a handle
  // created for GPU k may be driven from any thread
  int device() const { return device_; }

  // getters
  bool initialized() const { return is_initialized_; }
  double timestamp() const { return timestamp_; }
  const Var &imu() const { return *imu_; }
  int cov_dim() const { return N_; }
  void get_cov(double *out, int ld);
  int state_vector(double *out, int cap, int *meta, int meta_cap, int *nvars, bool fej = false);
  uvio_hp_timing_t timing() const { return timing_; }
  std::vector<double> clone_times() const;

  // live kernel timing of the roofline classes (kprof.h)
  // period 0: off; k: the camera frames whose index is a multiple of k are timed (events cost host time)
  void set_kernel_timing(int period) {
    ktime_period_ = period;
    kprof_.on = period > 0 && frames_ % period == 0;
  }
  void kernel_stats(bool flush, uvio_hp_kstat_t *out, int cap, int *n);

  // feature sharding
  void shard_init_rccl(int rank, int world, const uint8_t id[128], int min_features);
  void shard_init_host(int rank, int world, uvio_hp_allreduce_fn fn, void *user, int min_features);

  // standalone kernel-level entry points (parity tests)
  static int ekf_update_standalone(double *P, int N, const int *H_index, int n, const double *H, int r, const double *res,
                                   double sigma2, double *dx_out, bool compress = false);
  static int compress_standalone(const double *A, int m, int n, double *R_out);
  static int undistort_standalone(int model, const double cam[8], int n, const float *uv, float *uvn, uint8_t *amb);
  static int grid_order_standalone(const uint8_t *resp, const int *off, int ncell, int kmax, int depth,
                                   int *arrangement, int *top);

 private:
  uvio_hp_options_t o_;
  int device_;
  DeviceBufs d_;
  // ---- state (host mean + bookkeeping) ----
  double timestamp_ = -1;
  VarP imu_, calib_dt_, dw_, da_, tg_, qg_, qa_, p_IinU_;
  std::map<double, VarP> clones_;
  std::unordered_map<size_t, VarP> slam_;
  std::unordered_map<size_t, VarP> calib_pose_, calib_intr_;
  std::unordered_map<size_t, VarP> anchors_;
  CamParams cams_[UVIO_HP_MAX_CAMS];
  std::vector<VarP> vars_;
  int N_ = 0;
  // bumped by every write of P (propagation, clone, marginalization, EKF updates, initialization, uploads):
  // a side-stream prefactor is only used when P is unchanged since it was enqueued
  long long p_epoch_ = 0;
  double early_prop_s_ = 0.0;  // host time of a propagation run inside the tracker's wait (feed_camera)
  // ---- propagator ----
  std::mutex imu_mtx_;
  std::vector<ImuSample> imu_data_;
  bool have_last_prop_time_offset_ = false;
  double last_prop_time_offset_ = 0;
  // ---- KLT front-end (created on the first camera feed) ----
  std::unique_ptr<Tracker> tracker_;
  // ---- feature database (TrackSIM's / TrackKLT's) ----
  NodeSlabs db_nodes_;  // (declared before db_: it outlives the map's nodes)
  DbMap db_{SlabAlloc<std::pair<const size_t, FeatP>>(&db_nodes_)};
  // every feature of db_ in one contiguous array (order unrelated to db_'s; Feature::dense_idx is the slot)
  // for the walks whose outcome does not depend on the order (the per-frame measurement cleanup), which then
  // need not chase the hash map's nodes; db_insert / db_erase keep the two in step
  std::vector<Feature *> dense_;
  using DbIt = DbMap::iterator;
  DbIt db_insert(size_t id, const FeatP &f) {
    f->dense_idx = dense_.size();
    dense_.push_back(f.get());
    return db_.emplace(id, f).first;
  }
  DbIt db_erase(DbIt it) {
    const size_t i = it->second->dense_idx;
    dense_[i] = dense_.back();
    dense_[i]->dense_idx = i;
    dense_.pop_back();
    return db_.erase(it);
  }
  size_t currid_;
  // default-constructed features made while the host waits for the device chain (refill_feature_stock), so
  // that a feed's inserts -- sequential, in observation order -- do not allocate and clear each new object
  std::vector<FeatP> feat_stock_;
  size_t stock_target_ = 0;  // 1.5 x the last feed's new features
  FeatP new_feature(size_t id) {
    FeatP f;
    if (!feat_stock_.empty()) {
      f = std::move(feat_stock_.back());
      feat_stock_.pop_back();
    } else {
      f = std::make_shared<Feature>();
    }
    f->featid = id;
    return f;
  }
  // each stocked feature also gets the storage of its first track reserved (every new feature has one; the
  // feed's first append to it then does not allocate; reserving all cameras' tracks cost more than it saved
  // at cfg5, where a feature is seen by ~2.6 of 4 cameras)
  void refill_feature_stock() {
    const int r = g_track_reserve.load(std::memory_order_relaxed);
    while (feat_stock_.size() < stock_target_) {
      FeatP f = std::make_shared<Feature>();
      if (r > 0) f->tracks.t[0].m.v.reserve((size_t)r);
      feat_stock_.push_back(std::move(f));
    }
  }
  // ---- manager ----
  bool is_initialized_ = false;
  // VioManager::thread_init_success (VioManager.h:226): the initializer succeeded on an earlier frame; the
  // manager reports initialized only on the next camera frame (VioManagerHelper.cpp:91-93, 187)
  bool init_success_ = false;
  // inside feed_camera (the update chain then runs the tracker's next detection ahead, Tracker::predetect);
  // UVIO_HP_NO_PREDETECT=1 turns that off (A/B runs)
  bool camera_frame_ = false, predetect_on_ = true;
  double startup_time_ = -1, distance_ = 0, timelastupdate_ = -1;
  bool anchors_initialized_ = false;
  std::map<double, std::unordered_map<size_t, double>> past_uwb_;
  uvio_hp_timing_t timing_{};
  std::vector<double> chi2_table_;
  ShardComm shard_;
  WorkPool pool_;
  std::vector<FeatP> pending_delete_;  // features handed to an updater this frame (cleanup candidates)
  // host work that update_frame runs while the device executes the chain (set by the caller, cleared by the run)
  std::function<void()> chain_overlap_;
  // FeatureDatabase::cleanup_measurements(t) over the database's features, skipping the held ones if asked
  void cleanup_measurements(double t, bool skip_held);
  void chain_results_copy(int nreg, int fo);
  HostProf hprof_;                     // UVIO_HP_HOST_PROF section timer (debug)
  FILE *timing_csv_ = nullptr;         // record_timing_information (VioManager.cpp:105-122)
  KProf kprof_;                        // live per-class kernel timing (uvio_hp_set_kernel_timing)
  int ktime_period_ = 0;
  long long frames_ = 0;               // camera / simulated frames fed
  void frame_begin() {
    frames_++;
    kprof_.on = ktime_period_ > 0 && frames_ % ktime_period_ == 0;
  }
  void shard_allreduce(double *dev, size_t count);
  int msckf_update_sharded(std::vector<FeatP> &fv);

 public:
  struct FeatDebug {
    size_t id;
    double p_FinG[3];
    int status;
    double chi2;
  };
  std::vector<FeatDebug> last_msckf_;
  std::vector<FeatDebug> last_upd_;  // the last SLAM update / delayed initialization, per feature
  // every updater's per-feature results of the current frame: (kind 0 MSCKF / 1 SLAM update / 2 delayed
  // initialization, result), cleared when the frame's update stage begins (lock-step parity tests)
  std::vector<std::pair<int, FeatDebug>> frame_feats_;

  // updater-level entry points (engine_api.cpp; include/uvio_hp.h "Updater-level boundary")
  enum ApiUpdater { API_MSCKF = 0, API_SLAM = 1, API_DELAYED = 2 };
  int api_set_state(const double *val, const double *fej, int len, const double *P, int N, int ld);
  int api_propagate_and_clone(double t);
  int api_update(int which, int nfeat, const uint64_t *featids, const int *meas_off, const uvio_hp_feat_meas_t *meas,
                 uvio_hp_feat_result_t *out);
  int api_change_anchors();
  int api_marginalize_slam();
  int api_marginalize_old_clone();
  int api_uwb_update_single(uint64_t anchor_id, double range, int *applied);
  // the reference routine the host was in when the last call failed (error messages)
  const char *stage() const { return stage_; }

 private:
  const char *stage_ = "";

 private:

  // covariance ops (device)
  void alloc_device();
  void upload_P_full(const std::vector<double> &Ph, int N);
  void download_P(std::vector<double> &Ph);
  void cov_propagate(int s0, int p, const std::vector<int> &iold, const std::vector<double> &Phi,
                     const std::vector<double> &Q, const std::vector<int> *rows = nullptr);
  VarP clone_imu_pose(const double *dnc, bool do_dt, const double *staged = nullptr);
  VarP add_clone_var();
  bool cov_propagate_clone(int s0, int p, const std::vector<int> &iold, const std::vector<double> &Phi,
                           const std::vector<double> &Q, bool do_dt, const double *ddnc);
  void marginalize(const VarP &v);
  // a sequence of marginalize calls as one launch (the same covariance, k_marginalize_multi)
  void marginalize_many(const std::vector<VarP> &ms);
  void check_neg_diag(const char *who);
  void info_prefactor(const std::vector<int> &hidx);
  // joins an information-form prefactor its update did not consume (an early return or an exception in
  // between): the main stream waits for it, so no later P write can overlap its reads of P
  struct PrefactorJoin {
    Engine *e;
    explicit PrefactorJoin(Engine *x) : e(x) {}
    ~PrefactorJoin() {
      if (e->d_.pre_N < 0) return;
      (void)hipStreamWaitEvent(e->d_.stream, e->d_.ev_aux_out, 0);
      e->d_.pre_hidx.clear();
      e->d_.pre_N = -1;
    }
  };
  void ekf_update_info(int nch, int n, const std::vector<int> &hidx, double sigma2,
                       const std::function<bool()> &apply = nullptr, const int *gate = nullptr,
                       const double *partials = nullptr);
  // hidx_dev: the batch's column map already on the device (staged), or nullptr to stage `hidx`;
  // pre_apply runs after the readback, before dx is applied (initialize_invertible's landmark step)
  // gate (device count, may be null): the P update is skipped on the device when it is 0; after the
  // readback `apply` decides whether dx goes to the host mean (true when absent)
  void ekf_update_rows(const double *Hdev, int ldh, int r, int n, const std::vector<int> &hidx, const double *resdev,
                       int res_stride, double sigma2, const int *hidx_dev = nullptr,
                       const std::function<bool()> &apply = nullptr, const int *gate = nullptr,
                       const double *Tdev = nullptr);  // T = H P_II of these rows (ld ldh), if the chi2 gate left it
  void apply_dx(const double *dx);
  // staging (see DeviceBufs): returns the device address the table will have after stage_flush()
  void *stage_bytes(const void *src, size_t bytes);
  // reserve staging space the caller fills in place (host address in *host); same device-address rule.
  // Fill it before the next stage / stage_reserve call (either may flush and recycle the ring).
  void *stage_reserve(size_t bytes, void **host);
  template <class T>
  T *stage(const T *src, size_t n) {
    return (T *)stage_bytes(src, sizeof(T) * n);
  }
  void stage_flush(bool on_main = false);
  // wait for the device (counted in the frame's timing: device_syncs, sync_wait)
  void dev_sync();
  bool propagation_can_precede_tracking(double t) const;
  // dx + negative-diagonal count back to the host (one copy + sync); throws on a negative diagonal
  void read_dx(const char *who);
  void initialize_invertible_host(const VarP &v, const std::vector<std::pair<int, int>> &H_order,
                                  const std::vector<double> &H_R, const std::vector<double> &H_L,
                                  const std::vector<double> &R, const std::vector<double> &res);
  void set_initial_covariance(const std::vector<double> &cov, const std::vector<VarP> &order);

  // start-up from rest (engine_init.cpp): the InertialInitializer's IMU buffer (fed until initialized,
  // VioManager.cpp:180-182), FeatureDatabase::cleanup_measurements, and the initializers
  std::vector<ImuSample> init_imu_;
  void db_cleanup_measurements(double t);
  bool static_initialize(bool wait_for_jerk, double *t_init, std::vector<double> &cov);
  bool try_to_initialize();

  // UpdaterZeroVelocity (UpdaterZeroVelocity.cpp:65-329; VioManager.cpp:160, 186-188, 294-307, 360)
  std::vector<ImuSample> zupt_imu_;
  bool zupt_have_last_off_ = false;
  double zupt_last_off_ = 0.0, last_zupt_state_timestamp_ = 0.0;
  int last_zupt_count_ = 0;
  bool did_zupt_update_ = false, has_moved_since_zupt_ = false;
  // 1: the zero-velocity update was applied (state time moved to t); 0: not
  int zupt_try_update(double t);

  // propagator (host mean + Phi/Qd, device covariance)
  std::vector<ImuSample> select_imu_readings(double t0, double t1);
  static std::vector<ImuSample> select_imu(const std::vector<ImuSample> &imu, double t0, double t1);
  void accumulate_phi(const std::vector<ImuSample> &prop, std::vector<double> &Phi, std::vector<double> &Qd, int n);
  void predict_and_compute(const ImuSample &a, const ImuSample &b, double *F, double *Qd, int n);
  void last_w(const std::vector<ImuSample> &prop, double *w);
  std::vector<int> phi_order_ids(int *n);
  int propagate_and_clone(double t);
  int propagate_uwb(double t);

  // updates
  int after_tracking(double t, const std::vector<int> &camids, std::chrono::steady_clock::time_point rT1,
                     int track_syncs = 0, double track_wait = 0.0, bool try_init = false);
  int do_feature_propagate_update(double t, const std::vector<int> &camids, std::chrono::steady_clock::time_point rT2);
  int msckf_update(std::vector<FeatP> &feats);
  void gram(int m, int ncol, int *nch);
  // VioManager::retriangulate_active_tracks on the device (engine_retri.cpp)
  struct RetriState {
    int cap = 0, obs_cap = 0, slam_cap = 0, cur = 0, nslam = 0;
    unsigned long long *keys[2] = {nullptr, nullptr};
    DRetriEntry *ent[2] = {nullptr, nullptr};
    DRetriObs *d_obs = nullptr, *h_obs = nullptr;
    DRetriSlam *d_slam = nullptr, *h_slam = nullptr;
    double *scratch = nullptr;
    hipEvent_t copied = nullptr;
    bool copy_pending = false, valid = false;
    double time = -1;
    // the frame's job as taken at the reference's point (poses, landmarks, camera models, observations in
    // frame_obs_), run by retri_flush at the next feed's tracking wait or on demand
    bool pend = false, pend_undist = false;
    double pend_t = -1;
    RetriJob pend_job{};
    std::vector<DRetriSlam> pend_sl;
    CamParams pend_cams[UVIO_HP_MAX_CAMS];
  } rt_;
  std::vector<DRetriObs> frame_obs_;  // this frame's observations (simulated feed, or the tracker's last tracks)
  void retri_alloc(int nobs, int nslam);
  void retriangulate_active_tracks(double t, const std::vector<int> &camids);
  void retri_flush();

 public:
  int get_active_tracks(double *t, uint64_t *ids, double *posinG, double *uvd, int *uvd_valid, int cap);

 private:
  int slam_update(std::vector<FeatP> &feats);
  int slam_delayed_init(std::vector<FeatP> &feats);
  int slam_change_anchors();
  int uwb_update_single(size_t anchor_id, double range);
  // UpdaterUWB::update_single for every range of one UwbData message whose anchor is known, in the message's
  // order, as one device chain with one readback; returns the number of applied updates
  int uwb_update_message(const std::vector<std::pair<size_t, double>> &ranges);
  void marginalize_slam();
  void marginalize_old_clone();
  void db_update(size_t id, double t, size_t cam, float u, float v, float un, float vn);
  double margtimestep() const {
    double t = INFINITY;
    for (auto &c : clones_)
      if (c.first < t) t = c.first;
    return t;
  }

  // batch construction for the per-feature kernel
  struct Batch {
    std::vector<DFeat> feats;
    std::vector<DMeas> meas;
    std::vector<DVar> vars;
    std::vector<DClone> clones;
    std::vector<DCam> cams;
    std::vector<int> hidx;     // canonical column -> covariance id
    const int *hidx_dev = nullptr;  // its staged device copy
    bool finished = false;          // per-feature results read back (finish_batch)
    bool evtimed = false;           // the feature group is bracketed by the ev0 / ev1 timing events
    bool chi2 = true;               // the batch chi2 kernels ran (run_batch)
    std::vector<FeatP> fptrs;
    int n_canon = 0, rows = 0, max_meas = 0, max_nf = 0;
    // large batches write their measurement / variable tables straight into the upload staging
    // (add_features_to_batch); meas / vars then stay empty and these hold the staged tables
    const DMeas *meas_dev = nullptr;
    const DVar *vars_dev = nullptr;
    size_t n_meas_dev = 0, n_vars_dev = 0;
    long long stg_epoch = -1;  // staging ring epoch of the meas / vars reservation
    size_t n_meas() const { return meas_dev ? n_meas_dev : meas.size(); }
    size_t n_vars() const { return vars_dev ? n_vars_dev : vars.size(); }
    SlotTable slot_of_time;
    int fout_off = 0;  // its per-feature results in d_.fout / d_.fout_host start here
  };
  void build_clone_cam_tables(Batch &b, bool include_landmarks);
  void add_feature_to_batch(Batch &b, const FeatP &f, int mode, int rep);
  void add_features_to_batch(Batch &b, const std::vector<FeatP> &fv, size_t lo, size_t hi, int mode, int rep);
  // wait = false: only enqueue (kernels + result readback); the caller's next device sync completes it and
  // finish_batch then fills outs
  // chi2 = false: the feature kernel only (delayed init gates on its own update factor instead)
  DBatchParams batch_params(const Batch &b, double sigma_pix_sq, double chi2_mult) const;
  // one chain of delayed initializations: fv[idx[0..]] (triangulated) linearized, initialized and updated on
  // the device one after the other, one host wait at the end
  int slam_delayed_chain(std::vector<FeatP> &fv, const std::vector<size_t> &idx, int rep, double s2);
  // the frame's UpdaterMSCKF::update, UpdaterSLAM::update chunks and delayed_init as one device chain with one
  // host wait (engine_chain.cpp)
  int update_frame(std::vector<FeatP> &msckf, std::vector<FeatP> &slam_upd, std::vector<FeatP> &delayed);
  struct ChainItem;
  double chain_times_[3] = {0, 0, 0};  // host seconds of the chain's MSCKF / SLAM / delayed-init parts
  // UVIO_HP_NO_CHAIN set when the engine is created: the updaters one after the other with their host waits
  // (A/B runs and diagnostics)
  const bool no_chain_ = std::getenv("UVIO_HP_NO_CHAIN") != nullptr;
  // 3-wide variables (zeroed landmark slots) at the given covariance offsets leave P in one compaction
  void marginalize_slots(std::vector<int> slots);
  int run_batch(Batch &b, int mode, double sigma_pix_sq, double chi2_mult, bool wait, std::vector<DFeatOut> &outs,
                bool chi2 = true);
  void finish_batch(Batch &b, int mode, std::vector<DFeatOut> &outs);
};

}  // namespace uvhp
