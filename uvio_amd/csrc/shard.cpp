// Feature-sharded MSCKF update across GPUs.
//
// The reference's UpdaterMSCKF::update (UpdaterMSCKF.cpp:58-295) linearizes every selected feature
// against one read-only state, stacks the nullspace-projected rows and compresses them
// (measurement_compress_inplace, UpdaterHelper.cpp:456-487) before one EKFUpdate.  The features are
// independent until the stack, and the compressed update depends on the stack only through its Gram
// G = [H r]^T [H r], which is a sum over features.  So with the filter replicated on every
// rank, rank r takes a contiguous row-balanced chunk of the (already sorted) feature list, runs the same
// feature kernels and Gram on it, and one all-reduce of the (n+1)^2 + 2 doubles [G | accepted | rows]
// gives every rank the full update, which each applies identically.  Over xGMI the message is ~0.5 MB at
// cfg5 (n = 242), latency-bound; the work it splits is the per-feature linearization, chi2 gate and the
// Gram over ~80k stacked rows.
//
// RCCL is reached through dlopen: the library has no link-time dependency on it, and in a process where
// PyTorch already loaded its bundled RCCL that copy is reused instead of a second one being mapped.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>

#include "engine.h"

namespace uvhp {

// ---- RCCL loader ----
namespace {
struct Rccl {
  bool tried = false;
  void *lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl &rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
  for (const char *n : names)  // an already-mapped copy first (PyTorch's)
    if ((r.lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
  for (int k = 0; !r.lib && k < 3; k++) r.lib = dlopen(names[k], RTLD_NOW | RTLD_GLOBAL);
  if (!r.lib) return r;
  r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.lib, "ncclGetUniqueId");
  r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.lib, "ncclCommInitRank");
  r.all_reduce = (decltype(r.all_reduce))dlsym(r.lib, "ncclAllReduce");
  r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.lib, "ncclCommDestroy");
  r.error_string = (decltype(r.error_string))dlsym(r.lib, "ncclGetErrorString");
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy) r.lib = nullptr;
  return r;
}

void nccl_check(ncclResult_t rc, const char *what) {
  if (rc == ncclSuccess) return;
  const char *m = rccl().error_string ? rccl().error_string(rc) : "";
  throw HpError(UVIO_HP_E_DEVICE, std::string(what) + ": " + m);
}
}  // namespace

int rccl_unique_id(uint8_t id[128], std::string *err) {
  Rccl &r = rccl();
  if (!r.lib) {
    if (err) *err = "RCCL (librccl.so.1) not found";
    return UVIO_HP_E_DEVICE;
  }
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  ncclResult_t rc = r.get_unique_id(&u);
  if (rc != ncclSuccess) {
    if (err) *err = std::string("ncclGetUniqueId: ") + (r.error_string ? r.error_string(rc) : "");
    return UVIO_HP_E_DEVICE;
  }
  std::memcpy(id, &u, 128);
  return UVIO_HP_OK;
}

void *rccl_comm_init(int rank, int world, const uint8_t id[128]) {
  Rccl &r = rccl();
  if (!r.lib) throw HpError(UVIO_HP_E_DEVICE, "RCCL (librccl.so.1) not found");
  ncclUniqueId u;
  std::memcpy(&u, id, 128);
  ncclComm_t c = nullptr;
  nccl_check(r.comm_init_rank(&c, world, u, rank), "ncclCommInitRank");
  return (void *)c;
}

void rccl_allreduce_sum(void *comm, double *buf, size_t count, hipStream_t s) {
  nccl_check(rccl().all_reduce(buf, buf, count, ncclFloat64, ncclSum, (ncclComm_t)comm, s), "ncclAllReduce");
}

void rccl_comm_destroy(void *comm) {
  if (comm && rccl().comm_destroy) rccl().comm_destroy((ncclComm_t)comm);
}

// ---- partition ----
// Feature i (in the order the selection sorted them, VioManager.cpp:509-524) goes to the rank whose
// share of the total rows holds the midpoint of its own rows: rank floor(world (pre_i + rows_i / 2) / total).
// Contiguous, monotone, and each chunk within half a feature of total / world.
void shard_partition(const int *rows, int n, int world, int *bounds) {
  long long total = 0;
  for (int i = 0; i < n; i++) total += rows[i];
  bounds[0] = 0;
  long long pre = 0;
  int i = 0;
  for (int r = 1; r < world; r++) {
    while (i < n && (2 * pre + rows[i]) * world < 2LL * r * total) pre += rows[i++];
    bounds[r] = i;
  }
  bounds[world] = n;
}

// ---- engine ----
void Engine::shard_init_rccl(int rank, int world, const uint8_t id[128], int min_features) {
  if (world < 1 || rank < 0 || rank >= world) throw HpError(UVIO_HP_E_ARG, "bad rank / world");
  HP_HIP(hipSetDevice(device_));
  if (shard_.nccl) rccl_comm_destroy(shard_.nccl);
  shard_ = ShardComm{};
  shard_.nccl = rccl_comm_init(rank, world, id);
  shard_.rank = rank;
  shard_.world = world;
  shard_.min_features = std::max(min_features, 1);
  shard_.enabled = true;
}

void Engine::shard_init_host(int rank, int world, uvio_hp_allreduce_fn fn, void *user, int min_features) {
  if (world < 1 || rank < 0 || rank >= world || !fn) throw HpError(UVIO_HP_E_ARG, "bad rank / world / callback");
  if (shard_.nccl) rccl_comm_destroy(shard_.nccl);
  shard_ = ShardComm{};
  if (!d_.shard_host)
    HP_HIP(hipHostMalloc((void **)&d_.shard_host, sizeof(double) * ((size_t)d_.max_ncol * d_.max_ncol + 2),
                         hipHostMallocDefault));
  shard_.host_fn = fn;
  shard_.host_user = user;
  shard_.rank = rank;
  shard_.world = world;
  shard_.min_features = std::max(min_features, 1);
  shard_.enabled = true;
}

void Engine::shard_allreduce(double *dev, size_t count) {
  if (shard_.nccl) {
    rccl_allreduce_sum(shard_.nccl, dev, count, d_.stream);  // enqueued: no host wait
    return;
  }
  HP_HIP(hipMemcpyAsync(d_.shard_host, dev, sizeof(double) * count, hipMemcpyDeviceToHost, d_.stream));
  dev_sync();
  if (shard_.host_fn(d_.shard_host, count, shard_.host_user) != 0)
    throw HpError(UVIO_HP_E_DEVICE, "feature-shard all-reduce callback failed");
  HP_HIP(hipMemcpyAsync(dev, d_.shard_host, sizeof(double) * count, hipMemcpyHostToDevice, d_.stream));
}

// UpdaterMSCKF::update with the features split across ranks.  fv: the features after the reference's
// clean_old_measurements / count filter (identical on every rank); this rank linearizes its chunk.
int Engine::msckf_update_sharded(std::vector<FeatP> &fv) {
  const int F = (int)fv.size();
  std::vector<int> rows(F), bounds(shard_.world + 1);
  for (int i = 0; i < F; i++) rows[i] = 2 * fv[i]->count() - 3;
  shard_partition(rows.data(), F, shard_.world, bounds.data());
  const int lo = bounds[shard_.rank], hi = bounds[shard_.rank + 1];
  Batch b;
  build_clone_cam_tables(b, false);
  add_features_to_batch(b, fv, (size_t)lo, (size_t)hi, 0, o_.feat_rep_msckf);
  // the information-form update always follows: its P_II factor and V run beside this rank's feature
  // group and the all-reduce (Engine::info_prefactor)
  PrefactorJoin pj(this);
  info_prefactor(b.hidx);
  std::vector<DFeatOut> outs;
  const double s2 = o_.msckf_sigma_pix * o_.msckf_sigma_pix;
  const int m = run_batch(b, 0, s2, o_.msckf_chi2_multipler, false, outs);
  const int n = b.n_canon, ncol = n + 1;
  int nch = 0;
  if (m > 0) gram(m, ncol, &nch);
  const size_t count = (size_t)ncol * ncol + 2;
  launch_shard_pack(d_.stream, d_.partials, nch, ncol, d_.fout, (int)b.feats.size(), d_.acc, d_.shard);
  shard_allreduce(d_.shard, count);
  launch_shard_unpack(d_.stream, d_.shard, ncol, d_.acc);
  double *tot_host = d_.aux_host + 4;  // [accepted, rows] of all ranks, read back with dx
  HP_HIP(hipMemcpyAsync(tot_host, d_.shard + (size_t)ncol * ncol, 2 * sizeof(double), hipMemcpyDeviceToHost,
                        d_.stream));
  auto results = [&]() {
    finish_batch(b, 0, outs);
    for (size_t i = 0; i < outs.size(); i++) {
      const FeatP &f = fv[lo + i];
      last_msckf_.push_back(FeatDebug{f->featid, {outs[i].p_FinG[0], outs[i].p_FinG[1], outs[i].p_FinG[2]},
                                      outs[i].status == 2 ? 1 : outs[i].status, outs[i].chi2});
      frame_feats_.push_back({0, last_msckf_.back()});
      for (int k = 0; k < 3; k++) f->p_FinG[k] = outs[i].p_FinG[k], f->p_FinA[k] = outs[i].p_FinA[k];
    }
    for (auto &f : fv) f->to_delete = true;
    timing_.msckf_rows = (int)(tot_host[1] + 0.5);
    timing_.msckf_cols = n;
    return tot_host[0] > 0.5;
  };
  ekf_update_info(1, n, b.hidx, s2, results, d_.acc, d_.shard);
  return 0;
}

}  // namespace uvhp
