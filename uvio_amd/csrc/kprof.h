// Live per-launch device timing of the kernels the benchmark prices against a roofline: HIP event
// pairs recorded on the library stream around each launch (or launch chain) of a class, harvested
// without blocking once they have completed, accumulated per class together with the algorithmic FP64
// FLOPs / bytes the caller credits for those launches (SURVEY.md §8(d) formulas).
// Off by default (uvio_hp_set_kernel_timing); off, every begin/end is one branch.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace uvhp {

enum KClass {
  KC_FEATURE = 0,  // k_feature: triangulation + LM, Jacobians, left-nullspace reflections
  KC_CHI2,         // k_gemm_HPg(_tiled) + k_chi2: batched chi2 gate
  KC_GRAM,         // k_gram / k_gram_mfma: the compression Gram [H r]^T [H r]
  KC_EKF,          // one EKFUpdate (direct or information form): every kernel of the update chain
  KC_LDL,          // k_ekf_fact: LDL^T / Cholesky (+ inverse) of the innovation covariance (inside KC_EKF)
  KC_LK,           // k_lk: pyramidal LK
  KC_PYR,          // k_hist_multi + k_pyr_pair: equalizeHist + pyramid + Scharr
  KC_FAST,         // k_fast_score + k_fast_select: grid FAST + NMS + per-cell top-k (Grider_GRID.h:108-151)
  KC_SUBPIX,       // k_subpix: cornerSubPix of the new corners (Grider_GRID.h:174)
  KC_COUNT
};

struct KProf {
  bool on = false;
  hipStream_t stream = nullptr;
  struct Pair {
    int cls;
    hipEvent_t a, b;
    long long id;
    bool closed;
  };
  long long next_id_ = 0;
  std::vector<hipEvent_t> free_;
  std::vector<Pair> pending_;
  long long launches[KC_COUNT] = {0};
  double secs[KC_COUNT] = {0}, flops[KC_COUNT] = {0}, bytes[KC_COUNT] = {0};

  ~KProf() {
    for (auto &p : pending_) hipEventDestroy(p.a), hipEventDestroy(p.b);
    for (auto e : free_) hipEventDestroy(e);
  }
  hipEvent_t ev() {
    hipEvent_t e = nullptr;
    if (!free_.empty()) {
      e = free_.back();
      free_.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
      e = nullptr;
    }
    return e;
  }
  // token for end(); -1 when off
  long long begin(int cls) {
    if (!on) return -1;
    Pair p{cls, ev(), ev(), next_id_++, false};
    if (!p.a || !p.b) return -1;
    hipEventRecord(p.a, stream);
    pending_.push_back(p);
    return p.id;
  }
  void end(long long tok) {
    if (tok < 0) return;
    for (size_t k = pending_.size(); k-- > 0;)
      if (pending_[k].id == tok) {
        hipEventRecord(pending_[k].b, stream);
        pending_[k].closed = true;
        return;
      }
  }
  void credit(int cls, double f, double b) {
    if (!on) return;
    flops[cls] += f;
    bytes[cls] += b;
  }
  // harvest completed pairs (in order: a later pair cannot complete before an earlier one on one stream);
  // block = true after a stream synchronization (everything recorded has completed)
  void harvest(bool block) {
    size_t k = 0;
    for (; k < pending_.size(); k++) {
      Pair &p = pending_[k];
      if (!p.closed || (!block && hipEventQuery(p.b) != hipSuccess)) break;
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
        launches[p.cls]++;
        secs[p.cls] += 1e-3 * ms;
      } else {
        (void)hipGetLastError();
      }
      free_.push_back(p.a);
      free_.push_back(p.b);
    }
    pending_.erase(pending_.begin(), pending_.begin() + k);
  }
};

// RAII launch bracket
struct KScope {
  KProf *kp;
  long long tok;
  KScope(KProf *k, int cls) : kp(k), tok(k ? k->begin(cls) : -1) {}
  ~KScope() {
    if (kp) kp->end(tok);
  }
};

}  // namespace uvhp
