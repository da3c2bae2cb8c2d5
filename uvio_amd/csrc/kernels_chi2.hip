// Batched chi2 gate for a linearized update batch (UpdaterMSCKF.cpp:209-234, UpdaterSLAM.cpp:207-226
// and :370-391, StateHelper::initialize :451-470).
//
// Every feature's projected rows [Hhat_f | r_f] sit in H_all over the batch's canonical columns, and
// every feature's P_marg is a principal block of the same canonical covariance P_can = P[hidx, hidx]
// (zero columns of Hhat_f drop out).  So
//     T = H_all P_can                    one FP64 GEMM over the whole batch (m x n x n, MFMA, P_can
//                                        gathered from P in the operand loads),
//     S_f = T_f Hhat_f^T + s2 I          per feature, R_f x R_f,
// and the per-feature work is only the small S_f and its factorization.  One workgroup per feature
// stages T_f and Hhat_f in LDS, forms the lower triangle of [S_f ; r_f^T], runs the one-barrier-per-
// column LDL^T of dense_lds.h (the appended residual row becomes z = L_unit^-1 r), and
// chi2 = sum_k z_k^2 / d_k = r^T S^-1 r.  Rejected MSCKF / SLAM features get their rows zeroed so the
// batch Gram (compression) and the direct EKF see only accepted rows.
#include "dense_lds.h"
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace uvhp {

// T (m x n, ld ldt) = H (m x n, ld ldh) * P[hidx, hidx] with the covariance gather fused into the
// operand loads.  One 64-lane workgroup per 16x16 tile of T, v_mfma_f64_16x16x4_f64 over K = n.  The
// batches are small (cfg2: 486 x 100), so the kernel is load-latency bound: the column map is staged in
// LDS once (the P gather then needs no dependent hidx load), and K runs in 32-wide steps whose 16 operand
// loads are issued one step ahead of the step's 8 MFMAs (register double buffer).  The tiles run on two
// XCDs in contiguous row-block ranges (below), so P_can is fetched into two L2s instead of eight and each H
// row slab once (cfg2: 2.13 -> 0.75 MB per launch, profiles/r02u_pmc_traffic_cfg2.json).  The accumulation
// order over k is the plain ascending one of 4-wide MFMA steps, whatever the step width.
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int HPS = 32;  // K per load step
__global__ void __launch_bounds__(64) k_gemm_HPg(const double *__restrict__ H, int m, int n, int ldh,
                                                 const double *__restrict__ P, int ldp, const int *__restrict__ hidx,
                                                 double *__restrict__ T, int ldt, int *zero) {
  extern __shared__ int sh_hidx[];
  const int l = threadIdx.x, r16 = l & 15, kq = l >> 4;
  if (zero && l == 0 && blockIdx.x == 0) *zero = 0;  // the batch's accepted-feature count
  // Placement on XCD_GROUPS of the 8 XCDs only (blocks labelled blockIdx % 8 >= XCD_GROUPS exit at once):
  // every XCD that runs tiles fetches all of P_can into its L2, so the small batches (cfg2: 217 single-wave
  // tiles, a few per CU on two XCDs) read P_can twice instead of eight times; each group takes a contiguous
  // range of tiles, i.e. whole row blocks of H.
  constexpr int XCD_GROUPS = 2;
  const int x = blockIdx.x % 8;
  if (x >= XCD_GROUPS) return;
  const int tc = (n + 15) / 16, nwg = tc * ((m + 15) / 16), per = (nwg + XCD_GROUPS - 1) / XCD_GROUPS;
  const int wid = x * per + blockIdx.x / 8;
  if (wid >= nwg || wid >= (x + 1) * per) return;
  const int ti = wid / tc, tj = wid - ti * tc;
  for (int e = l; e < n; e += 64) sh_hidx[e] = hidx[e];
  __syncthreads();
  const int i0 = ti * 16, j0 = tj * 16;
  const int arow = i0 + r16, bcol = j0 + r16;
  const double *Hr = H + (size_t)min(arow, m - 1) * ldh;
  const double *Pc = P + ((bcol < n) ? sh_hidx[bcol] : 0);
  const bool ain = arow < m, bin = bcol < n;
  double a0[HPS / 4], b0[HPS / 4], a1[HPS / 4], b1[HPS / 4];
  auto load = [&](int k0, double *a, double *b) {
#pragma unroll
    for (int u = 0; u < HPS / 4; u++) {
      const int k = k0 + 4 * u + kq;
      const bool kin = k < n;
      a[u] = (ain && kin) ? Hr[k] : 0.0;
      b[u] = (bin && kin) ? Pc[(size_t)sh_hidx[k] * ldp] : 0.0;
    }
  };
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  load(0, a0, b0);
  for (int k0 = 0; k0 < n; k0 += 2 * HPS) {
    if (k0 + HPS < n) load(k0 + HPS, a1, b1);
#pragma unroll
    for (int u = 0; u < HPS / 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[u], b0[u], acc, 0, 0, 0);
    if (k0 + HPS >= n) break;
    if (k0 + 2 * HPS < n) load(k0 + 2 * HPS, a0, b0);
#pragma unroll
    for (int u = 0; u < HPS / 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[u], b1[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int row = i0 + kq + 4 * q, col = j0 + r16;
    if (row < m && col < n) T[(size_t)row * ldt + col] = acc[q];
  }
}

// The same product for large batches (configs 4-5: m ~ 80k stacked rows, n = 172-242): 256-thread
// workgroups own a 64 x 64 tile of T, K runs in slabs of 16 staged in LDS (the H slab as rows, the
// P_can slab as a 16 x 64 block), each wave computes a 32 x 32 quarter with four MFMA tiles.  Two LDS stages:
// slab s + 1 is loaded (global -> registers) before slab s's MFMAs and written to the other stage after them,
// one barrier per slab.  Operand reuse: every staged element feeds 4 MFMAs instead of 1 (k_gemm_HPg reloads per
// tile).  HIDX: P_can gathered from P through hidx in the loads; without it P is P_can itself (dense n x n,
// gathered once by k_gather_pcan), which is how the engine runs it.  A compile-time choice: the runtime branch
// on hidx cost the pcan path half again its time (cfg5: 350 against 224 us per launch, tools/bench_hpg.hip).
// The accumulation over k is the same ascending 4-wide MFMA chain per element in every variant (bit-identical).
constexpr int HPB = 64, HPK = 16;
template <bool HIDX>
__global__ void __launch_bounds__(256) k_gemm_HPg_tiled(const double *__restrict__ H, int m, int n, int ldh,
                                                        const double *__restrict__ P, int ldp,
                                                        const int *__restrict__ hidx, double *__restrict__ T, int ldt,
                                                        int *zero) {
  __shared__ double As[2][HPB][HPK + 1];
  __shared__ double Bs[2][HPK][HPB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  if (zero && tid == 0 && blockIdx.x == 0) *zero = 0;
  // work index = row tile * column tiles + column tile, XCD-swizzled: a row slab of H is fetched once per
  // XCD (its column tiles run side by side there) instead of once per column tile
  const int tc = (n + HPB - 1) / HPB;
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), ti = wid / tc;
  const int i0 = ti * HPB, j0 = (wid - ti * tc) * HPB;
  // staging map: A slab element e = tid + 256 u (u < 4): row e / 16, k e % 16; B slab: k e / 64, col e % 64
  int pcol[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int c = j0 + ((tid + 256 * u) & 63);
    pcol[u] = (c < n) ? (HIDX ? hidx[c] : c) : 0;
  }
  double ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      const int ar = i0 + (e >> 4), ak = k0 + (e & 15);
      ra[u] = (ar < m && ak < n) ? H[(size_t)ar * ldh + ak] : 0.0;
      const int bk = k0 + (e >> 6), bc = j0 + (e & 63);
      rb[u] = (bk < n && bc < n) ? P[(size_t)(HIDX ? hidx[bk] : bk) * ldp + pcol[u]] : 0.0;
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      As[st][e >> 4][e & 15] = ra[u];
      Bs[st][e >> 6][e & 63] = rb[u];
    }
  };
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(0);
  store(0);
  __syncthreads();
  int st = 0;
  for (int k0 = 0; k0 < n; k0 += HPK) {
    const bool more = k0 + HPK < n;
    if (more) load(k0 + HPK);
#pragma unroll
    for (int kk = 0; kk < HPK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[t] = As[st][32 * wr + 16 * t + r16][kk + kq];
        b[t] = Bs[st][kk + kq][32 * wc + 16 * t + r16];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ta++)
#pragma unroll
        for (int tb = 0; tb < 2; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
    if (more) store(st ^ 1);  // the other stage: its last readers finished before the previous barrier
    __syncthreads();
    st ^= 1;
  }
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 2; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 32 * wr + 16 * ta + kq + 4 * q, col = j0 + 32 * wc + 16 * tb + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}

// P_can = P[hidx, hidx] (n x n, dense) for the large-batch T GEMM
__global__ void __launch_bounds__(256) k_gather_pcan(const double *__restrict__ P, int ldp,
                                                     const int *__restrict__ hidx, int n, double *__restrict__ Pc) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * n) return;
  const int i = e / n, j = e - i * n;
  Pc[e] = P[(size_t)hidx[i] * ldp + hidx[j]];
}

size_t chi2_lds_bytes(int max_rows_f, int n) {
  size_t R = max_rows_f;
  return (2 * R * (size_t)(n | 1) + (R + 1) * (R | 1) + 4 * (R + 1)) * sizeof(double);
}

// One workgroup per feature.  out[f] carries the feature kernel's status / rows; chi2 rows are the
// feature's H_all rows from c0 = (mode >= 2 ? 3 : 0) on (delayed init tests the update rows against
// chi2(dof = all rows), StateHelper.cpp:463-468).
constexpr int kChi2Threads = 512;

// The lower triangle of S = T Hhat^T + s2 I of every feature whose H and T rows do not fit k_chi2's LDS: one wave
// per 16x16 tile (k-ascending MFMA chain, the expression k_chi2 uses), kChiSWaves tiles per workgroup, so the
// rows are pulled by many CUs at once instead of one.  S_f lands at Sbuf + f * stride in k_chi2's LDS layout
// (row stride R|1).  Workgroup blockIdx serves feature f = 8 (k / groups) + blockIdx % 8 with k = blockIdx / 8:
// all of a feature's tiles run on the XCD that k_chi2's workgroup f runs on (blockIdx % 8 labels the XCD), so
// that workgroup reads S out of its own L2.
constexpr int kChiSWaves = 4;
__global__ void __launch_bounds__(64 * kChiSWaves) k_chi2_S(DBatchParams bp, const DFeat *__restrict__ feats,
                                                            const double *__restrict__ H_all,
                                                            const double *__restrict__ T_all,
                                                            const DFeatOut *__restrict__ out, double *__restrict__ Sbuf,
                                                            size_t stride, int groups) {
  const int k = blockIdx.x / 8, f = 8 * (k / groups) + blockIdx.x % 8, g = k % groups;
  if (f >= bp.nfeat) return;
  const DFeatOut o = out[f];
  if (o.status != 0 || o.rows <= 0) return;
  const DFeat F = feats[f];
  const int n = bp.n_canon, ldh = bp.ldh, c0 = (F.mode >= 2) ? 3 : 0, R = o.rows - c0;
  const int lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const int nt = (R + 15) / 16, t = g * kChiSWaves + (threadIdx.x >> 6);
  if (R <= 0 || t >= nt * (nt + 1) / 2) return;
  int ti = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
  while (ti * (ti + 1) / 2 > t) ti--;
  while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
  const int tj = t - ti * (ti + 1) / 2;
  const int arow = 16 * ti + r16, bcol = 16 * tj + r16;
  const double *ta = T_all + (size_t)(F.row_off + c0 + min(arow, R - 1)) * ldh;
  const double *hb = H_all + (size_t)(F.row_off + c0 + min(bcol, R - 1)) * ldh;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  auto la = [&](int kk) { return (arow < R && kk < n) ? ta[kk] : 0.0; };
  auto lb = [&](int kk) { return (bcol < R && kk < n) ? hb[kk] : 0.0; };
  acc = tile_chain<16>(0, n, kq, la, lb, acc);
  double *S = Sbuf + (size_t)f * stride;
  const int ldS = R | 1;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int i = 16 * ti + kq + 4 * q, j = 16 * tj + r16;
    if (i < R && j <= i) S[(size_t)i * ldS + j] = acc[q] + (i == j ? bp.sigma_pix_sq : 0.0);
  }
}
// The same S with one workgroup per feature: the feature's T and H rows are staged in LDS once per 32-column chunk
// and shared by all its tiles (k_chi2_S reads them again for every tile, from L2 or HBM: about three times the bytes
// at cfg4 / cfg5).  Wave w keeps the accumulators of tiles w, w + 4, ... across the chunks; every tile is the same
// ascending chain of 4-wide MFMA steps over k as k_chi2_S's tile_chain (a step exists iff its first k is < n, zero
// operands past n and past the feature's rows), so S is bit-identical.  Workgroup f serves feature f, on the XCD
// that k_chi2's workgroup f reads S from.  (256 threads with 9 tiles per wave: 308 VGPRs, one wave per SIMD,
// 191 / 147 us per launch at cfg5 / cfg4 against k_chi2_S's 209 / 206.)
constexpr int kS2Threads = 512, kS2Waves = kS2Threads / 64, kS2KC = 32, kS2Tiles = 5;  // up to 40 >= 36 tiles, R <= 128
__global__ void __launch_bounds__(kS2Threads) k_chi2_S2(DBatchParams bp, const DFeat *__restrict__ feats,
                                                       const double *__restrict__ H_all, const double *__restrict__ T_all,
                                                       const DFeatOut *__restrict__ out, double *__restrict__ Sbuf,
                                                       size_t stride) {
  extern __shared__ double lds[];
  const int f = blockIdx.x;
  if (f >= bp.nfeat) return;
  const DFeatOut o = out[f];
  if (o.status != 0 || o.rows <= 0) return;
  const DFeat F = feats[f];
  const int n = bp.n_canon, ldh = bp.ldh, c0 = (F.mode >= 2) ? 3 : 0, R = o.rows - c0;
  if (R <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r16 = lane & 15, kq = lane >> 4;
  const int nt = (R + 15) / 16, ntiles = nt * (nt + 1) / 2, Rp = 16 * nt;
  constexpr int LDK = kS2KC + 1;  // odd row stride: the operand reads of a tile hit distinct banks
  double *Ts = lds, *Hs = lds + (size_t)Rp * LDK;
  const double *tg = T_all + (size_t)(F.row_off + c0) * ldh, *hg = H_all + (size_t)(F.row_off + c0) * ldh;
  int ti[kS2Tiles], tj[kS2Tiles];
#pragma unroll
  for (int q = 0; q < kS2Tiles; q++) {
    const int t = wid + kS2Waves * q;
    int a = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
    while (a * (a + 1) / 2 > t) a--;
    while ((a + 1) * (a + 2) / 2 <= t) a++;
    ti[q] = a;
    tj[q] = t - a * (a + 1) / 2;
  }
  dbl4 acc[kS2Tiles];
#pragma unroll
  for (int q = 0; q < kS2Tiles; q++) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
  // a chunk's loads all issued before its LDS stores (one memory round trip per chunk), the next chunk's issued
  // before this chunk's MFMAs
  constexpr int NU = 128 * kS2KC / kS2Threads;
  double rt[NU], rh[NU];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int e = tid + kS2Threads * u, r = e / kS2KC, k = k0 + (e % kS2KC);
      const bool in = r < R && k < n;
      rt[u] = in ? tg[(size_t)r * ldh + k] : 0.0;
      rh[u] = in ? hg[(size_t)r * ldh + k] : 0.0;
    }
  };
  load(0);
  for (int k0 = 0; k0 < n; k0 += kS2KC) {
    __syncthreads();  // the previous chunk's operand reads are done
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int e = tid + kS2Threads * u, r = e / kS2KC, c = e % kS2KC;
      if (r < Rp) {
        Ts[r * LDK + c] = rt[u];
        Hs[r * LDK + c] = rh[u];
      }
    }
    __syncthreads();
    if (k0 + kS2KC < n) load(k0 + kS2KC);
    for (int s = 0; s < kS2KC && k0 + s < n; s += 4) {
#pragma unroll
      for (int q = 0; q < kS2Tiles; q++)
        if (wid + kS2Waves * q < ntiles) {
          const double a = Ts[(16 * ti[q] + r16) * LDK + s + kq];
          const double b = Hs[(16 * tj[q] + r16) * LDK + s + kq];
          acc[q] = mfma4(a, b, acc[q]);
        }
    }
  }
  double *S = Sbuf + (size_t)f * stride;
  const int ldS = R | 1;
#pragma unroll
  for (int q = 0; q < kS2Tiles; q++)
    if (wid + kS2Waves * q < ntiles)
#pragma unroll
      for (int qq = 0; qq < 4; qq++) {
        const int i = 16 * ti[q] + kq + 4 * qq, j = 16 * tj[q] + r16;
        if (i < R && j <= i) S[(size_t)i * ldS + j] = acc[q][qq] + (i == j ? bp.sigma_pix_sq : 0.0);
      }
}

// SMAX: the factorization's panel rows per lane (dense_lds.h ldl_wave_inv), from the batch's largest feature: a
// compile-time choice, so a batch of small features does not carry the register footprint of the largest instance
// (one instance for all sizes took 214 VGPRs and one 512-thread workgroup per CU)
template <int SMAX>
__global__ void __launch_bounds__(kChi2Threads) k_chi2(DBatchParams bp, const DFeat *__restrict__ feats, double *__restrict__ H_all,
                                              double *__restrict__ T_all, const double *__restrict__ chi2_table,
                                              DFeatOut *__restrict__ out, int use_lds, int *acc_count,
                                              const double *__restrict__ Sg, size_t sg_stride) {
  extern __shared__ double lds[];
  __shared__ double red[kChi2Threads];
  __shared__ int st;
  const int f = blockIdx.x;
  long long *tsp = bp.dbg_ts ? bp.dbg_ts + (size_t)f * 16 + 8 : nullptr;  // debug phase stamps
#define CHI2_TS(k) \
  if (tsp && threadIdx.x == 0) tsp[k] = clock64();
  CHI2_TS(0)
  const DFeat F = feats[f];
  const DFeatOut o = out[f];
  if (o.status != 0 || o.rows <= 0) return;
  const int n = bp.n_canon, ldh = bp.ldh;
  const int c0 = (F.mode >= 2) ? 3 : 0;
  const int R = o.rows - c0;
  const int tid = threadIdx.x;
  if (R <= 0) {
    if (tid == 0) {
      out[f].chi2 = 0.0;
      if (acc_count) atomicAdd(acc_count, 1);
    }
    return;
  }
  const double *Hg = H_all + (size_t)(F.row_off + c0) * ldh;
  const double *Tg = T_all + (size_t)(F.row_off + c0) * ldh;
  const double *Hs = Hg, *Ts = Tg;
  int ldx = ldh;
  double *S = lds;
  const int ldS = R | 1;
  double *Lp = lds + (size_t)(R + 1) * ldS;
  if (Sg) {
    // S formed by k_chi2_S: the lower triangle rows in this layout already
    const double *Sf = Sg + (size_t)f * sg_stride;
    staged_copy(
        R * ldS, [&](int e) { return (e % ldS <= e / ldS) ? Sf[e] : 0.0; }, [&](int e, double v) { S[e] = v; });
  } else if (use_lds) {
    const int ldl = n | 1;  // odd row stride: the MFMA operand reads below hit distinct banks
    double *Hl = Lp + (size_t)(R + 1) * 4;
    double *Tl = Hl + (size_t)R * ldl;
    staged_copy(
        2 * R * n,
        [&](int e) {
          const int h = e >= R * n, f = e - h * R * n, i = f / n, j = f - i * n;
          return (h ? Tg : Hg)[(size_t)i * ldh + j];
        },
        [&](int e, double v) {
          const int h = e >= R * n, f = e - h * R * n, i = f / n, j = f - i * n;
          (h ? Tl : Hl)[(size_t)i * ldl + j] = v;
        });
    Hs = Hl;
    Ts = Tl;
    ldx = ldl;
    __syncthreads();
  }
  // lower triangle of S = T Hhat^T + s2 I on the matrix cores (16x16 tiles, K = n), then the residual row
  if (!Sg) {
    const int lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6, r16 = lane & 15, kq = lane >> 4;
    const int nt = (R + 15) / 16, ntiles = nt * (nt + 1) / 2;
    for (int t = wid; t < ntiles; t += nw) {
      int ti = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
      while (ti * (ti + 1) / 2 > t) ti--;
      while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
      const int tj = t - ti * (ti + 1) / 2;
      const int arow = 16 * ti + r16, bcol = 16 * tj + r16;
      const double *ta = Ts + (size_t)min(arow, R - 1) * ldx, *hb = Hs + (size_t)min(bcol, R - 1) * ldx;
      // 16 k-slabs (64 columns) of loads in flight per round trip: from global memory (rows too long for LDS)
      // the tile costs ceil(n / 64) memory round trips instead of one per 16 columns; ascending k either way
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
      auto la = [&](int k) { return (arow < R && k < n) ? ta[k] : 0.0; };
      auto lb = [&](int k) { return (bcol < R && k < n) ? hb[k] : 0.0; };
      acc = tile_chain<16>(0, n, kq, la, lb, acc);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int i = 16 * ti + kq + 4 * q, j = 16 * tj + r16;
        if (i < R && j <= i) S[i * ldS + j] = acc[q] + (i == j ? bp.sigma_pix_sq : 0.0);
      }
    }
  }
  for (int j = tid; j < R; j += blockDim.x) S[R * ldS + j] = Hg[(size_t)j * ldh + n];
  __syncthreads();
  CHI2_TS(1)
  // LDL^T with the serial chain on one wave (dense_lds.h ldl_wave): the residual row leaves as
  // y = D^-1 L_u^-1 r, so chi2 = r^T S^-1 r = sum_k d_k y_k^2
  double *Dd = Lp;
  ldl_wave_inv<SMAX>(S, SqLayout{ldS}, R, R + 1, Dd, false);
  CHI2_TS(2)
  double c2 = 0.0;
  for (int k = tid; k < R; k += blockDim.x) {
    const double y = S[R * ldS + k];
    c2 += Dd[k] * (y * y);
  }
  red[tid] = c2;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    double chi2 = red[0];
    double thr = chi2_table[min(F.mode >= 2 ? o.rows : R, 999)];
    int reject = chi2 > bp.chi2_mult * thr;
    out[f].chi2 = chi2;
    if (reject) {
      out[f].status = 3;
      out[f].rows = 0;
    } else if (acc_count) {
      atomicAdd(acc_count, 1);
    }
    st = reject;
  }
  CHI2_TS(3)
#undef CHI2_TS
  __syncthreads();
  if (st && F.mode <= 1) {
    // the rejected feature's rows of H_all and of T = H_all P_can (the direct update's S reuses T)
    double *rows = H_all + (size_t)F.row_off * ldh;
    double *trows = T_all + (size_t)F.row_off * ldh;
    for (int e = tid; e < o.rows * (n + 1); e += blockDim.x) {
      int i = e / (n + 1), j = e - i * (n + 1);
      rows[(size_t)i * ldh + j] = 0.0;
      if (j < n) trows[(size_t)i * ldh + j] = 0.0;
    }
  }
}

void launch_chi2_batch(hipStream_t s, const DBatchParams &bp, const DFeat *feats, const double *P, const int *hidx,
                       double *H_all, int m, double *T_all, const double *chi2_table, DFeatOut *out, int max_rows_f,
                       int *acc_count, double *pcan, double **sbuf, size_t *sbuf_cap) {
  if (bp.nfeat <= 0 || m <= 0) return;
  const int n = bp.n_canon;
  if (m >= 4096) {  // enough 64 x 64 tiles to fill the 256 CUs
    if (pcan)
      hipLaunchKernelGGL(k_gather_pcan, dim3((n * n + 255) / 256), dim3(256), 0, s, P, bp.ldp, hidx, n, pcan);
    const dim3 grid(((n + HPB - 1) / HPB) * ((m + HPB - 1) / HPB));
    if (pcan)
      hipLaunchKernelGGL(k_gemm_HPg_tiled<false>, grid, dim3(256), 0, s, H_all, m, n, bp.ldh, pcan, n, nullptr, T_all,
                         bp.ldh, acc_count);
    else
      hipLaunchKernelGGL(k_gemm_HPg_tiled<true>, grid, dim3(256), 0, s, H_all, m, n, bp.ldh, P, bp.ldp, hidx, T_all,
                         bp.ldh, acc_count);
  } else
    hipLaunchKernelGGL(k_gemm_HPg, dim3(8 * ((((n + 15) / 16) * ((m + 15) / 16) + 1) / 2)), dim3(64),
                       sizeof(int) * (size_t)n, s, H_all, m, n, bp.ldh, P, bp.ldp, hidx, T_all, bp.ldh, acc_count);
  if (max_rows_f + 1 > kWaveMaxRows)
    throw std::runtime_error("feature with " + std::to_string(max_rows_f) + " rows: wider than the chi2 factorization panel");
  size_t bytes = chi2_lds_bytes(max_rows_f, n);
  int use_lds = bytes <= kMaxDynLds;
  if (!use_lds) bytes = ((size_t)(max_rows_f + 1) * (max_rows_f | 1) + 4 * (size_t)(max_rows_f + 1)) * sizeof(double);
  // the instance for the batch's largest feature (R + 1 rows with the residual row)
  const int smax = (max_rows_f + 1 + 63) / 64;
  typedef void (*Chi2Fn)(DBatchParams, const DFeat *, double *, double *, const double *, DFeatOut *, int, int *,
                         const double *, size_t);
  static const Chi2Fn kChi2Fn[4] = {k_chi2<1>, k_chi2<2>, k_chi2<3>, k_chi2<4>};
  const Chi2Fn chi2_fn = kChi2Fn[std::min(std::max(smax, 1), 4) - 1];
  static int granted_inst[4] = {-1, -1, -1, -1};
  int &granted = granted_inst[std::min(std::max(smax, 1), 4) - 1];
  if (granted < 0) granted = set_dyn_lds((const void *)chi2_fn, kMaxDynLds);
  if (bytes > 64 * 1024 && (int)bytes > granted)
    throw std::runtime_error("k_chi2 needs " + std::to_string(bytes) + " B of LDS, granted " + std::to_string(granted));
  // features too large for the LDS staging: S over many CUs first (k_chi2_S), k_chi2 reads it
  double *Sg = nullptr;
  size_t stride = 0;
  static const bool no_s = std::getenv("UVIO_HP_NO_CHI2_S") != nullptr;  // A/B switch: k_chi2 forms S itself
  if (!use_lds && sbuf && sbuf_cap && !no_s) {
    stride = (size_t)max_rows_f * (max_rows_f | 1);
    const size_t need = stride * (size_t)bp.nfeat;
    if (need > *sbuf_cap) {
      auto ok = [](hipError_t e, const char *what) {
        if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
      };
      if (*sbuf) {
        ok(hipStreamSynchronize(s), "chi2 S buffer: stream sync");  // the old buffer may still be read
        ok(hipFree(*sbuf), "chi2 S buffer: free");
      }
      *sbuf = nullptr;
      *sbuf_cap = 0;
      ok(hipMalloc(sbuf, need * 3 / 2 * sizeof(double)), "chi2 S buffer: alloc");
      *sbuf_cap = need * 3 / 2;
    }
    Sg = *sbuf;
    const int nt = (max_rows_f + 15) / 16, groups = (nt * (nt + 1) / 2 + kChiSWaves - 1) / kChiSWaves;
    static const bool per_tile = std::getenv("UVIO_HP_CHI2_S_TILES") != nullptr;  // A/B switch: k_chi2_S
    const size_t s2_bytes = (size_t)2 * 16 * nt * (kS2KC + 1) * sizeof(double);
    if (!per_tile && nt * (nt + 1) / 2 <= kS2Waves * kS2Tiles) {
      static int granted2 = -1;
      if (granted2 < 0) granted2 = set_dyn_lds((const void *)k_chi2_S2, kMaxDynLds);
      if (s2_bytes > 64 * 1024 && (int)s2_bytes > granted2)
        throw std::runtime_error("k_chi2_S2 needs " + std::to_string(s2_bytes) + " B of LDS, granted " + std::to_string(granted2));
      hipLaunchKernelGGL(k_chi2_S2, dim3(bp.nfeat), dim3(kS2Threads), s2_bytes, s, bp, feats, H_all, T_all, out, Sg,
                         stride);
    } else {
      hipLaunchKernelGGL(k_chi2_S, dim3(8 * ((bp.nfeat + 7) / 8) * groups), dim3(64 * kChiSWaves), 0, s, bp, feats,
                         H_all, T_all, out, Sg, stride, groups);
    }
  }
  hipLaunchKernelGGL(chi2_fn, dim3(bp.nfeat), dim3(kChi2Threads), bytes, s, bp, feats, H_all, T_all, chi2_table, out, use_lds,
                     acc_count, Sg, stride);
}

}  // namespace uvhp
