// Small dense factorizations for ONE workgroup, matrices resident in LDS.
//
// The estimator's dense solves are small (r, n <= ~256) and sequential by nature, so they are
// latency bound: the cost is (number of sequential steps) x (latency of one step).  Long dependent
// chains inside a step (a single lane walking a row through LDS, or a wave-level 16x16 factor with
// v_readlane hops) cost far more than the barrier itself, so both routines take ONE barrier per
// column and make every step a flat parallel update whose only latency is one LDS round trip:
//   ldl_inplace      : right-looking LDL^T with unnormalized columns (no intra-step race); extra rows
//                      below n are right-hand sides (an appended residual row yields L_unit^-1 r, so
//                      chi2 = sum_k z_k^2 / d_k without a triangular solve);
//   ldl_to_chol      : L D^1/2 (the LLT factor StateHelper.cpp:160 uses) in one parallel pass;
//   trtri_gj_inplace : L^-1 by in-place Gauss-Jordan, one thread per row, one barrier per column.
// Measured on MI355X (tools/bench_dense.hip): see DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>

namespace uvhp {

// Stage `count` doubles: st(e, ld(e)) for e < count, with the global loads batched kStageBatch per
// thread (issued together, so staging costs one memory round trip per batch instead of one per element).
constexpr int kStageBatch = 8;
template <class LoadF, class StoreF>
__device__ __forceinline__ void staged_copy(int count, LoadF ld, StoreF st) {
  for (int e0 = threadIdx.x; e0 < count; e0 += kStageBatch * blockDim.x) {
    double v[kStageBatch];
#pragma unroll
    for (int u = 0; u < kStageBatch; u++) {
      const int e = e0 + u * blockDim.x;
      v[u] = (e < count) ? ld(e) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kStageBatch; u++) {
      const int e = e0 + u * blockDim.x;
      if (e < count) st(e, v[u]);
    }
  }
}

// LDS bytes for an (nrows x n) factorization: A with an odd row stride (ld = n | 1)
__host__ __device__ inline size_t dense_lds_bytes(int nrows, int n) { return (size_t)nrows * (n | 1) * sizeof(double); }

// In-place LDL^T of the n x n lower triangle of A (right-looking, ONE barrier per column): after
// it, A[k][k] = d_k and A[i][k] = d_k L[i][k] for i > k (columns are left unnormalized, so step k
// only reads column k and writes columns > k -- no intra-step race).  Rows n .. nrows-1 are extra
// right-hand-side rows: they leave as z = L_unit^-1 b (unnormalized, z_k = d_k (row)_k).
// Thread mapping: 8 consecutive lanes share a row and stride its columns by 8 (rows never straddle
// a wavefront, no integer division in the loop).
constexpr int kRowLanes = 8;
__device__ void ldl_inplace(double *A, int ld, int n, int nrows) {
  const int c0 = threadIdx.x % kRowLanes, rstep = blockDim.x / kRowLanes;
  for (int k = 0; k < n; k++) {
    const double dinv = 1.0 / A[k * ld + k];
    const double *__restrict__ colk = A + k;
    for (int i = k + 1 + threadIdx.x / kRowLanes; i < nrows; i += rstep) {
      double *__restrict__ Ai = A + i * ld;
      const double aik = Ai[k] * dinv;
      const int jmax = min(i, n - 1);
      for (int j = k + 1 + c0; j <= jmax; j += kRowLanes) Ai[j] -= aik * colk[j * ld];
    }
    __syncthreads();
  }
}

// LDL^T (as left by ldl_inplace) -> Cholesky factor L D^1/2 in place; extra rows -> b L^-T.
__device__ void ldl_to_chol(double *A, int ld, int n, int nrows) {
  // d_k^-1/2 formed once per column (256-column chunks through LDS), then the rows scale by it
  __shared__ double isd[256];
  const int c0 = threadIdx.x % kRowLanes, rstep = blockDim.x / kRowLanes;
  for (int k0 = 0; k0 < n; k0 += 256) {
    const int k1 = min(n, k0 + 256);
    for (int k = k0 + threadIdx.x; k < k1; k += blockDim.x) isd[k - k0] = 1.0 / sqrt(A[k * ld + k]);
    __syncthreads();
    for (int i = threadIdx.x / kRowLanes; i < nrows; i += rstep) {
      const int jmax = min(min(i - 1, n - 1), k1 - 1);
      for (int k = k0 + c0; k <= jmax; k += kRowLanes) A[i * ld + k] *= isd[k - k0];
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < n; k += blockDim.x) A[k * ld + k] = sqrt(A[k * ld + k]);
  __syncthreads();
}

// In-place inverse of a lower-triangular L by Gauss-Jordan elimination (ONE barrier per column).
// Row i keeps its not-yet-eliminated L entries at columns >= k and the inverse's entries at columns
// < k; the final pass divides by the pivots.  8 lanes per row as in ldl_inplace; the lanes of a row
// read A[i][k] before the row's first lane overwrites it (same wavefront, in-order LDS).
__device__ void trtri_gj_inplace(double *A, int ld, int n) {
  const int c0 = threadIdx.x % kRowLanes, rstep = blockDim.x / kRowLanes;
  for (int k = 0; k < n; k++) {
    const double pinv = 1.0 / A[k * ld + k];
    const double *__restrict__ Rk = A + k * ld;
    for (int i = k + 1 + threadIdx.x / kRowLanes; i < n; i += rstep) {
      double *__restrict__ Ri = A + i * ld;
      const double f = Ri[k] * pinv;
      for (int j = c0; j < k; j += kRowLanes) Ri[j] -= f * Rk[j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (c0 == 0) Ri[k] = -f;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x / kRowLanes; i < n; i += rstep) {
    const double s = 1.0 / A[i * ld + i];
    for (int j = c0; j < i; j += kRowLanes) A[i * ld + j] *= s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) A[i * ld + i] = 1.0 / A[i * ld + i];
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// Blocked LDL^T, same in/out convention as ldl_inplace, in 4-column panels:
//   * every thread owns one panel row (rows K .. nrows-1, strided by blockDim) and eliminates its 4
//     panel entries against the 4x4 diagonal block, whose LDL every thread recomputes in registers
//     from 10 broadcast LDS reads (no barrier inside the panel); the unnormalized entries go back to
//     A, the normalized multipliers to Lp (nrows x 4 scratch);
//   * the rank-4 trailing update A22 -= L21 (D L21^T) is ONE v_mfma_f64_16x16x4_f64 per 16x16 tile of
//     the lower triangle (A operand: -Lp rows, B operand: the panel rows' unnormalized entries).
// Two barriers per 4 columns instead of one per column, and the update work runs on the matrix cores.
typedef double dbl4 __attribute__((ext_vector_type(4)));

// XCD-aware work index (bijective on [0, nwg)): the dispatcher deals workgroups out to the 8 XCDs round
// robin (blockIdx % 8 labels the blocks that share one XCD and its L2), so consecutive work indices --
// the tiles of one row block, or the tile pairs of one row chunk -- land on the same XCD and share the
// operand rows it has cached instead of each XCD fetching them again.  Only placement changes: every work
// index is computed exactly as before.
__device__ __forceinline__ dbl4 mfma4(double a, double b, dbl4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Accumulate one 16x16 tile over k in [0, kend): acc += sum_k A(r16, k) B(k, r16) with the operands fetched
// through the callables (k = 4 s + kq); the loads of U k-slabs are issued before their MFMAs, so a chunk of
// 4U columns costs one memory round trip.  U = 8 by default; 16 for the products whose operands come from
// global memory behind a long latency (the chi2 S tiles, k_ekf_MS).  (32-slab chunks measured slower in
// k_ekf_MS / k_ekf_WP in round 2: 24.4 / 10.3 against 19-22 / 8.9 us at cfg2, profiles/r02e_cfg2_per_frame.txt.)
template <int U = 8, class LA, class LB>
__device__ __forceinline__ dbl4 tile_chain(int kbeg, int kend, int kq, LA la, LB lb, dbl4 acc) {
  for (int k0 = kbeg; k0 < kend; k0 += 4 * U) {
    double a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = k0 + 4 * u + kq;
      const bool in = k < kend;
      a[u] = in ? la(k) : 0.0;
      b[u] = in ? lb(k) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (k0 + 4 * u < kend) acc = mfma4(a[u], b[u], acc);
  }
  return acc;
}

__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = orig % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
}

__device__ void ldl_panel4(double *A, int ld, int n, int nrows, double *Lp) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int K = 0; K < n; K += 4) {
    const int B = min(4, n - K);
    // 4x4 diagonal block LDL (identical arithmetic in every thread)
    double c[4][4];  // unnormalized final values of the diagonal block rows (lower)
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int p = 0; p <= q; p++) c[q][p] = (q < B) ? A[(K + q) * ld + K + p] : 0.0;
    double dinv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      dinv[k] = (k < B) ? 1.0 / c[k][k] : 0.0;
#pragma unroll
      for (int q = k + 1; q < 4; q++) {
        const double a = c[q][k] * dinv[k];
#pragma unroll
        for (int p = k + 1; p <= q; p++) c[q][p] -= a * c[p][k];
      }
    }
    __syncthreads();  // every wave has read the diagonal block before the panel rows overwrite it
    // panel rows
    for (int i = K + threadIdx.x; i < nrows; i += blockDim.x) {
      double v[4];
#pragma unroll
      for (int p = 0; p < 4; p++) v[p] = (p < B && K + p <= i) ? A[i * ld + K + p] : 0.0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (k < B && i > K + k) {
          const double a = v[k] * dinv[k];
#pragma unroll
          for (int p = k + 1; p < 4; p++)
            if (p < B && K + p <= i) v[p] -= a * c[p][k];
        }
      }
#pragma unroll
      for (int p = 0; p < 4; p++) {
        if (p < B && K + p <= i) A[i * ld + K + p] = v[p];
        Lp[(size_t)i * 4 + p] = (p < B && K + p < i) ? v[p] * dinv[p] : 0.0;
      }
    }
    __syncthreads();
    const int T0 = K + B;
    if (T0 < n) {
      const int nti = (nrows - T0 + 15) / 16, ntj = (n - T0 + 15) / 16;
      const int r16 = lane & 15, kq = lane >> 4;
      for (int t = wid; t < nti * ntj; t += nw) {
        const int ti = t / ntj, tj = t - ti * ntj;
        if (tj > ti) continue;
        const int i0 = T0 + 16 * ti, j0 = T0 + 16 * tj;
        dbl4 acc;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int row = i0 + kq + 4 * q, col = j0 + r16;
          acc[q] = (row < nrows && col < n && col <= row) ? A[row * ld + col] : 0.0;
        }
        const int arow = i0 + r16, bcol = j0 + r16;
        const double a = (arow < nrows) ? -Lp[(size_t)arow * 4 + kq] : 0.0;
        const double b = (bcol < n && kq < B) ? A[bcol * ld + K + kq] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int row = i0 + kq + 4 * q, col = j0 + r16;
          if (row < nrows && col < n && col <= row) A[row * ld + col] = acc[q];
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Two-level blocked LDL^T, same in/out convention (and the same nrows x 4 scratch Lp) as ldl_panel4.
// Columns go in blocks of 16; inside a block the 4-column steps of ldl_panel4 update only the block's
// own later columns (one 16-wide tile column), and the rest of the matrix gets the block's rank-16
// update once, as four v_mfma_f64_16x16x4_f64 per tile with the normalized multipliers formed from the
// stored unnormalized entries and the block's 1/d_k.  The per-step work that scales with the trailing
// size runs once per 16 columns instead of once per 4.
__device__ void ldl_blk16(double *A, int ld, int n, int nrows, double *Lp) {
  __shared__ double Dv[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  for (int KB = 0; KB < n; KB += 16) {
    const int nb = min(n, KB + 16);  // columns KB .. nb-1 form the block
    for (int K = KB; K < nb; K += 4) {
      const int B = min(4, nb - K);
      double c[4][4];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int p = 0; p <= q; p++) c[q][p] = (q < B) ? A[(size_t)(K + q) * ld + K + p] : 0.0;
      double dinv[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        dinv[k] = (k < B) ? 1.0 / c[k][k] : 0.0;
#pragma unroll
        for (int q = k + 1; q < 4; q++) {
          const double a = c[q][k] * dinv[k];
#pragma unroll
          for (int p = k + 1; p <= q; p++) c[q][p] -= a * c[p][k];
        }
      }
      if (threadIdx.x < 4) Dv[K - KB + threadIdx.x] = dinv[threadIdx.x];
      __syncthreads();  // every wave has read the diagonal block before the panel rows overwrite it
      for (int i = K + threadIdx.x; i < nrows; i += blockDim.x) {
        double v[4];
#pragma unroll
        for (int p = 0; p < 4; p++) v[p] = (p < B && K + p <= i) ? A[(size_t)i * ld + K + p] : 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (k < B && i > K + k) {
            const double a = v[k] * dinv[k];
#pragma unroll
            for (int p = k + 1; p < 4; p++)
              if (p < B && K + p <= i) v[p] -= a * c[p][k];
          }
        }
#pragma unroll
        for (int p = 0; p < 4; p++) {
          if (p < B && K + p <= i) A[(size_t)i * ld + K + p] = v[p];
          Lp[(size_t)i * 4 + p] = (p < B && K + p < i) ? v[p] * dinv[p] : 0.0;
        }
      }
      __syncthreads();
      // rank-4 update of the block's own later columns (one tile column)
      const int T0 = K + B;
      if (T0 < nb) {
        const int nti = (nrows - T0 + 15) / 16;
        for (int ti = wid; ti < nti; ti += nw) {
          const int i0 = T0 + 16 * ti, j0 = T0;
          dbl4 acc;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int row = i0 + kq + 4 * q, col = j0 + r16;
            acc[q] = (row < nrows && col < nb && col <= row) ? A[(size_t)row * ld + col] : 0.0;
          }
          const int arow = i0 + r16, bcol = j0 + r16;
          const double a = (arow < nrows) ? -Lp[(size_t)arow * 4 + kq] : 0.0;
          const double b = (bcol < nb && kq < B) ? A[(size_t)bcol * ld + K + kq] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int row = i0 + kq + 4 * q, col = j0 + r16;
            if (row < nrows && col < nb && col <= row) A[(size_t)row * ld + col] = acc[q];
          }
        }
        __syncthreads();
      }
    }
    // rank-16 update of everything right of the block (rows >= nb, columns nb .. n-1)
    if (nb < n) {
      const int BB = nb - KB;
      const int nti = (nrows - nb + 15) / 16, ntj = (n - nb + 15) / 16;
      for (int t = wid; t < nti * ntj; t += nw) {
        const int ti = t / ntj, tj = t - ti * ntj;
        if (tj > ti) continue;
        const int i0 = nb + 16 * ti, j0 = nb + 16 * tj;
        const int arow = i0 + r16, bcol = j0 + r16;
        const double *Ar = A + (size_t)min(arow, nrows - 1) * ld + KB;
        const double *Br = A + (size_t)min(bcol, n - 1) * ld + KB;
        double a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int kk = 4 * u + kq;
          a[u] = (arow < nrows && kk < BB) ? -Ar[kk] * Dv[kk] : 0.0;
          b[u] = (bcol < n && kk < BB) ? Br[kk] : 0.0;
        }
        dbl4 acc;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int row = i0 + kq + 4 * q, col = j0 + r16;
          acc[q] = (row < nrows && col < n && col <= row) ? A[(size_t)row * ld + col] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int row = i0 + kq + 4 * q, col = j0 + r16;
          if (row < nrows && col < n && col <= row) A[(size_t)row * ld + col] = acc[q];
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 1 / d with one Newton step on v_rcp_f64 (the IEEE division sequence is ~2x longer on the serial chain)
__device__ __forceinline__ double frcp1(double d) {
  const double x = __builtin_amdgcn_rcp(d);
  return fma(x, fma(-d, x, 1.0), x);
}

// ---------------------------------------------------------------------------------------------
// LDL^T with the serial chain confined to ONE wavefront and (optionally) the unit-lower inverse built
// alongside, for one workgroup of nw >= 2 waves.  A: the nrows x n lower triangle (rows n .. nrows-1 are
// right-hand-side rows) in a storage layout (SqLayout: ld-strided square, whose upper triangle then holds
// the inverse; PkLayout: packed lower triangle, row i at i(i+1)/2, for the large factors that only fit in
// LDS packed).  Work goes in slots of 16 columns, ONE workgroup barrier per slot:
//   wave 0, slot J : waits (LDS counter) for the helpers' rank-16 update of block column J by block J-1, then
//                    factors the 16 x (nrows - 16 J) panel in registers (lane l owns rows 16 J + l + 64 s): per
//                    column one 16-entry LDS broadcast of the pivot column of the block's own rows, frcp1;
//   waves 1.., slot J: the rank-16 update of block column J by block J-1 first (one MFMA tile per wave,
//                    counted), then that of block columns J+1 .., the 16x16 inverse X_PP = L_PP^-1 of block
//                    P = J-1 (unit lower, quad-parallel, no divisions) and the off-diagonal inverse blocks
//                    of block row I = J-2: X_IK = -X_II sum_{K'=K..I-1} L_IK' X_K'K (MFMA).
// Output: A(i, k) (i > k) = L_u[i][k] (unit-lower LDL factor), Dd[k] = d_k; RHS rows hold D^-1 L_u^-1 b;
// with_inv (SqLayout only): A(j, i) (j < i < n) = X[i][j], X = L_u^-1 (diagonal 1).
// Measured on MI355X (tools/bench_fact.hip, r = 100 with the residual row): 105k cycles for LDL^T + the
// inverse against 161k for ldl_blk16 + ldl_to_chol + a blocked triangular inverse.
// Panel rows per lane <= SMAX: nrows <= 64 SMAX.
struct SqLayout {
  static constexpr bool square = true;
  int ld;
  __device__ __forceinline__ size_t operator()(int i, int j) const { return (size_t)i * ld + j; }
};
struct PkLayout {
  static constexpr bool square = false;
  __device__ __forceinline__ size_t operator()(int i, int j) const { return (size_t)i * (i + 1) / 2 + j; }
};
__host__ __device__ inline size_t packed_lds_doubles(int nrows) { return (size_t)nrows * (nrows + 1) / 2; }

// acc (C layout) of the 16x16 tile at (i0, j0), masked to the stored lower triangle (col <= row)
template <class LA>
__device__ __forceinline__ dbl4 tile_load_lower(const double *A, LA la, int i0, int j0, int nrows, int n, int kq,
                                                int r16) {
  dbl4 acc;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int row = i0 + kq + 4 * q, col = j0 + r16;
    acc[q] = (row < nrows && col < n && col <= row) ? A[la(row, col)] : 0.0;
  }
  return acc;
}
template <class LA>
__device__ __forceinline__ void tile_store_lower(double *A, LA la, int i0, int j0, int nrows, int n, int kq, int r16,
                                                 dbl4 acc) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int row = i0 + kq + 4 * q, col = j0 + r16;
    if (row < nrows && col < n && col <= row) A[la(row, col)] = acc[q];
  }
}
// acc -= L(i0.., oP..) D_P L(j0.., oP..)^T: the rank-16 update by the factored block column P
template <class LA>
__device__ __forceinline__ dbl4 tile_rank16(const double *A, LA la, const double *Dd, int i0, int j0, int oP,
                                            int nrows, int n, int kq, int r16, dbl4 acc) {
  const int arow = min(i0 + r16, nrows - 1), bcol = min(j0 + r16, n - 1);
  const bool av = i0 + r16 < nrows, bv = j0 + r16 < n;
  double a[4], b[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int kk = 4 * u + kq;
    a[u] = av ? -A[la(arow, oP + kk)] * Dd[oP + kk] : 0.0;
    b[u] = bv ? A[la(bcol, oP + kk)] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
  return acc;
}

// One column step K of the wave-resident panel; compile-time loop bounds keep the panel in registers.  The
// pivot column of the block's own rows (lane p holds row oJ + p) reaches every lane by v_readlane (uniform
// values, no LDS round trip): step K receives d and w (column K at rows oJ + p, p > K), computes l for this
// lane, updates the NEXT pivot column first and reads it out of lanes K+1 .. 15 for step K+1 before the bulk
// of its row update.  The reciprocal's Newton step is folded into l (l = l0 + l0 (1 - d x), l0 = v x,
// x = v_rcp_f64(d)).  Lanes <= K take l = 0 (their row is left as it is), without a branch.
// (Two-column steps with a 2x2 pivot block measured slower: the redundant elimination of the second
// column costs more FP64 issue than the saved broadcast.)
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// Software-pipelined: step K receives the pivot's reciprocal x = v_rcp_f64(d_K) and e = 1 - d_K x from step
// K - 1, which issued the reciprocal as soon as d_K was read out (pinned there: the compiler would sink it
// into step K), so its latency runs under the read-out instead of in front of step K; the bulk of the row
// update is issued before the read-out and covers the next pivot column's FMA latency.  With one panel row per
// lane (SMAX = 1) the 16 steps have no branch between them: the whole panel is one scheduling region, and a
// last panel narrower than 16 columns runs its padding steps on zero columns whose results are never stored
// (rcp(0) = inf makes them NaN there; the branch per step cost 20 % of the panel, tools/bench_wave_slots.hip,
// profiles/r05_ldl_panel_pipeline.txt).  With SMAX > 1 the per-step branch stays (removing it measured 7-10 %
// slower there).  Lanes <= K (rows of the diagonal block above the pivot) apply their multiplier to
// upper-triangle entries that are never read out or stored; the pivot lane keeps d_K in its column K.  Every
// stored value is the one the unpipelined step computes (bit-identical factors and inverses).
template <int SMAX, int K>
__device__ __forceinline__ void panel_steps(double (&v)[SMAX][16], int oJ, int n, int lane, double x, double e,
                                            const double (&w)[16]) {
  if constexpr (K < 16) {
    if constexpr (SMAX > 1)
      if (oJ + K >= n) return;
    const double l0 = v[0][K] * x;
    const double l = fma(l0, e, l0);
    v[0][K] = (lane > K) ? l : v[0][K];
    if constexpr (K + 1 < 16) v[0][K + 1] = fma(-l, w[K + 1], v[0][K + 1]);
    // the bulk of the row update first: its issue covers the next pivot column's FMA latency
#pragma unroll
    for (int p = K + 2; p < 16; p++) v[0][p] = fma(-l, w[p], v[0][p]);
#pragma unroll
    for (int s = 1; s < SMAX; s++) {  // rows 64 s + lane: all below the panel's diagonal block
      const double ls0 = v[s][K] * x;
      const double ls = fma(ls0, e, ls0);
      v[s][K] = ls;
#pragma unroll
      for (int p = K + 1; p < 16; p++) v[s][p] = fma(-ls, w[p], v[s][p]);
    }
    double xn = 0.0, en = 0.0, wn[16];
    if constexpr (K + 1 < 16) {
      const double dn = readlane_f64(v[0][K + 1], K + 1);
      xn = __builtin_amdgcn_rcp(dn);
      asm volatile("" : "+v"(xn));
      en = fma(-dn, xn, 1.0);
#pragma unroll
      for (int p = K + 2; p < 16; p++) wn[p] = readlane_f64(v[0][K + 1], p);
    }
    if constexpr (K + 1 < 16) panel_steps<SMAX, K + 1>(v, oJ, n, lane, xn, en, wn);
  }
}

// X[k][c] from lane 4c + (k & 3) of the quad (DPP quad_perm broadcast of both halves)
template <int KK>
__device__ __forceinline__ double quad_bcast(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  constexpr int ctrl = KK * 85;  // quad_perm [KK, KK, KK, KK]
  const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)u, ctrl, 0xf, 0xf, false);
  const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(u >> 32), ctrl, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// steps k = K .. 14 of the quad-parallel unit-lower 16x16 inverse of the block at (o, o) of A (layout la)
template <int K, class LA>
__device__ __forceinline__ void quad_inv_steps(double (&x)[4], const double *A, LA la, int o, int bn, int q) {
  if constexpr (K < 15) {
    const double xk = quad_bcast<(K & 3)>(x[K >> 2]);
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int i = q + 4 * m;
      if (i > K && i < bn) x[m] = fma(-A[la(o + i, o + K)], xk, x[m]);
    }
    quad_inv_steps<K + 1>(x, A, la, o, bn, q);
  }
}

// W > 1 (with SMAX = 1): W panel waves share each 16-column panel.  Every one of them holds the block's own
// 16 rows in lanes 0 .. 15 (the same arithmetic, so the same values: the pivot column reaches each wave by its
// own v_readlane) and 48 further rows in lanes 16 .. 63 (wave w: rows 16 + 48 w ..), so a panel of up to
// 16 + 48 W rows costs one SMAX = 1 column step per column instead of an SMAX = ceil(rows / 64) step; waves
// W .. are the helpers.  Every value is computed exactly as with W = 1.
template <int SMAX, class LA, int W = 1>
__device__ __forceinline__ void ldl_wave_inv(double *A, LA la, int n, int nrows, double *Dd, bool with_inv,
                                             double *Xd = nullptr, long long *prof = nullptr) {
  static_assert(W == 1 || SMAX == 1, "several panel waves hold one slot each");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // this lane's panel row of slot s, relative to the panel's first row
  auto prow = [&](int s) { return W == 1 ? lane + 64 * s : (lane < 16 ? lane : 16 + 48 * wid + lane - 16); };
  const int r16 = lane & 15, kq = lane >> 4;
  const int nb = (n + 15) / 16, nbr = (nrows + 15) / 16;
  if (!LA::square) with_inv = false;
  const int nslot = with_inv ? nb + 2 : (Xd ? nb + 1 : nb);
  __shared__ int colcnt;  // column-update tiles finished so far (helpers -> wave 0)
  __shared__ int pload;   // W > 1: panel waves that have read their panel so far (-> wave 0's store of the block rows)
  if (threadIdx.x == 0) colcnt = 0, pload = 0;
  __syncthreads();
  int coltarget = 0, ptarget = 0;
  for (int J = 0; J < nslot; J++) {
    const int P = J - 1;
    if (P >= 0 && J < nb) coltarget += nbr - J;
    if (W > 1 && J < nb)
      for (int w = 0; w < W; w++) ptarget += (w == 0 || 16 + 48 * w < nrows - 16 * J) ? 1 : 0;
    const long long tslot = prof ? (long long)clock64() : 0;
    if (wid < W) {
      if (J < nb && (wid == 0 || 16 + 48 * wid < nrows - 16 * J)) {
        const int oJ = 16 * J;
        if (P >= 0) {
          while (__hip_atomic_load(&colcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < coltarget)
            __builtin_amdgcn_s_sleep(1);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        double v[SMAX][16];
#pragma unroll
        for (int s = 0; s < SMAX; s++) {
          const int ro = prow(s), i = oJ + ro;
#pragma unroll
          for (int p = 0; p < 16; p++) v[s][p] = (i < nrows && oJ + p < n && p <= ro) ? A[la(i, oJ + p)] : 0.0;
        }
        if (W > 1) {  // this wave's reads of the block rows are done (wave 0 overwrites them with the factor)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_fetch_add(&pload, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        double w0[16];
#pragma unroll
        for (int p = 1; p < 16; p++) w0[p] = readlane_f64(v[0][0], p);
        const double d0 = readlane_f64(v[0][0], 0), x0 = __builtin_amdgcn_rcp(d0);
        panel_steps<SMAX, 0>(v, oJ, n, lane, x0, fma(-d0, x0, 1.0), w0);
        // the pivots: lane p < 16 still holds d_p on its diagonal (step p leaves its own row as it is)
#pragma unroll
        for (int p = 0; p < 16; p++)
          if (wid == 0 && lane == p && oJ + p < n) Dd[oJ + p] = v[0][p];
        // W > 1: every panel wave reads the block's own rows, wave 0 alone writes their factor back; it waits until
        // all have read them (normally long done: the read is the first thing a panel wave does, the factor takes
        // thousands of cycles, but a wave descheduled on a busy CU could otherwise read factored values)
        if (W > 1 && wid == 0) {
          while (__hip_atomic_load(&pload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < ptarget)
            __builtin_amdgcn_s_sleep(1);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
#pragma unroll
        for (int s = 0; s < SMAX; s++) {
          const int ro = prow(s), i = oJ + ro;
          if (W > 1 && wid > 0 && lane < 16) continue;  // the block's own rows: wave 0 stores them
#pragma unroll
          for (int p = 0; p < 16; p++)
            if (i < nrows && oJ + p < n && p < ro) A[la(i, oJ + p)] = v[s][p];
        }
      }
    } else {
      const int nh = nw - W, hw = wid - W;
      // the rank-16 update of block column J by block P (the panel waves wait for it), one tile per helper
      if (P >= 0 && J < nb) {
        for (int I = J + hw; I < nbr; I += nh) {
          dbl4 acc = tile_load_lower(A, la, 16 * I, 16 * J, nrows, n, kq, r16);
          acc = tile_rank16(A, la, Dd, 16 * I, 16 * J, 16 * P, nrows, n, kq, r16, acc);
          tile_store_lower(A, la, 16 * I, 16 * J, nrows, n, kq, r16, acc);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_fetch_add(&colcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      // then: [X_PP] [X_IK, K < I = J-2] [rank-16 tiles (I, C), C >= J+1]
      const bool do_xd = (with_inv || Xd) && P >= 0 && P < nb;
      const int I2 = J - 2;
      const int nxo = (with_inv && I2 >= 1 && I2 < nb) ? I2 : 0;
      int ntr = 0;
      if (P >= 0 && P < nb)
        for (int C = J + 1; C < nb; C++) ntr += nbr - C;
      const int ntask = (do_xd ? 1 : 0) + nxo + ntr;
      for (int t = hw; t < ntask; t += nh) {
        int u = t;
        if (do_xd && u == 0) {
          // X_PP = L_PP^-1 (unit lower), right-looking, no divisions: lane 4c + q keeps column c's entries
          // of rows q + 4m; step k broadcasts X[k][c] inside the quad (DPP) and the rows below update.  To the
          // upper triangle of A (with_inv) and / or as a row-major 16 x 16 block to Xd + 256 P (rows past n:
          // identity)
          const int oP = 16 * P, bn = min(16, n - oP);
          const int c = lane >> 2, q = lane & 3;
          double x[4];
#pragma unroll
          for (int m = 0; m < 4; m++) x[m] = (q + 4 * m == c) ? 1.0 : 0.0;
          quad_inv_steps<0>(x, A, la, oP, bn, q);
#pragma unroll
          for (int m = 0; m < 4; m++) {
            const int i = q + 4 * m;
            if constexpr (LA::square)
              if (with_inv && i > c && i < bn && c < bn) A[(size_t)(oP + c) * la.ld + oP + i] = x[m];
            if (Xd) Xd[(size_t)256 * P + 16 * i + c] = x[m];
          }
          continue;
        }
        u -= do_xd ? 1 : 0;
        if constexpr (LA::square) {
          const int ld = la.ld;
          if (u < nxo) {
            // X_IK = -X_II sum_{K' = K .. I-1} L_IK' X_K'K
            const int I = I2, K = u, oI = 16 * I, oK = 16 * K, ri = oI + r16;
            dbl4 y = {0.0, 0.0, 0.0, 0.0};
            for (int Kp = K; Kp < I; Kp++) {
              const int oKp = 16 * Kp;
              double a[4], b[4];
#pragma unroll
              for (int s = 0; s < 4; s++) {
                const int kp = oKp + 4 * s + kq;  // row of X_K'K = column of L_IK'
                const int j = oK + r16;           // column of X_K'K
                a[s] = (ri < n && kp < n) ? A[(size_t)ri * ld + kp] : 0.0;
                double xb = 0.0;
                if (kp < n && j < n) {
                  if (kp > j)
                    xb = A[(size_t)j * ld + kp];
                  else if (kp == j)
                    xb = 1.0;
                }
                b[s] = xb;
              }
#pragma unroll
              for (int s = 0; s < 4; s++) y = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], y, 0, 0, 0);
            }
            // X_IK = -X_II Y: Y's C layout (register q = Y[kq + 4q][r16]) is the B operand of k-slab q
            dbl4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const int m = oI + 4 * q + kq;  // column of X_II (row ri)
              double xa = 0.0;
              if (ri < n && m < n) {
                if (m < ri)
                  xa = -A[(size_t)m * ld + ri];
                else if (m == ri)
                  xa = -1.0;
              }
              x = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, y[q], x, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const int i = oI + kq + 4 * q, j = oK + r16;
              if (i < n && j < n) A[(size_t)j * ld + i] = x[q];
            }
            continue;
          }
          u -= nxo;
        }
        int C = J + 1;
        while (u >= nbr - C) {
          u -= nbr - C;
          C++;
        }
        const int I = C + u;
        dbl4 acc = tile_load_lower(A, la, 16 * I, 16 * C, nrows, n, kq, r16);
        acc = tile_rank16(A, la, Dd, 16 * I, 16 * C, 16 * P, nrows, n, kq, r16, acc);
        tile_store_lower(A, la, 16 * I, 16 * C, nrows, n, kq, r16, acc);
      }
    }
    if (prof && lane == 0 && (wid == 0 || wid == W) && J < 32) prof[wid ? 32 + J : J] = (long long)clock64() - tslot;
    __syncthreads();
  }
}

// SMAX dispatch: the panel rows one lane owns
template <class LA>
__device__ __forceinline__ void ldl_wave(double *A, LA la, int n, int nrows, double *Dd, bool with_inv) {
  if (nrows <= 64)
    ldl_wave_inv<1>(A, la, n, nrows, Dd, with_inv);
  else if (nrows <= 128)
    ldl_wave_inv<2>(A, la, n, nrows, Dd, with_inv);
  else if (nrows <= 192)
    ldl_wave_inv<3>(A, la, n, nrows, Dd, with_inv);
  else
    ldl_wave_inv<4>(A, la, n, nrows, Dd, with_inv);
}
constexpr int kWaveMaxRows = 256;  // ldl_wave's panel capacity (4 rows per lane)
// The single-workgroup factor kernels (k_ekf_fact, k_info_cholP / Z): 16 waves, W = panel_waves(rows) of them
// share each panel (ldl_wave_inv<1, LA, W>), the rest are helpers.  On MI355X (tools/bench_wave_slots.hip,
// profiles/r04j_ldl_panel_waves.txt) r = 100 with the inverse: 102k -> 89k cycles, r = 135: 126k -> 97k.
constexpr int kFactThreads = 1024;
__host__ __device__ constexpr int panel_waves(int rows) { return rows <= 64 ? 1 : (rows - 16 + 47) / 48; }
static_assert(panel_waves(kWaveMaxRows) <= 5, "panel waves of the largest factor");

}  // namespace uvhp
