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

}  // namespace uvhp
