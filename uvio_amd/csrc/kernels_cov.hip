// gfx950 kernels for the dense covariance P (HBM-resident, row-major, leading dimension ld):
//   EKFPropagation         StateHelper.cpp:36-114
//   clone / augment_clone  StateHelper.cpp:341-391, 579-616
//   marginalize            StateHelper.cpp:271-339
//   measurement compression (UpdaterHelper.cpp:456-487) as CholeskyQR of [H | r]:
//     G = [H r]^T [H r] (tiled FP64, split over row chunks), then the upper Cholesky factor of G is
//     the R factor of the QR of [H r] up to row signs: R = rows of the reference's Givens-compressed
//     [H_x | res] (DESIGN.md "Compression").
//   EKFUpdate              StateHelper.cpp:116-197 as M = P[:,I] H^T, S = H M[I,:] + s2 I = L L^T,
//                          W = M L^-T, P -= W W^T (upper, mirrored), dx = W L^-1 r.
#include <stdexcept>
#include <algorithm>
#include <string>

#include "kernels.h"
#include "dense_lds.h"

namespace uvhp {

static void ensure_lds_attrs();  // large dynamic LDS (> 64 KiB) opt-in, defined at the end

// ----------------------------------------------------------------------------------------------
// EKFPropagation
// T[i][a] = sum_b P[i][iold[b]] * Phi[a][b]    (Cov_PhiT, StateHelper.cpp:80-85)
__global__ void k_prop_T(const double *__restrict__ P, int ld, int N, int p, const int *__restrict__ iold, int q,
                         const double *__restrict__ Phi, double *__restrict__ T) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * p) return;
  int i = idx / p, a = idx % p;
  const double *Pi = P + (size_t)i * ld;
  double acc = 0.0;
  for (int b = 0; b < q; b++) acc += Pi[iold[b]] * Phi[a * q + b];
  T[(size_t)i * p + a] = acc;
}

// rows/cols of the new block <- T, block <- Q(upper-sym) + Phi * T[iold,:]   (StateHelper.cpp:88-101).
// The new block is rows s0 .. s0+p-1, or the listed rows (rows != nullptr): several variables
// propagated at once with a block-row Phi (each row of Phi references only its own variable's inputs).
__global__ void k_prop_write(double *__restrict__ P, int ld, int N, int s0, const int *__restrict__ rows, int p,
                             const int *__restrict__ iold, int q, const double *__restrict__ Phi,
                             const double *__restrict__ Q, const double *__restrict__ T) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * p) return;
  int i = idx / p, a = idx % p;
  int x = -1;
  if (rows) {
    for (int k = 0; k < p; k++)
      if (rows[k] == i) x = k;
  } else if (i >= s0 && i < s0 + p) {
    x = i - s0;
  }
  const int col = rows ? rows[a] : s0 + a;
  if (x >= 0) {
    double acc = (x <= a) ? Q[x * p + a] : Q[a * p + x];
    for (int c = 0; c < q; c++) acc += Phi[x * q + c] * T[(size_t)iold[c] * p + a];
    P[(size_t)i * ld + col] = acc;
  } else {
    double v = T[(size_t)i * p + a];
    P[(size_t)i * ld + col] = v;
    P[(size_t)col * ld + i] = v;
  }
}

void launch_cov_propagate(hipStream_t s, double *P, int ld, int N, int s0, int p, const int *iold, int q,
                          const double *Phi, const double *Q, double *T, const int *rows) {
  int n = N * p, bs = 256, gs = (n + bs - 1) / bs;
  hipLaunchKernelGGL(k_prop_T, dim3(gs), dim3(bs), 0, s, P, ld, N, p, iold, q, Phi, T);
  hipLaunchKernelGGL(k_prop_write, dim3(gs), dim3(bs), 0, s, P, ld, N, s0, rows, p, iold, q, Phi, Q, T);
}

// ----------------------------------------------------------------------------------------------
// clone of the 6-dof IMU pose (ids src0..src0+5) appended at N, plus the time-offset cross term
__global__ void k_clone(double *__restrict__ P, int ld, int N, int src0, int dt_id, const double *__restrict__ dnc,
                        int do_dt) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (N + 6) * 6) return;
  int i = idx / 6, b = idx % 6;
  double db = do_dt ? dnc[b] : 0.0;
  if (i < N) {
    double col = P[(size_t)i * ld + src0 + b];
    double row = P[(size_t)(src0 + b) * ld + i];
    if (do_dt) {
      col += P[(size_t)i * ld + dt_id] * db;
      row += db * P[(size_t)dt_id * ld + i];
    }
    P[(size_t)i * ld + N + b] = col;
    P[(size_t)(N + b) * ld + i] = row;
  } else {
    int a = i - N;
    double v = P[(size_t)(src0 + a) * ld + src0 + b];
    if (do_dt) {
      double da = dnc[a];
      v += P[(size_t)(src0 + a) * ld + dt_id] * db;
      v += da * (P[(size_t)dt_id * ld + src0 + b] + P[(size_t)dt_id * ld + dt_id] * db);
    }
    P[(size_t)i * ld + N + b] = v;
  }
}

// EKFPropagation of the contiguous block s0 .. s0+p-1 and the IMU-pose clone in ONE workgroup launch: the three
// phases above (T, the block write, the clone) with a workgroup barrier between them instead of a kernel
// boundary, each element computed by the same expression as in k_prop_T / k_prop_write / k_clone (so the
// result is bit-identical).  For the propagations of N p <= 8192 and p, q <= 32
// (cfg2-4): the frame loses two launches.
constexpr int kPropCloneThreads = 512, kPropCloneMaxEl = 16, kPropCloneMaxPQ = 32;
__global__ void __launch_bounds__(kPropCloneThreads) k_prop_clone(double *__restrict__ P, int ld, int N, int s0, int p,
                                                                  const int *__restrict__ iold, int q,
                                                                  const double *__restrict__ Phi,
                                                                  const double *__restrict__ Q, double *__restrict__ T,
                                                                  int src0, int dt_id, const double *__restrict__ dnc,
                                                                  int do_dt) {
  // Phi, Q and the column map in LDS; T rows of the block (rows iold[c]) also kept in LDS for the block write
  __shared__ double sPhi[kPropCloneMaxPQ * kPropCloneMaxPQ], sQ[kPropCloneMaxPQ * kPropCloneMaxPQ],
      sT[kPropCloneMaxPQ * kPropCloneMaxPQ];
  __shared__ int siold[kPropCloneMaxPQ];
  for (int e = threadIdx.x; e < p * q; e += blockDim.x) sPhi[e] = Phi[e];
  for (int e = threadIdx.x; e < p * p; e += blockDim.x) sQ[e] = Q[e];
  for (int e = threadIdx.x; e < q; e += blockDim.x) siold[e] = iold[e];
  __syncthreads();
  // T, one covariance row per thread: the row's q inputs loaded at once (one memory round trip), then its p
  // outputs eight at a time (independent sums side by side); each output's sum runs over b in ascending order,
  // as in k_prop_T
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const double *Pi = P + (size_t)i * ld;
    double pv[kPropCloneMaxPQ];
    int ci = -1;  // this row's position in the column map (a row of the propagated block)
#pragma unroll
    for (int b = 0; b < kPropCloneMaxPQ; b++) {
      pv[b] = (b < q) ? Pi[siold[b]] : 0.0;
      if (b < q && siold[b] == i) ci = b;
    }
    for (int a0 = 0; a0 < p; a0 += 8) {
      double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int b = 0; b < kPropCloneMaxPQ; b++) {
        if (b < q) {
#pragma unroll
          for (int u = 0; u < 8; u++) acc[u] += pv[b] * sPhi[min(a0 + u, p - 1) * q + b];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (a0 + u < p) {
          T[(size_t)i * p + a0 + u] = acc[u];
          if (ci >= 0) sT[ci * p + a0 + u] = acc[u];
        }
      }
    }
  }
  __syncthreads();
  // the block rows / columns, eight elements per thread and round: every load of a round before its stores
  constexpr int U = 8;
  for (int base = threadIdx.x; base < N * p; base += U * blockDim.x) {
    double tv[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int idx = base + u * blockDim.x;
      tv[u] = (idx < N * p) ? T[idx] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int idx = base + u * blockDim.x;
      if (idx >= N * p) continue;
      const int i = idx / p, a = idx % p, col = s0 + a;
      if (i >= s0 && i < s0 + p) {
        const int x = i - s0;
        double acc = (x <= a) ? sQ[x * p + a] : sQ[a * p + x];
        for (int c = 0; c < q; c++) acc += sPhi[x * q + c] * sT[c * p + a];
        P[(size_t)i * ld + col] = acc;
      } else {
        P[(size_t)i * ld + col] = tv[u];
        P[(size_t)col * ld + i] = tv[u];
      }
    }
  }
  __syncthreads();
  // the clone's rows / columns N .. N+5 (reads never touch them): a round's values first, then its stores
  for (int base = threadIdx.x; base < (N + 6) * 6; base += U * blockDim.x) {
    double vc[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int idx = base + u * blockDim.x;
      vc[u] = vr[u] = 0.0;
      if (idx >= (N + 6) * 6) continue;
      const int i = idx / 6, b = idx % 6;
      const double db = do_dt ? dnc[b] : 0.0;
      if (i < N) {
        double col = P[(size_t)i * ld + src0 + b];
        double row = P[(size_t)(src0 + b) * ld + i];
        if (do_dt) {
          col += P[(size_t)i * ld + dt_id] * db;
          row += db * P[(size_t)dt_id * ld + i];
        }
        vc[u] = col;
        vr[u] = row;
      } else {
        const int a = i - N;
        double v = P[(size_t)(src0 + a) * ld + src0 + b];
        if (do_dt) {
          const double da = dnc[a];
          v += P[(size_t)(src0 + a) * ld + dt_id] * db;
          v += da * (P[(size_t)dt_id * ld + src0 + b] + P[(size_t)dt_id * ld + dt_id] * db);
        }
        vc[u] = v;
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int idx = base + u * blockDim.x;
      if (idx >= (N + 6) * 6) continue;
      const int i = idx / 6, b = idx % 6;
      P[(size_t)i * ld + N + b] = vc[u];
      if (i < N) P[(size_t)(N + b) * ld + i] = vr[u];
    }
  }
}

bool launch_prop_clone(hipStream_t s, double *P, int ld, int N, int s0, int p, const int *iold, int q,
                       const double *Phi, const double *Q, double *T, int src0, int dt_id, const double *dnc_dev,
                       int do_dt) {
  if (N * p > kPropCloneMaxEl * kPropCloneThreads || p > kPropCloneMaxPQ || q > kPropCloneMaxPQ) return false;
  hipLaunchKernelGGL(k_prop_clone, dim3(1), dim3(kPropCloneThreads), 0, s, P, ld, N, s0, p, iold, q, Phi, Q, T, src0,
                     dt_id, dnc_dev, do_dt);
  return true;
}

void launch_clone(hipStream_t s, double *P, int ld, int N, int src0, int dt_id, const double *dnc_dev, int do_dt) {
  int n = (N + 6) * 6, bs = 256, gs = (n + bs - 1) / bs;
  hipLaunchKernelGGL(k_clone, dim3(gs), dim3(bs), 0, s, P, ld, N, src0, dt_id, dnc_dev, do_dt);
}

// ----------------------------------------------------------------------------------------------
__global__ void k_marginalize(const double *__restrict__ P, double *__restrict__ Po, int ld, int N, int m0, int ms) {
  int Nn = N - ms;
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  int i = blockIdx.y;
  if (j >= Nn || i >= Nn) return;
  int mi = i < m0 ? i : i + ms, mj = j < m0 ? j : j + ms;
  double v;
  if (i >= m0 && j < m0)
    v = P[(size_t)j * ld + mi];  // Cov_new(x2,x1) = Cov_new(x1,x2)^T (StateHelper.cpp:303-304)
  else
    v = P[(size_t)mi * ld + mj];
  Po[(size_t)i * ld + j] = v;
}

void launch_marginalize(hipStream_t s, const double *P, double *Pout, int ld, int N, int m0, int ms) {
  int Nn = N - ms;
  if (Nn <= 0) return;
  hipLaunchKernelGGL(k_marginalize, dim3((Nn + 127) / 128, Nn), dim3(128), 0, s, P, Pout, ld, N, m0, ms);
}

// several variables at once: Po (Nn x Nn) = P[src, src] (P is exactly symmetric: both triangles are written
// with the same values by every update, so the gather equals the sequence of single marginalizations)
__global__ void k_compact(const double *__restrict__ P, double *__restrict__ Po, int ld, int Nn, const int *__restrict__ src) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y;
  if (j >= Nn || i >= Nn) return;
  Po[(size_t)i * ld + j] = P[(size_t)src[i] * ld + src[j]];
}
void launch_compact(hipStream_t s, const double *P, double *Pout, int ld, int Nn, const int *src) {
  if (Nn <= 0) return;
  hipLaunchKernelGGL(k_compact, dim3((Nn + 127) / 128, Nn), dim3(128), 0, s, P, Pout, ld, Nn, src);
}

// StateHelper::marginalize (StateHelper.cpp:271-339) of several variables in one launch, with the result of the
// sequence of single marginalizations: each one copies its lower-left block from the transposed upper-right
// (Cov_new(x2,x1) = Cov_new(x1,x2)^T), so a lower element (i > j) of the final matrix comes from the upper
// triangle exactly when some marginalized index lies between the kept pair, i.e. when more indices were removed
// before src[i] than before src[j] (src[i] - i > src[j] - j); any order of the sequence gives the same matrix.
__global__ void k_marginalize_multi(const double *__restrict__ P, double *__restrict__ Po, int ld, int Nn,
                                    const int *__restrict__ src) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y;
  if (j >= Nn || i >= Nn) return;
  const int si = src[i], sj = src[j];
  const bool flip = i > j && si - i > sj - j;
  Po[(size_t)i * ld + j] = flip ? P[(size_t)sj * ld + si] : P[(size_t)si * ld + sj];
}
void launch_marginalize_multi(hipStream_t s, const double *P, double *Pout, int ld, int Nn, const int *src) {
  if (Nn <= 0) return;
  hipLaunchKernelGGL(k_marginalize_multi, dim3((Nn + 127) / 128, Nn), dim3(128), 0, s, P, Pout, ld, Nn, src);
}

__global__ void k_check_diag(const double *__restrict__ P, int ld, int N, int *neg) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N && P[(size_t)i * ld + i] < 0.0) atomicAdd(neg, 1);
}
void launch_check_diag(hipStream_t s, const double *P, int ld, int N, int *neg) {
  hipLaunchKernelGGL(k_check_diag, dim3((N + 255) / 256), dim3(256), 0, s, P, ld, N, neg);
}

// ----------------------------------------------------------------------------------------------
// Compression: Gram partials.  Grid: (upper tile pairs, row chunks).  Tile 32x32, 256 threads,
// each thread 2x2 outputs.  A is m x ncol, row-major, ld = ldh.
constexpr int GT = 32;         // tile edge
constexpr int GCHUNK = 512;    // rows per chunk
constexpr int GCHUNK_SMALL = 64, GSMALL_ROWS = 2048;  // stacks up to 2048 rows: 64-row chunks

// Rows per chunk of the VALU Gram.  A small stack (cfg2's ~500 rows) in 512-row chunks is one chunk: ~10
// workgroups each walking 16 dependent row slabs; 64-row chunks give ~8x the workgroups of two slabs each,
// and the fixed-order reduction adds the chunk partials.
static int gram_chunk_rows(int m) { return m <= GSMALL_ROWS ? GCHUNK_SMALL : GCHUNK; }
int gram_num_chunks(int m) { return (m + gram_chunk_rows(m) - 1) / gram_chunk_rows(m); }

__global__ void __launch_bounds__(256) k_gram(const double *__restrict__ A, int m, int ncol, int ldh, int crows,
                                              double *__restrict__ partials) {
  __shared__ double As[GT][GT + 1];
  __shared__ double Bs[GT][GT + 1];
  int nt = (ncol + GT - 1) / GT;
  // work index = chunk * pairs + pair, XCD-swizzled (a chunk's tile pairs share one L2); decode the upper
  // tile pair (ti <= tj)
  const int npairs = nt * (nt + 1) / 2, wid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int chunk = wid / npairs;
  int pair = wid - chunk * npairs, ti = 0;
  while (pair >= nt - ti) {
    pair -= nt - ti;
    ti++;
  }
  int tj = ti + pair;
  int r0 = chunk * crows, r1 = min(m, r0 + crows);
  int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
  double acc[2][2] = {{0, 0}, {0, 0}};
  for (int rb = r0; rb < r1; rb += GT) {
    for (int e = threadIdx.x; e < GT * GT; e += 256) {
      int rr = e / GT, cc = e % GT;
      int row = rb + rr;
      int ca = ti * GT + cc, cb = tj * GT + cc;
      As[rr][cc] = (row < r1 && ca < ncol) ? A[(size_t)row * ldh + ca] : 0.0;
      Bs[rr][cc] = (row < r1 && cb < ncol) ? A[(size_t)row * ldh + cb] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < GT; k++) {
      double a0 = As[k][ty], a1 = As[k][ty + 16];
      double b0 = Bs[k][tx], b1 = Bs[k][tx + 16];
      acc[0][0] += a0 * b0;
      acc[0][1] += a0 * b1;
      acc[1][0] += a1 * b0;
      acc[1][1] += a1 * b1;
    }
    __syncthreads();
  }
  double *out = partials + (size_t)chunk * ncol * ncol;
  for (int u = 0; u < 2; u++)
    for (int v = 0; v < 2; v++) {
      int a = ti * GT + ty + 16 * u, b = tj * GT + tx + 16 * v;
      if (a < ncol && b < ncol) out[(size_t)a * ncol + b] = acc[u][v];
    }
}

// The Gram of a large stack (configs 4-5: ~80k rows x 173-243 columns) on the matrix cores: a 256-thread
// workgroup owns a 64 x 64 upper tile pair of G for one chunk of GCHUNK_BIG rows; rows run in slabs of
// 32 staged in LDS (the two 16 x 64 column blocks of the slab), each wave accumulates a 32 x 32 quarter
// with four v_mfma_f64_16x16x4_f64 tiles (A operand = the slab transposed: k = row).  The next slab's
// loads are issued before the current slab's MFMAs.  Partials: same layout as k_gram (chunk-major,
// every entry a <= b written).
constexpr int GB = 64, GK = 32, GCHUNK_BIG = 1024;
__global__ void __launch_bounds__(256) k_gram_mfma(const double *__restrict__ A, int m, int ncol, int ldh,
                                                   double *__restrict__ partials) {
  __shared__ double Xs[GK][GB + 1];
  __shared__ double Ys[GK][GB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int nt = (ncol + GB - 1) / GB, npairs = nt * (nt + 1) / 2;
  // work index = chunk * npairs + pair, XCD-swizzled: a chunk's tile pairs share one XCD's L2
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), chunk = wid / npairs;
  int pair = wid - chunk * npairs, ti = 0;
  while (pair >= nt - ti) {
    pair -= nt - ti;
    ti++;
  }
  const int tj = ti + pair;
  const int c0i = ti * GB, c0j = tj * GB;
  const int r0 = chunk * GCHUNK_BIG, r1 = min(m, r0 + GCHUNK_BIG);
  constexpr int NU = GK / 4;  // slab elements per thread
  double rx[NU], ry[NU];
  auto load = [&](int rb) {
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int e = tid + 256 * u, row = rb + (e >> 6), c = e & 63;
      rx[u] = (row < r1 && c0i + c < ncol) ? A[(size_t)row * ldh + c0i + c] : 0.0;
      ry[u] = (row < r1 && c0j + c < ncol) ? A[(size_t)row * ldh + c0j + c] : 0.0;
    }
  };
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(r0);
  for (int rb = r0; rb < r1; rb += GK) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int e = tid + 256 * u;
      Xs[e >> 6][e & 63] = rx[u];
      Ys[e >> 6][e & 63] = ry[u];
    }
    __syncthreads();
    if (rb + GK < r1) load(rb + GK);
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[t] = Xs[kk + kq][32 * wr + 16 * t + r16];
        b[t] = Ys[kk + kq][32 * wc + 16 * t + r16];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ta++)
#pragma unroll
        for (int tb = 0; tb < 2; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
  }
  double *out = partials + (size_t)chunk * ncol * ncol;
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 2; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int a = c0i + 32 * wr + 16 * ta + kq + 4 * q, b = c0j + 32 * wc + 16 * tb + r16;
        if (a < ncol && b < ncol) out[(size_t)a * ncol + b] = acc[ta][tb][q];
      }
}

void launch_gram(hipStream_t s, const double *A, int m, int ncol, int ldh, double *partials, int *nchunks_out) {
  if (m >= 8 * GCHUNK_BIG) {
    const int ntb = (ncol + GB - 1) / GB, nchb = (m + GCHUNK_BIG - 1) / GCHUNK_BIG;
    *nchunks_out = nchb;
    hipLaunchKernelGGL(k_gram_mfma, dim3(ntb * (ntb + 1) / 2 * nchb), dim3(256), 0, s, A, m, ncol, ldh, partials);
    return;
  }
  int nt = (ncol + GT - 1) / GT;
  int pairs = nt * (nt + 1) / 2;
  int nch = gram_num_chunks(m);
  *nchunks_out = nch;
  hipLaunchKernelGGL(k_gram, dim3(pairs * nch), dim3(256), 0, s, A, m, ncol, ldh, gram_chunk_rows(m), partials);
}

// Feature sharding: one rank's contribution to the all-reduced information block.  Upper triangle of the
// rank's Gram (chunks summed in fixed order; the lower triangle is written as zero so the reduced buffer is
// defined everywhere), then the accepted-feature count and the accepted rows of the rank's batch.
__global__ void __launch_bounds__(256) k_shard_pack(const double *__restrict__ partials, int nch, int ncol,
                                                    const DFeatOut *__restrict__ fout, int nf,
                                                    const int *__restrict__ acc, double *__restrict__ buf) {
  const int nn = ncol * ncol;
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nn) {
    int a = e / ncol, b = e % ncol;
    double v = 0.0;
    if (a <= b)
      for (int c = 0; c < nch; c++) v += partials[(size_t)c * nn + e];
    buf[e] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // one wavefront: accepted rows of the batch
    int rows = 0;
    for (int i = threadIdx.x; i < nf; i += 64)
      if (fout[i].status == 0) rows += fout[i].rows;
    for (int o = 32; o > 0; o >>= 1) rows += __shfl_down(rows, o, 64);
    if (threadIdx.x == 0) {
      buf[nn] = (nf > 0) ? (double)*acc : 0.0;
      buf[nn + 1] = (double)rows;
    }
  }
}

__global__ void k_shard_unpack(const double *__restrict__ buf, int ncol, int *__restrict__ acc) {
  if (threadIdx.x == 0) *acc = (int)(buf[ncol * ncol] + 0.5);
}

void launch_shard_pack(hipStream_t s, const double *partials, int nch, int ncol, const DFeatOut *fout, int nf,
                       const int *acc, double *buf) {
  int nn = ncol * ncol;
  hipLaunchKernelGGL(k_shard_pack, dim3((nn + 255) / 256), dim3(256), 0, s, partials, nch, ncol, fout, nf, acc, buf);
}

void launch_shard_unpack(hipStream_t s, const double *buf, int ncol, int *acc) {
  hipLaunchKernelGGL(k_shard_unpack, dim3(1), dim3(64), 0, s, buf, ncol, acc);
}

// Sum partials (fixed chunk order) into the upper triangle of G, then upper Cholesky G = R^T R.
// G lives in `W` (LDS when it fits, else global scratch `gbuf`). Pivots <= tol*G_jj give zero rows.
__global__ void __launch_bounds__(1024) k_gram_reduce_chol(const double *__restrict__ partials, int nch, int ncol,
                                                           double *__restrict__ R, int ldr, double *gbuf, int use_lds) {
  extern __shared__ double lds[];
  double *G = use_lds ? lds : gbuf;
  __shared__ double piv;
  __shared__ int zero_row;
  int n = ncol;
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    int a = e / n, b = e % n;
    double acc = 0.0;
    if (b >= a)
      for (int c = 0; c < nch; c++) acc += partials[(size_t)c * n * n + e];
    G[e] = acc;
  }
  __syncthreads();
  // keep the original diagonal for the rank tolerance in the (unused) lower-left corner
  for (int k = 0; k < n; k++) {
    if (threadIdx.x == 0) {
      double d = G[k * n + k];
      double g0 = 0.0;
      // original diagonal recomputed from partials (cheap: one entry)
      for (int c = 0; c < nch; c++) g0 += partials[(size_t)c * n * n + k * n + k];
      if (d > 1e-13 * g0 && d > 0.0) {
        piv = sqrt(d);
        zero_row = 0;
      } else {
        piv = 0.0;
        zero_row = 1;
      }
      G[k * n + k] = piv;
    }
    __syncthreads();
    // row k of R: R[k][j] = G[k][j] / piv
    for (int j = k + 1 + threadIdx.x; j < n; j += blockDim.x) G[k * n + j] = zero_row ? 0.0 : G[k * n + j] / piv;
    __syncthreads();
    // trailing update G[i][j] -= R[k][i] R[k][j] for k < i <= j
    int m = n - k - 1;
    int tot = m * m;
    for (int e = threadIdx.x; e < tot; e += blockDim.x) {
      int i = k + 1 + e / m, j = k + 1 + e % m;
      if (j >= i) G[i * n + j] -= G[k * n + i] * G[k * n + j];
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    int a = e / n, b = e % n;
    R[(size_t)a * ldr + b] = (b >= a) ? G[e] : 0.0;
  }
}

void launch_gram_reduce_chol(hipStream_t s, const double *partials, int nchunks, int ncol, double *R, int ldr) {
  size_t bytes = (size_t)ncol * ncol * sizeof(double);
  int use_lds = bytes <= 150 * 1024;
  // global scratch for large ncol lives right after R (caller sizes R for 2 * ncol^2)
  double *gbuf = R + (size_t)ncol * ldr;
  ensure_lds_attrs();
  hipLaunchKernelGGL(k_gram_reduce_chol, dim3(1), dim3(1024), use_lds ? bytes : 0, s, partials, nchunks, ncol, R, ldr,
                     gbuf, use_lds);
}

// Inverses of the 16x16 diagonal blocks of a lower-triangular L (r x r, ld): one 64-lane workgroup per
// block stages the block in LDS (one load round), then lane c < 16 forms column c by forward
// substitution.  Dinv: block b at Dinv + 256 b, row-major.  Rows past r are treated as identity.
__global__ void __launch_bounds__(64) k_trinv16(const double *__restrict__ L, int ld, int r, double *__restrict__ Dinv) {
  __shared__ double Lb[16][17];
  const int b = blockIdx.x, l = threadIdx.x, o = 16 * b;
  const int nb = min(16, r - o);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int e = l + 64 * q, i = e >> 4, k = e & 15;
    Lb[i][k] = (i < nb && k <= i) ? L[(size_t)(o + i) * ld + o + k] : 0.0;
  }
  __syncthreads();
  if (l >= 16) return;
  const int c = l;
  double x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    if (i < c) {
      x[i] = 0.0;
    } else if (i >= nb) {
      x[i] = (i == c) ? 1.0 : 0.0;
    } else {
      double acc = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < i; k++)
        if (k >= c) acc -= Lb[i][k] * x[k];
      x[i] = acc / Lb[i][i];
    }
  }
#pragma unroll
  for (int i = 0; i < 16; i++) Dinv[(size_t)256 * b + i * 16 + c] = x[i];
}

// W (N x r, ld r) = M L^-T, i.e. W L^T = M, blocked by 16 columns with the matrix cores:
//   tile = M[:, p] - W[:, <p] L[p, <p]^T   (v_mfma_f64_16x16x4_f64 over the solved columns)
//   W[:, p] = tile Dinv_p^T                 (4 MFMAs with the diagonal block inverse)
// One 64-lane workgroup per 16 rows of M; the solved part of its rows stays in LDS.  Loads are batched so
// that few memory round trips sit on the block chain: the column map is staged in LDS once, the next block's
// M tile is loaded while the current one is solved, and L (L2-resident) is read 64 columns (16 loads per
// lane) per batch before their 16 MFMAs (one round trip per batch instead of one per 16 columns).  The
// accumulation order is the plain ascending k order either way.  With hidx, M is read as P[row][hidx[k]]
// (ldm = ldp), i.e. the columns P[:, I] of the covariance.
constexpr int kTrsmMaxR = 264;
__global__ void __launch_bounds__(64) k_trsm_lt(const double *__restrict__ M, int ldm, const int *__restrict__ hidx, int N,
                                                int r, const double *__restrict__ L, int ldl,
                                                const double *__restrict__ Dinv, double *__restrict__ W) {
  __shared__ double Wt[16][kTrsmMaxR + 1];
  __shared__ double Tt[16][17];
  __shared__ int hs[kTrsmMaxR];
  const int l = threadIdx.x, r16 = l & 15, kq = l >> 4;
  const int row0 = blockIdx.x * 16;
  if (hidx)
    for (int k = l; k < r; k += 64) hs[k] = hidx[k];
  __syncthreads();
  auto load_m = [&](int j0, double (&m)[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = row0 + kq + 4 * q, col = j0 + r16;
      m[q] = (row < N && col < r) ? (hidx ? M[(size_t)row * ldm + hs[col]] : M[(size_t)row * ldm + col]) : 0.0;
    }
  };
  double mnext[4];
  load_m(0, mnext);
  for (int j0 = 0; j0 < r; j0 += 16) {
    dbl4 acc;
#pragma unroll
    for (int q = 0; q < 4; q++) acc[q] = mnext[q];
    if (j0 + 16 < r) load_m(j0 + 16, mnext);  // in flight while this block is solved
    // a column jj >= r of the last block reads row r - 1 of L (finite): its tile column is never stored, and
    // its contribution to the valid columns goes through Dinv[j][m] with m > j, which is 0 (lower triangular)
    const int jj = j0 + r16;
    const double *Lj = L + (size_t)min(jj, r - 1) * ldl;
    int k0 = 0;
    for (; k0 + 64 <= j0; k0 += 64) {  // 64 solved columns per batch: 16 L loads per lane in flight
      double a[16], b[16];
#pragma unroll
      for (int u = 0; u < 16; u++) b[u] = Lj[k0 + 4 * u + kq];  // unconditional: see below
#pragma unroll
      for (int u = 0; u < 16; u++) a[u] = -Wt[r16][k0 + 4 * u + kq];
#pragma unroll
      for (int u = 0; u < 16; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
    }
    for (; k0 < j0; k0 += 16) {  // j0 is a multiple of 16
      double a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        a[u] = -Wt[r16][k0 + 4 * u + kq];
        b[u] = Lj[k0 + 4 * u + kq];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
    }
    // acc (C layout) -> A-operand layout through LDS
#pragma unroll
    for (int q = 0; q < 4; q++) Tt[kq + 4 * q][r16] = acc[q];
    __syncthreads();
    dbl4 w = {0.0, 0.0, 0.0, 0.0};
    const double *Db = Dinv + (size_t)256 * (j0 / 16);
#pragma unroll
    for (int m0 = 0; m0 < 16; m0 += 4) {
      const double a = Tt[r16][m0 + kq];
      const double b = Db[r16 * 16 + m0 + kq];  // B[m][j] = Dinv[j][m]
      w = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, w, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int rr = kq + 4 * q, col = j0 + r16;
      if (col < r) {
        Wt[rr][col] = w[q];
        if (row0 + rr < N) W[(size_t)(row0 + rr) * r + col] = w[q];
      }
    }
    __syncthreads();
  }
}

void launch_trsm_lt(hipStream_t s, const double *M, int ldm, const int *hidx, int N, int r, const double *L, int ldl,
                    double *Dinv, double *W, bool form_dinv) {
  if (r > kTrsmMaxR) throw std::runtime_error("triangular solve wider than the kernel's LDS row");
  if (form_dinv) hipLaunchKernelGGL(k_trinv16, dim3((r + 15) / 16), dim3(64), 0, s, L, ldl, r, Dinv);
  hipLaunchKernelGGL(k_trsm_lt, dim3((N + 15) / 16), dim3(64), 0, s, M, ldm, hidx, N, r, L, ldl, Dinv, W);
}

// ----------------------------------------------------------------------------------------------
// Information-form EKF update for compressed (m > n) batches.
//
// The reference compresses [H | r] with Givens (UpdaterHelper.cpp:456-487) and runs EKFUpdate on the
// n x n R factor.  EKFUpdate depends on R only through G = R^T R = H^T H and b = R^T z = H^T r:
//   P+ = P - P[:,I] (G P_II + s2 I)^-1 G P[I,:],   dx = P[:,I] (G P_II + s2 I)^-1 b
// (push-through identity on K = P H^T (H P H^T + s2 I)^-1).  G is the fixed-order Gram of the stacked
// rows; no factor of G is formed, so the gauge directions in which H is exactly singular (cond ~1e17 on
// real MSCKF batches) stay at rounding level instead of picking up sqrt(eps)-sized rows the way a
// Cholesky factor of a singular Gram does.  The eigenvalues of G P_II + s2 I are >= s2, so the LU solve
// below is well conditioned.

// the upper triangle of G (ncol x ncol, ld = ncol) from the chunk partials (upper triangles, fixed chunk
// order).  One workgroup row per G row a: thread b >= a reads the partials' (a, b) entries (coalesced along the
// row, only the upper triangle is fetched) and writes G[a][b].  The lower triangle is never written: its one
// consumer (k_gemm_mfma with symA) reads G[b][a] for b < a -- a mirror store here wrote one double per cache
// line (PMC r03t: 0.20 MB written for an 82 KB G at cfg2).
__global__ void __launch_bounds__(256) k_gram_reduce(const double *__restrict__ partials, int nch, int ncol,
                                                     double *__restrict__ G, int *zero) {
  const int a = blockIdx.y, b = blockIdx.x * blockDim.x + threadIdx.x;
  if (zero && a == 0 && b == 0) *zero = 0;  // the update's negative-diagonal count
  if (b < a || b >= ncol) return;
  const size_t u = (size_t)a * ncol + b, stride = (size_t)ncol * ncol;
  double acc = 0.0;
  int c = 0;
  for (; c + 4 <= nch; c += 4) {  // four loads in flight, the sum in chunk order
    const double p0 = partials[c * stride + u], p1 = partials[(c + 1) * stride + u];
    const double p2 = partials[(c + 2) * stride + u], p3 = partials[(c + 3) * stride + u];
    acc += p0;
    acc += p1;
    acc += p2;
    acc += p3;
  }
  for (; c < nch; c++) acc += partials[c * stride + u];
  G[u] = acc;
}

// C (m x n) = op(A) op(B); op(X) = X or X^T.  The small dense products of the information form (E = L^T G L,
// (n+1)^2 with n ~ 100-243) on the matrix cores: one 16 x 16 output tile per wave (v_mfma_f64_16x16x4f64,
// eight k-slabs loaded ahead of their MFMAs).  tri = 1: B is lower triangular (k >= j0 only), tri = 2:
// op(A) is upper triangular (k >= i0 only) -- the zero blocks of the triangular factor are skipped.  symA: A is
// symmetric with only its upper triangle stored (element (i, k) read at (min, max)).  Like k_info_P the
// workgroups run on kGemmXcds XCDs only (each reads both operands into its L2).
constexpr int kGemmWaves = 4, kGemmXcds = 2;
__global__ void __launch_bounds__(64 * kGemmWaves) k_gemm_mfma(int ta, int tb, int tri, int symA, int m, int n, int k,
                                                              const double *__restrict__ A, int lda,
                                                              const double *__restrict__ B, int ldb,
                                                              double *__restrict__ C, int ldc) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int ntj = (n + 15) / 16;
  const int nwg = ((m + 15) / 16 * ntj + kGemmWaves - 1) / kGemmWaves, per = (nwg + kGemmXcds - 1) / kGemmXcds;
  const int xcd = blockIdx.x % 8, wg = xcd * per + blockIdx.x / 8;
  if (xcd >= kGemmXcds || wg >= nwg || wg >= (xcd + 1) * per) return;
  const int tile = wg * kGemmWaves + wid, ti = tile / ntj, tj = tile - ti * ntj;
  const int i0 = 16 * ti, j0 = 16 * tj;
  if (i0 >= m) return;  // a whole wave (no barriers in this kernel)
  const int ia = min(i0 + r16, m - 1), jb = min(j0 + r16, n - 1);
  const bool iv = i0 + r16 < m, jv = j0 + r16 < n;
  const int kbeg = tri == 1 ? j0 : tri == 2 ? i0 : 0;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = tile_chain(
      kbeg, k, kq,
      [&](int kk) {
        if (!iv) return 0.0;
        if (symA) return A[(size_t)min(ia, kk) * lda + max(ia, kk)];
        return ta ? A[(size_t)kk * lda + ia] : A[(size_t)ia * lda + kk];
      },
      [&](int kk) { return jv ? (tb ? B[(size_t)jb * ldb + kk] : B[(size_t)kk * ldb + jb]) : 0.0; }, acc);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int row = i0 + kq + 4 * q, col = j0 + r16;
    if (row < m && col < n) C[(size_t)row * ldc + col] = acc[q];
  }
}
static void launch_gemm_mfma(hipStream_t s, int ta, int tb, int tri, int symA, int m, int n, int k, const double *A,
                             int lda, const double *B, int ldb, double *C, int ldc) {
  const int tiles = ((m + 15) / 16) * ((n + 15) / 16), nwg = (tiles + kGemmWaves - 1) / kGemmWaves;
  hipLaunchKernelGGL(k_gemm_mfma, dim3(8 * ((nwg + kGemmXcds - 1) / kGemmXcds)), dim3(64 * kGemmWaves), 0, s, ta, tb, tri, symA,
                     m, n, k, A, lda, B, ldb, C, ldc);
}

// Single-workgroup Cholesky factors of the information-form update (dense_lds.h ldl_wave: one wave
// factors each 16-column panel, the other waves do the rank-16 updates).  Storage mode: 0 = square in
// LDS, 1 = packed lower triangle in LDS (n up to ~195), 2 = square in the global scratch gbuf.
// L_c = L_u D^1/2; an extra right-hand-side row b leaves as L_c^-1 b = D^1/2 (D^-1 L_u^-1 b).
// Dinv: the inverses of L_c's 16 x 16 diagonal blocks for k_trsm_lt (k_trinv16's layout: block b row-major at
// Dinv + 256 b, rows past n identity), D^-1/2 times the unit-lower block inverses the factorization forms
// on its helper waves -- the solve that follows needs no k_trinv16 launch.
template <int W, class LA>
__device__ __forceinline__ void info_chol_body(double *A, LA la, double *Dd, int n, int nrows, double *Dinv) {
  ldl_wave_inv<1, LA, W>(A, la, n, nrows, Dd, false, Dinv);
  for (int k = threadIdx.x; k < n; k += blockDim.x) Dd[k] = sqrt(Dd[k]);  // sqrt(d)
  __syncthreads();
  const int nb = (n + 15) / 16;
  for (int e = threadIdx.x; e < 256 * nb; e += blockDim.x) {
    const int row = 16 * (e >> 8) + ((e >> 4) & 15);
    if (row < n) Dinv[e] = Dinv[e] / Dd[row];
  }
}

// P_II = P[hidx, hidx] = L_P L_P^T.  Writes Laug = diag(L_P, 1) ((n+1) x (n+1), zero upper) and L_P (n x n).
// MODE: the storage (compile-time, so LDS accesses are DS instructions rather than FLAT)
template <int W, int MODE>
__global__ void __launch_bounds__(kFactThreads) k_info_cholP(const double *__restrict__ P, int ldp, const int *__restrict__ hidx,
                                                    int n, double *__restrict__ Laug, double *__restrict__ Lout,
                                                    double *gbuf, int mode, double *__restrict__ Dinv) {
  constexpr int PACKED = MODE == 1;
  extern __shared__ double lds[];
  double *A = (MODE == 2) ? gbuf : lds;
  (void)mode;
  const int ld = n | 1;
  const size_t asz = PACKED ? packed_lds_doubles(n) : (size_t)n * ld;
  double *Dd = A + asz;
  auto idx = [&](int a, int b) { return PACKED ? (size_t)a * (a + 1) / 2 + b : (size_t)a * ld + b; };
  staged_copy(
      n * n,
      [&](int e) {
        const int a = e / n, b = e - a * n;
        return (b <= a) ? P[(size_t)hidx[a] * ldp + hidx[b]] : 0.0;
      },
      [&](int e, double v) {
        const int a = e / n, b = e - a * n;
        if (b <= a) A[idx(a, b)] = v;
      });
  __syncthreads();
  if constexpr (PACKED)
    info_chol_body<W>(A, PkLayout{}, Dd, n, n, Dinv);
  else
    info_chol_body<W>(A, SqLayout{ld}, Dd, n, n, Dinv);
  const int na = n + 1;
  for (int e = threadIdx.x; e < na * na; e += blockDim.x) {
    const int a = e / na, b = e - a * na;
    double v = 0.0;
    if (a < n && b < n) v = (b < a) ? A[idx(a, b)] * Dd[b] : (b == a ? Dd[a] : 0.0);
    else if (a == n && b == n) v = 1.0;
    Laug[e] = v;
    if (a < n && b < n) Lout[(size_t)a * n + b] = v;
  }
}

// [E c; c^T .] = Laug^T G Laug;  Z = E + s2 I = U U^T with the augmented row c^T -> w = U^-1 c.
// Writes U (n x n, ld n) and w (n).
template <int W, int MODE>
__global__ void __launch_bounds__(kFactThreads) k_info_cholZ(const double *__restrict__ E, int n, double s2,
                                                    double *__restrict__ Uout, double *__restrict__ w, double *gbuf,
                                                    int mode, double *__restrict__ Dinv) {
  constexpr int PACKED = MODE == 1;
  extern __shared__ double lds[];
  double *A = (MODE == 2) ? gbuf : lds;
  (void)mode;
  const int ld = n | 1;
  const int na = n + 1;
  const size_t asz = PACKED ? packed_lds_doubles(na) : (size_t)na * ld;
  double *Dd = A + asz;
  auto idx = [&](int a, int b) { return PACKED ? (size_t)a * (a + 1) / 2 + b : (size_t)a * ld + b; };
  staged_copy(
      (n + 1) * n,
      [&](int e) {
        const int a = e / n, b = e - a * n;
        return (b <= a) ? E[(size_t)a * na + b] + ((a == b) ? s2 : 0.0) : 0.0;
      },
      [&](int e, double v) {
        const int a = e / n, b = e - a * n;
        if (b <= a) A[idx(a, b)] = v;
      });
  __syncthreads();
  if constexpr (PACKED)
    info_chol_body<W>(A, PkLayout{}, Dd, n, n + 1, Dinv);
  else
    info_chol_body<W>(A, SqLayout{ld}, Dd, n, n + 1, Dinv);
  for (int j = threadIdx.x; j < n; j += blockDim.x) w[j] = A[idx(n, j)] * Dd[j];
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    const int a = e / n, b = e - a * n;
    Uout[e] = (b < a) ? A[idx(a, b)] * Dd[b] : (b == a ? Dd[a] : 0.0);
  }
}
// the instantiation for a factor of `rows` rows (panel rows per lane) and storage mode
template <class KP>
static KP pick_info_kernel(const KP (&tab)[5][3], int rows, int mode) {
  return tab[panel_waves(rows) - 1][mode];
}
typedef void (*CholPFn)(const double *, int, const int *, int, double *, double *, double *, int, double *);
typedef void (*CholZFn)(const double *, int, double, double *, double *, double *, int, double *);
static const CholPFn kCholP[5][3] = {{k_info_cholP<1, 0>, k_info_cholP<1, 1>, k_info_cholP<1, 2>},
                                     {k_info_cholP<2, 0>, k_info_cholP<2, 1>, k_info_cholP<2, 2>},
                                     {k_info_cholP<3, 0>, k_info_cholP<3, 1>, k_info_cholP<3, 2>},
                                     {k_info_cholP<4, 0>, k_info_cholP<4, 1>, k_info_cholP<4, 2>},
                                     {k_info_cholP<5, 0>, k_info_cholP<5, 1>, k_info_cholP<5, 2>}};
static const CholZFn kCholZ[5][3] = {{k_info_cholZ<1, 0>, k_info_cholZ<1, 1>, k_info_cholZ<1, 2>},
                                     {k_info_cholZ<2, 0>, k_info_cholZ<2, 1>, k_info_cholZ<2, 2>},
                                     {k_info_cholZ<3, 0>, k_info_cholZ<3, 1>, k_info_cholZ<3, 2>},
                                     {k_info_cholZ<4, 0>, k_info_cholZ<4, 1>, k_info_cholZ<4, 2>},
                                     {k_info_cholZ<5, 0>, k_info_cholZ<5, 1>, k_info_cholZ<5, 2>}};

// storage mode and dynamic LDS bytes of an info-form factor of nrows x n (+ the n doubles of D)
static int info_chol_mode(int nrows, int n, size_t *bytes) {
  const size_t sq = ((size_t)nrows * (n | 1) + n) * sizeof(double);
  const size_t pk = (packed_lds_doubles(nrows) + n) * sizeof(double);
  if (sq <= (size_t)kMaxDynLds) {
    *bytes = sq;
    return 0;
  }
  if (pk <= (size_t)kMaxDynLds) {
    *bytes = pk;
    return 1;
  }
  *bytes = 0;
  return 2;
}


// ---- the information-form factors too large for LDS (n + 1 rows beyond the packed triangle, cfg5: 243): split ----
// Mode 2 ran the one-workgroup factor out of global memory (cfg5: P_II 350 us, Z 290 us per launch).  The split runs
// the same right-looking LDL^T in four launches, every stored value the one the one-workgroup factor computes:
//   1  the first n1 columns (a multiple of 16) over ALL rows in LDS, the rows below n1 held in a trapezoid layout
//      (ldl_wave_inv treats them as right-hand-side rows: the same panel steps and rank-16 tiles as in the full
//      factor); L_u of those columns and their raw pivots to global memory (G, Dg), their diagonal-block inverses;
//   2  the trailing block's Schur complement A22 - L21 D1 L21^T, tile by tile: the source value, then the rank-16
//      updates by blocks 0 .. n1/16 - 1 in order, four MFMAs each with tile_rank16's operands (-L d, L) -- the chain
//      the one-workgroup factor applies to those tiles, with the same intermediate values;
//   3  the trailing block (n - n1 columns, N - n1 rows) factored in LDS, packed, its pivots and block inverses;
//   4  info_chol_body's epilogue (sqrt of the pivots, the scaled block inverses) and the kernel's outputs.
// SRC 0: P[hidx, hidx] (k_info_cholP), 1: E + s2 I with the augmented row (k_info_cholZ).
struct TrapLayout {  // rows < n1: packed lower triangle; rows >= n1: n1 columns at an odd stride
  static constexpr bool square = false;
  int n1, ld;
  size_t base;
  __device__ __forceinline__ size_t operator()(int i, int j) const {
    return i < n1 ? (size_t)i * (i + 1) / 2 + j : base + (size_t)(i - n1) * ld + j;
  }
};
__host__ __device__ inline size_t trap_lds_doubles(int N, int n1) {
  return (size_t)n1 * (n1 + 1) / 2 + (size_t)(N - n1) * (n1 | 1) + n1;  // + the pivots
}
template <int SRC>
__device__ __forceinline__ double info_src(const double *src, int lds_, const int *hidx, double s2, int a, int b) {
  if (SRC == 0) return src[(size_t)hidx[a] * lds_ + hidx[b]];
  return src[(size_t)a * lds_ + b] + ((a == b) ? s2 : 0.0);
}
template <int W, int SRC>
__global__ void __launch_bounds__(kFactThreads) k_info_split1(const double *__restrict__ src, int lds_,
                                                              const int *__restrict__ hidx, double s2, int N, int n1,
                                                              double *__restrict__ G, int ldg, double *__restrict__ Dg,
                                                              double *__restrict__ Dinv) {
  extern __shared__ double lds[];
  const TrapLayout la{n1, n1 | 1, (size_t)n1 * (n1 + 1) / 2};
  double *A = lds, *Dd = lds + la.base + (size_t)(N - n1) * la.ld;
  staged_copy(
      N * n1,
      [&](int e) {
        const int a = e / n1, b = e - a * n1;
        return (b <= a) ? info_src<SRC>(src, lds_, hidx, s2, a, b) : 0.0;
      },
      [&](int e, double v) {
        const int a = e / n1, b = e - a * n1;
        if (b <= a) A[la(a, b)] = v;
      });
  __syncthreads();
  ldl_wave_inv<1, TrapLayout, W>(A, la, n1, N, Dd, false, Dinv);
  for (int e = threadIdx.x; e < N * n1; e += blockDim.x) {
    const int a = e / n1, b = e - a * n1;
    if (b < a) G[(size_t)a * ldg + b] = A[la(a, b)];
  }
  for (int k = threadIdx.x; k < n1; k += blockDim.x) Dg[k] = Dd[k];
}
// one wave per 16 x 16 lower tile (I, C) of the trailing block (rows n1 .. N - 1, columns n1 .. n - 1)
template <int SRC>
__global__ void __launch_bounds__(256) k_info_split_schur(const double *__restrict__ src, int lds_,
                                                         const int *__restrict__ hidx, double s2, int N, int n, int n1,
                                                         double *__restrict__ G, int ldg, const double *__restrict__ Dg) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const int nbr = (N - n1 + 15) / 16, nbc = (n - n1 + 15) / 16;
  int t = blockIdx.x * 4 + (threadIdx.x >> 6), I = 0;
  // lower tiles (I, C), C <= min(I, nbc - 1), row-major
  while (I < nbr && t >= min(I, nbc - 1) + 1) {
    t -= min(I, nbc - 1) + 1;
    I++;
  }
  if (I >= nbr) return;
  const int C = t, i0 = n1 + 16 * I, j0 = n1 + 16 * C;
  dbl4 acc;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int row = i0 + kq + 4 * q, col = j0 + r16;
    acc[q] = (row < N && col < n && col <= row) ? info_src<SRC>(src, lds_, hidx, s2, row, col) : 0.0;
  }
  const int arow = min(i0 + r16, N - 1), bcol = min(j0 + r16, n - 1);
  const bool av = i0 + r16 < N, bv = j0 + r16 < n;
  for (int oP = 0; oP < n1; oP += 16) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int kk = oP + 4 * u + kq;
      a[u] = av ? -G[(size_t)arow * ldg + kk] * Dg[kk] : 0.0;
      b[u] = bv ? G[(size_t)bcol * ldg + kk] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int row = i0 + kq + 4 * q, col = j0 + r16;
    if (row < N && col < n && col <= row) G[(size_t)row * ldg + col] = acc[q];
  }
}
template <int W>
__global__ void __launch_bounds__(kFactThreads) k_info_split3(double *__restrict__ G, int ldg, int N, int n, int n1,
                                                              double *__restrict__ Dg, double *__restrict__ Dinv) {
  extern __shared__ double lds[];
  const int m = n - n1, R = N - n1;
  double *A = lds, *Dd = lds + packed_lds_doubles(R);
  const PkLayout la{};
  staged_copy(
      R * m,
      [&](int e) {
        const int a = e / m, b = e - a * m;
        return (b <= a) ? G[(size_t)(n1 + a) * ldg + n1 + b] : 0.0;
      },
      [&](int e, double v) {
        const int a = e / m, b = e - a * m;
        if (b <= a) A[la(a, b)] = v;
      });
  __syncthreads();
  ldl_wave_inv<1, PkLayout, W>(A, la, m, R, Dd, false, Dinv + (size_t)256 * (n1 / 16));
  for (int e = threadIdx.x; e < R * m; e += blockDim.x) {
    const int a = e / m, b = e - a * m;
    if (b < a) G[(size_t)(n1 + a) * ldg + n1 + b] = A[la(a, b)];
  }
  for (int k = threadIdx.x; k < m; k += blockDim.x) Dg[n1 + k] = Dd[k];
}
// info_chol_body's epilogue and the factor kernel's outputs.  OUT 0 (k_info_cholP): Laug, Lout; 1 (k_info_cholZ):
// U (out0), w (out1, the augmented row).  Dg: the raw pivots, replaced by their square roots.
template <int OUT>
__global__ void __launch_bounds__(256) k_info_split_out(const double *__restrict__ G, int ldg, int n,
                                                       double *__restrict__ Dg, double *__restrict__ Dinv,
                                                       double *__restrict__ out0, double *__restrict__ out1) {
  __shared__ double Ds[kWaveMaxRows];
  for (int k = threadIdx.x; k < n; k += blockDim.x) Ds[k] = sqrt(Dg[k]);
  __syncthreads();
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  const int nb = (n + 15) / 16;
  for (int e = tid; e < 256 * nb; e += nth) {
    const int row = 16 * (e >> 8) + ((e >> 4) & 15);
    if (row < n) Dinv[e] = Dinv[e] / Ds[row];
  }
  if (OUT == 0) {
    const int na = n + 1;
    for (int e = tid; e < na * na; e += nth) {
      const int a = e / na, b = e - a * na;
      double v = 0.0;
      if (a < n && b < n) v = (b < a) ? G[(size_t)a * ldg + b] * Ds[b] : (b == a ? Ds[a] : 0.0);
      else if (a == n && b == n) v = 1.0;
      out0[e] = v;
      if (a < n && b < n) out1[(size_t)a * n + b] = v;
    }
  } else {
    for (int j = tid; j < n; j += nth) out1[j] = G[(size_t)n * ldg + j] * Ds[j];
    for (int e = tid; e < n * n; e += nth) {
      const int a = e / n, b = e - a * n;
      out0[e] = (b < a) ? G[(size_t)a * ldg + b] * Ds[b] : (b == a ? Ds[a] : 0.0);
    }
  }
  // the pivots' square roots are written back only after every block has read the raw ones: not needed, Dg is
  // scratch (each block forms its own Ds)
}
typedef void (*Split1Fn)(const double *, int, const int *, double, int, int, double *, int, double *, double *);
typedef void (*Split3Fn)(double *, int, int, int, int, double *, double *);
static const Split1Fn kSplit1[2][5] = {
    {k_info_split1<1, 0>, k_info_split1<2, 0>, k_info_split1<3, 0>, k_info_split1<4, 0>, k_info_split1<5, 0>},
    {k_info_split1<1, 1>, k_info_split1<2, 1>, k_info_split1<3, 1>, k_info_split1<4, 1>, k_info_split1<5, 1>}};
static const Split3Fn kSplit3[5] = {k_info_split3<1>, k_info_split3<2>, k_info_split3<3>, k_info_split3<4>,
                                    k_info_split3<5>};
// the split's first block: the widest multiple of 16 whose trapezoid fits in LDS and leaves a trailing block that
// fits packed; 0 when there is none
static int info_split_n1(int N, int n) {
  for (int n1 = (n - 1) / 16 * 16; n1 >= 16; n1 -= 16) {
    const size_t t1 = trap_lds_doubles(N, n1) * sizeof(double);
    const size_t t3 = (packed_lds_doubles(N - n1) + (n - n1)) * sizeof(double);
    if (t1 <= (size_t)kMaxDynLds && t3 <= (size_t)kMaxDynLds) return n1;
  }
  return 0;
}
// the factor of an N x n matrix (N = n or n + 1) from SRC through the split; G (ld ldg) and Dg scratch
template <int SRC, int OUT>
static void launch_info_split(hipStream_t s, int n1, const double *src, int lds_, const int *hidx, double s2, int N,
                              int n, double *G, int ldg, double *Dg, double *Dinv, double *out0, double *out1) {
  static bool attrs = false;
  if (!attrs) {
    for (int w = 0; w < 5; w++)
      if (set_dyn_lds((const void *)kSplit1[SRC][w], kMaxDynLds) < kMaxDynLds ||
          set_dyn_lds((const void *)kSplit3[w], kMaxDynLds) < kMaxDynLds)
        throw std::runtime_error("dynamic LDS limit not granted for the split information-form factor");
    attrs = true;
  }
  hipLaunchKernelGGL(kSplit1[SRC][panel_waves(N) - 1], dim3(1), dim3(kFactThreads), trap_lds_doubles(N, n1) * sizeof(double),
                     s, src, lds_, hidx, s2, N, n1, G, ldg, Dg, Dinv);
  const int nbr = (N - n1 + 15) / 16, nbc = (n - n1 + 15) / 16;
  int tiles = 0;
  for (int I = 0; I < nbr; I++) tiles += std::min(I, nbc - 1) + 1;
  hipLaunchKernelGGL(k_info_split_schur<SRC>, dim3((tiles + 3) / 4), dim3(256), 0, s, src, lds_, hidx, s2, N, n, n1, G,
                     ldg, Dg);
  hipLaunchKernelGGL(kSplit3[panel_waves(N - n1) - 1], dim3(1), dim3(kFactThreads),
                     (packed_lds_doubles(N - n1) + (n - n1)) * sizeof(double), s, G, ldg, N, n, n1, Dg, Dinv);
  hipLaunchKernelGGL(k_info_split_out<OUT>, dim3(32), dim3(256), 0, s, G, ldg, n, Dg, Dinv, out0, out1);
}

// P[i][j] -= sum_k V[i][k] V[j][k] - s2 sum_k X[i][k] X[j][k]  for j >= i, mirrored;  dx = X w;
// negative-diagonal count.   (P+ = P - V (I - s2 Z^-1) V^T, see launch_ekf_info)
// Grid over the upper 16 x 16 tile pairs (bi <= bj) of P, 4 waves: wave w accumulates both products over the
// k-slabs w, w + 4, ... on the matrix cores (four slabs' loads issued ahead of their MFMAs), the waves' partial
// tiles are added in LDS in a fixed order.  The tile pairs run on kInfoPXcds of the 8 XCDs (blocks labelled
// blockIdx % 8 >= kInfoPXcds exit at once), each XCD a contiguous range of pairs: every XCD that runs tiles
// reads nearly all of V and X into its own L2, so eight XCDs fetched them eight times (PMC r03o: 4.2 MB per
// launch at cfg2 against 1.2 MB of operands).
constexpr int kInfoPXcds = 2;
__global__ void __launch_bounds__(256) k_info_P(double *__restrict__ P, int ldp, int N, const double *__restrict__ V,
                                                const double *__restrict__ X, int n, double s2,
                                                const double *__restrict__ w, double *__restrict__ dx, int *neg,
                                                const int *gate, int nb) {
  const int xcd = blockIdx.x % 8, npair = nb * (nb + 1) / 2, per = (npair + kInfoPXcds - 1) / kInfoPXcds;
  int b = xcd * per + blockIdx.x / 8;
  if (xcd >= kInfoPXcds || b >= npair || b >= (xcd + 1) * per) return;
  if (gate && *gate == 0) return;  // no accepted rows: the reference makes no update
  __shared__ double red[2][4][256];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  int bi = 0;
  while (b >= nb - bi) {
    b -= nb - bi;
    bi++;
  }
  const int bj = bi + b;
  // this thread's P element, fetched before the products so its latency is hidden
  const int ei = threadIdx.x >> 4, ej = threadIdx.x & 15;
  const int gi = 16 * bi + ei, gj = 16 * bj + ej;
  const bool pw = gi < N && gj < N && (bi < bj || ej >= ei);
  const double pv = pw ? P[(size_t)gi * ldp + gj] : 0.0;
  const int ri = 16 * bi + r16, rj = 16 * bj + r16;
  const bool vi = ri < N, vj = rj < N;
  const double *Vi = V + (size_t)min(ri, N - 1) * n, *Vj = V + (size_t)min(rj, N - 1) * n;
  const double *Xi = X + (size_t)min(ri, N - 1) * n, *Xj = X + (size_t)min(rj, N - 1) * n;
  dbl4 av = {0.0, 0.0, 0.0, 0.0}, ax = {0.0, 0.0, 0.0, 0.0};
  constexpr int U = 4;
  for (int k0 = 4 * wid; k0 < n; k0 += 16 * U) {
    double a0[U], b0[U], a1[U], b1[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = k0 + 16 * u + kq;
      const bool in = k < n;
      a0[u] = (in && vi) ? Vi[k] : 0.0;
      b0[u] = (in && vj) ? Vj[k] : 0.0;
      a1[u] = (in && vi) ? Xi[k] : 0.0;
      b1[u] = (in && vj) ? Xj[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (k0 + 16 * u < n) {
        av = mfma4(a0[u], b0[u], av);
        ax = mfma4(a1[u], b1[u], ax);
      }
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    red[0][wid][(kq + 4 * q) * 16 + r16] = av[q];
    red[1][wid][(kq + 4 * q) * 16 + r16] = ax[q];
  }
  __syncthreads();
  if (pw) {
    const int e = threadIdx.x;
    const double sv = (red[0][0][e] + red[0][1][e]) + (red[0][2][e] + red[0][3][e]);
    const double sx = (red[1][0][e] + red[1][1][e]) + (red[1][2][e] + red[1][3][e]);
    const double v = pv - (sv - s2 * sx);
    P[(size_t)gi * ldp + gj] = v;
    P[(size_t)gj * ldp + gi] = v;
    if (gi == gj && v < 0.0) atomicAdd(neg, 1);
  }
  if (bi == bj && wid == 1) {
    const int i = lane >> 2, part = lane & 3, row = 16 * bi + i;
    double a = 0.0;
    if (row < N)
      for (int k = part; k < n; k += 4) a += X[(size_t)row * n + k] * w[k];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (part == 0 && row < N) dx[row] = a;
  }
}

// Compressed update in information form on the Gram G = [H r]^T [H r]:
//   P_II = L L^T,  E = L^T G_nn L,  c = L^T b,  Z = E + s2 I = U U^T,  V = P[:,I] L^-T,  X = V U^-T
//   P+ = P - V V^T + s2 X X^T  (= P - P[:,I] (G P_II + s2 I)^-1 G P[I,:]),   dx = X U^-1 c.
// Z has eigenvalues >= s2, so both Cholesky factors are of SPD matrices and G itself is never
// factored (it is exactly singular in the gauge directions of an MSCKF stack).
//
// The chain splits at the Gram: the prefactor (P_II = L L^T and V = P[:,I] L^-T) reads only P and the
// column map, both fixed once the batch's columns are known, so the engine runs it on a side stream while
// the feature group forms the rows (launch_ekf_info_pre); launch_ekf_info_post is the rest.
// Scratch: sc.S holds Laug | L_P | T1 | E | U (5 (n+1)^2), sc.M holds V (and is cholP's global work buffer
// before that), sc.W is cholZ's global work buffer and then X, sc.Dinv the diagonal-block inverses.
void launch_ekf_info_pre(hipStream_t s, const double *P, int ldp, int N, int n, const int *hidx, EkfScratch &sc) {
  const int na = n + 1;
  double *Laug = sc.S;
  double *Lf = Laug + (size_t)na * na;
  ensure_lds_attrs();
  if (n + 1 > kWaveMaxRows) throw std::runtime_error("information-form update wider than the factorization panel");
  size_t b1 = 0;
  const int m1 = info_chol_mode(n, n, &b1);
  static const bool no_split = std::getenv("UVIO_HP_NO_INFO_SPLIT") != nullptr;  // A/B: the global-memory factor
  const int s1 = (m1 == 2 && !no_split) ? info_split_n1(n, n) : 0;
  if (s1 > 0)  // the raw pivots in T1 (free until the post half)
    launch_info_split<0, 0>(s, s1, P, ldp, hidx, 0.0, n, n, sc.M, n | 1, Lf + (size_t)n * n, sc.Dinv, Laug, Lf);
  else
    hipLaunchKernelGGL(pick_info_kernel(kCholP, n, m1), dim3(1), dim3(kFactThreads), b1, s, P, ldp, hidx, n, Laug, Lf,
                       sc.M, m1, sc.Dinv);
  launch_trsm_lt(s, P, ldp, hidx, N, n, Lf, n, sc.Dinv, sc.M, false);  // V = P[:,I] L^-T
}

void launch_ekf_info_post(hipStream_t s, double *P, int ldp, int N, const double *partials, int nch, int n,
                          double sigma2, double *Gbuf, EkfScratch &sc) {
  const int na = n + 1;
  hipLaunchKernelGGL(k_gram_reduce, dim3((na + 255) / 256, na), dim3(256), 0, s, partials, nch, na, Gbuf, sc.neg);
  double *Laug = sc.S;                            // (n+1)^2
  double *Lf = Laug + (size_t)na * na;            // n^2   L_P
  double *T1 = Lf + (size_t)n * n;                // (n+1)^2
  double *E = T1 + (size_t)na * na;               // (n+1)^2
  double *Uf = E + (size_t)na * na;               // n^2   U   (5 (n+1)^2 in total)
  double *w = sc.y;
  launch_gemm_mfma(s, 0, 0, 1, 1, na, na, na, Gbuf, na, Laug, na, T1, na);  // G Laug (G upper-stored, Laug lower)
  launch_gemm_mfma(s, 1, 0, 2, 0, na, na, na, Laug, na, T1, na, E, na);     // Laug^T (G Laug)
  size_t b2 = 0;
  const int m2 = info_chol_mode(n + 1, n, &b2);
  static const bool no_split = std::getenv("UVIO_HP_NO_INFO_SPLIT") != nullptr;
  const int s2 = (m2 == 2 && !no_split) ? info_split_n1(n + 1, n) : 0;
  if (s2 > 0)  // the raw pivots in T1 (consumed by the second product above)
    launch_info_split<1, 1>(s, s2, E, na, nullptr, sigma2, n + 1, n, sc.W, n | 1, T1, sc.Dinv, Uf, w);
  else
    hipLaunchKernelGGL(pick_info_kernel(kCholZ, n + 1, m2), dim3(1), dim3(kFactThreads), b2, s, E, n, sigma2, Uf, w, sc.W,
                       m2, sc.Dinv);
  launch_trsm_lt(s, sc.M, n, nullptr, N, n, Uf, n, sc.Dinv, sc.W, false);  // X = V U^-T
  const int nb = (N + 15) / 16;
  const int per = (nb * (nb + 1) / 2 + kInfoPXcds - 1) / kInfoPXcds;
  hipLaunchKernelGGL(k_info_P, dim3(8 * per), dim3(256), 0, s, P, ldp, N, sc.M, sc.W, n, sigma2, w, sc.dx, sc.neg,
                     sc.gate, nb);
}

void launch_ekf_info(hipStream_t s, double *P, int ldp, int N, const double *partials, int nch, int n,
                     const int *hidx, double sigma2, double *Gbuf, EkfScratch &sc) {
  launch_ekf_info_pre(s, P, ldp, N, n, hidx, sc);
  launch_ekf_info_post(s, P, ldp, N, partials, nch, n, sigma2, Gbuf, sc);
}

// StateHelper::initialize_invertible (StateHelper.cpp:484-577) for a 3-dof landmark appended at N:
// M = P[:, hidx] Hx^T is in sc.M (N x 3, from launch_ekf_M); Hx (3 x n, ld), HLinv (3x3, device), s2.
// With fout (delayed init enqueued behind its feature group): H_Linv is the inverse of the feature's
// H_finit (DFeatOut::HfR), formed here with the host's cofactor formula, and the whole step is skipped
// when the gate (the batch's accepted-feature count) is 0.
__global__ void k_init_invertible(double *__restrict__ P, int ldp, int N, const double *__restrict__ M,
                                  const double *__restrict__ Hx, int ldh, int n, const int *__restrict__ hidx,
                                  const double *__restrict__ HLinv_in, double s2, const DFeatOut *__restrict__ fout,
                                  const int *__restrict__ gate, double *__restrict__ resout) {
  __shared__ double S3[9], PLL[9], Hinv[9];
  if (resout && blockIdx.x == 0 && threadIdx.x < 3) resout[threadIdx.x] = Hx[(size_t)threadIdx.x * ldh + n];
  if (gate && *gate == 0) return;
  if (threadIdx.x == 0) {
    if (fout)
      inv3_cofactor(fout->HfR, Hinv);
    else
      for (int k = 0; k < 9; k++) Hinv[k] = HLinv_in[k];
  }
  __syncthreads();
  const double *HLinv = Hinv;
  int t = threadIdx.x + blockIdx.x * blockDim.x;
  if (blockIdx.x == 0) {
    // S3 = Hx M[hidx, :] + s2 I: each of the 9 entries summed by 28 threads over strided k, the 28
    // partials then added in fixed order (blockDim = 256 >= 9 x 28)
    __shared__ double part[9][28];
    const int e = threadIdx.x / 28, j = threadIdx.x % 28;
    if (e < 9) {
      const int a = e / 3, b = e % 3;
      double acc = 0.0;
      for (int k = j; k < n; k += 28) acc += Hx[(size_t)a * ldh + k] * M[(size_t)hidx[k] * 3 + b];
      part[e][j] = acc;
    }
    __syncthreads();
    if (threadIdx.x < 9) {
      const int a = threadIdx.x / 3, b = threadIdx.x % 3;
      double acc = 0.0;
      for (int q = 0; q < 28; q++) acc += part[threadIdx.x][q];
      // M.selfadjointView<Upper>(): use the upper element for both halves
      S3[threadIdx.x] = acc + (a == b ? s2 : 0.0);
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 9) {
    int a = threadIdx.x / 3, b = threadIdx.x % 3;
    double acc = 0.0;
    for (int c = 0; c < 3; c++)
      for (int e = 0; e < 3; e++) {
        double sce = (c <= e) ? S3[c * 3 + e] : S3[e * 3 + c];
        acc += HLinv[a * 3 + c] * sce * HLinv[b * 3 + e];
      }
    PLL[threadIdx.x] = acc;
  }
  __syncthreads();
  if (t < N * 3) {
    int i = t / 3, a = t % 3;
    double acc = 0.0;
    for (int b = 0; b < 3; b++) acc += M[(size_t)i * 3 + b] * HLinv[a * 3 + b];
    P[(size_t)i * ldp + N + a] = -acc;
    P[(size_t)(N + a) * ldp + i] = -acc;
  }
  if (blockIdx.x == 0 && threadIdx.x < 9) {
    int a = threadIdx.x / 3, b = threadIdx.x % 3;
    P[(size_t)(N + a) * ldp + N + b] = PLL[threadIdx.x];
  }
}

void launch_init_invertible(hipStream_t s, double *P, int ldp, int N, const double *Hx, int ldh, int n,
                            const int *hidx, const double *HLinv, double s2, EkfScratch &sc, const DFeatOut *fout,
                            const int *gate, double *resout) {
  launch_ekf_M(s, P, ldp, N, Hx, ldh, 3, n, hidx, sc.M, nullptr);
  int nt = N * 3;
  hipLaunchKernelGGL(k_init_invertible, dim3((nt + 255) / 256), dim3(256), 0, s, P, ldp, N, sc.M, Hx, ldh, n, hidx,
                     HLinv, s2, fout, gate, resout);
}

static void ensure_lds_attrs() {
  static bool done = false;
  if (done) return;
  if (set_dyn_lds((const void *)k_gram_reduce_chol, 150 * 1024) < 150 * 1024)
    throw std::runtime_error("dynamic LDS limit not granted for k_gram_reduce_chol");
  for (int a = 0; a < 5; a++)
    for (int b = 0; b < 2; b++)
      if (set_dyn_lds((const void *)kCholP[a][b], kMaxDynLds) < kMaxDynLds ||
          set_dyn_lds((const void *)kCholZ[a][b], kMaxDynLds) < kMaxDynLds)
        throw std::runtime_error("dynamic LDS limit not granted for an information-form factor kernel");
  done = true;
}

}  // namespace uvhp
