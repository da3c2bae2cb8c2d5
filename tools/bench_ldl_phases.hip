// Phase split of ldl_blk16 (dense_lds.h) on one workgroup: cycles in the diagonal-block, panel,
// block-column and trailing-update phases (thread 0's clock64 after each barrier).  The body below is
// ldl_blk16 with the timers added.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_ldl_phases.hip -o build/bench_ldl_phases
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "dense_lds.h"
using namespace uvhp;

__device__ void ldl_blk16_prof(double *A, int ld, int n, int nrows, double *Lp, long long *pf) {
  long long tq = clock64();
#define TQ(k) if (threadIdx.x == 0) { long long t2 = clock64(); pf[k] += t2 - tq; tq = t2; }
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
      __syncthreads(); TQ(0)  // every wave has read the diagonal block before the panel rows overwrite it
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
      __syncthreads(); TQ(1)
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
        __syncthreads(); TQ(2)
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
      __syncthreads(); TQ(3)
    }
  }
}
#undef TQ

__global__ void __launch_bounds__(1024) k_test(const double *Ain, int n, int nrows, long long *pf) {
  extern __shared__ double lds[];
  const int ld = n | 1;
  double *A = lds, *wsp = lds + (size_t)nrows * ld;
  for (int e = threadIdx.x; e < nrows * n; e += blockDim.x) A[(e / n) * ld + e % n] = Ain[e];
  __syncthreads();
  long long t0 = clock64();
  ldl_blk16_prof(A, ld, n, nrows, wsp, pf);
  __syncthreads();
  if (threadIdx.x == 0) pf[7] = clock64() - t0;
}

int main(int argc, char **argv) {
  int n = argc > 1 ? atoi(argv[1]) : 101;
  int nt = argc > 2 ? atoi(argv[2]) : 512;
  int nrows = n + 1;
  std::vector<double> A(nrows * n), B(n * n);
  srand(n);
  for (auto &x : B) x = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = (i == j) ? 0.1 : 0;
      for (int k = 0; k < n; k++) s += B[i * n + k] * B[j * n + k];
      A[i * n + j] = s;
    }
  for (int j = 0; j < n; j++) A[n * n + j] = (double)rand() / RAND_MAX - 0.5;
  double *dA;
  long long *dpf;
  (void)hipMalloc(&dA, 8 * nrows * n);
  (void)hipMalloc(&dpf, 8 * 8);
  (void)hipMemcpy(dA, A.data(), 8 * nrows * n, hipMemcpyHostToDevice);
  size_t bytes = (size_t)nrows * (n | 1) * 8 + (size_t)(4 * nrows) * 8;
  (void)hipFuncSetAttribute((const void *)k_test, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024);
  for (int it = 0; it < 3; it++) {
    (void)hipMemset(dpf, 0, 64);
    hipLaunchKernelGGL(k_test, dim3(1), dim3(nt), bytes, 0, dA, n, nrows, dpf);
    (void)hipDeviceSynchronize();
  }
  long long pf[8];
  (void)hipMemcpy(pf, dpf, 64, hipMemcpyDeviceToHost);
  printf("n=%d nt=%d total %lld cyc: diag %lld  panel %lld  blockcol %lld  trailing %lld\n", n, nt, pf[7], pf[0], pf[1],
         pf[2], pf[3]);
  return 0;
}
