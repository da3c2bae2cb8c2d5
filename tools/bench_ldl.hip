// chol_inv_regs (register-resident) vs ldl_inplace + ldl_to_chol + trtri_gj_inplace: agreement and
// single-workgroup time on MI355X.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_ldl.hip -o build/bench_ldl
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "dense_lds.h"
using namespace uvhp;

__global__ void __launch_bounds__(1024) k_test(const double *Ain, int n, int nrows, int which, int mode, double *out,
                                              long long *ts, double *gA) {
  extern __shared__ double lds[];
  const int ld = n | 1;
  double *A = (which == 5 || which == 4) ? gA : lds, *wsp = lds + (size_t)nrows * ld;
  for (int e = threadIdx.x; e < nrows * n; e += blockDim.x) A[(e / n) * ld + e % n] = Ain[e];
  __syncthreads();
  long long t0 = clock64();
  if (which == 2) {
    ldl_panel4(A, ld, n, nrows, wsp);
  } else if (which == 5) {
    ldl_panel4(A, ld, n, nrows, wsp);
  } else if (which == 3 || which == 4) {
    ldl_blk16(A, ld, n, nrows, wsp);
  } else {
    ldl_inplace(A, ld, n, nrows);
  }
  if (mode & 1) ldl_to_chol(A, ld, n, nrows);
  if (mode & 2) trtri_gj_inplace(A, ld, n);
  __syncthreads();
  long long t1 = clock64();
  for (int e = threadIdx.x; e < nrows * n; e += blockDim.x) out[e] = A[(e / n) * ld + e % n];
  if (threadIdx.x == 0) ts[0] = t1 - t0;
}

int main(int argc, char **argv) {
  int n = argc > 1 ? atoi(argv[1]) : 100;
  int nt = argc > 2 ? atoi(argv[2]) : 512;
  int mode = argc > 3 ? atoi(argv[3]) : 3;
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
  double *dA, *dO0, *dO1;
  long long *dts;
  (void)hipMalloc(&dA, 8 * nrows * n);
  (void)hipMalloc(&dO0, 8 * nrows * n);
  (void)hipMalloc(&dO1, 8 * nrows * n);
  (void)hipMalloc(&dts, 16);
  (void)hipMemcpy(dA, A.data(), 8 * nrows * n, hipMemcpyHostToDevice);
  size_t bytes = (size_t)nrows * (n | 1) * 8 + (size_t)(4 * nrows) * 8;
  // static + dynamic LDS must fit the CU's 160 KiB (the same rule as set_dyn_lds in kernels.h): a launch
  // asking for more aborts the queue (HSA_STATUS_ERROR_INVALID_ALLOCATION), so it is refused here
  hipFuncAttributes fa{};
  (void)hipFuncGetAttributes(&fa, (const void *)k_test);
  const size_t lds_limit = 160 * 1024 - (size_t)fa.sharedSizeBytes;
  if (bytes > lds_limit) {
    printf("n=%d needs %zu B of dynamic LDS > %zu available: skipped\n", n, bytes, lds_limit);
    return 0;
  }
  if (hipFuncSetAttribute((const void *)k_test, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_limit) !=
      hipSuccess) {
    printf("dynamic LDS limit not granted\n");
    return 1;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<double> o2(nrows * n);
  double *dO2, *dG;
  (void)hipMalloc(&dO2, 8 * nrows * n);
  (void)hipMalloc(&dG, 8 * (size_t)nrows * (n | 1));
  const char *names[] = {"lds  ", "regs ", "panel4", "blk16", "blk16-global", "panel4-global"};
  std::vector<std::vector<double>> outs;
  for (int which : {0, 2, 5, 3, 4}) {
    for (int it = 0; it < 3; it++) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_test, dim3(1), dim3(nt), bytes, 0, dA, n, nrows, which, mode, dO2, dts, dG);
      hipError_t le = hipGetLastError();
      if (le != hipSuccess) {
        printf("launch failed: %s\n", hipGetErrorString(le));
        return 1;
      }
      (void)hipEventRecord(e1);
      if (hipEventSynchronize(e1) != hipSuccess) {
        printf("kernel failed\n");
        return 1;
      }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      long long ts;
      (void)hipMemcpy(&ts, dts, 8, hipMemcpyDeviceToHost);
      if (it == 2)
        printf("%-15s n=%d nt=%d mode=%d kernel %.1f us  %lld cyc\n", names[which], n, nt, mode, ms * 1e3, ts);
    }
    (void)hipMemcpy(o2.data(), dO2, 8 * nrows * n, hipMemcpyDeviceToHost);
    outs.push_back(o2);
  }
  int bad = 0;
  for (size_t w = 1; w < outs.size(); w++) {
    double err = 0, mx = 0;
    for (int i = 0; i < nrows; i++)
      for (int j = 0; j < n && j <= i; j++) {
        err = fmax(err, fabs(outs[0][i * n + j] - outs[w][i * n + j]));
        mx = fmax(mx, fabs(outs[0][i * n + j]));
      }
    printf("variant %zu: max |x - lds| / max|lds| = %.3e\n", w, err / mx);
    if (!(err / mx < 1e-11)) bad++;
  }
  return bad;
}
