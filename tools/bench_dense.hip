// Microbenchmark of the single-workgroup dense routines (dense_lds.h): per-phase cycle counts.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -ffp-contract=off -I uvio_amd/csrc tools/bench_dense.hip -o build/bench_dense
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "dense_lds.h"
using namespace uvhp;

__global__ void __launch_bounds__(1024) k_test(const double *Ain, int n, double *out, long long *ts) {
  extern __shared__ double lds[];
  const int ld = n | 1;
  double *A = lds;
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) A[(e / n) * ld + e % n] = Ain[e];
  __syncthreads();
  long long t0 = clock64();
  ldl_inplace(A, ld, n, n);
  ldl_to_chol(A, ld, n, n);
  __syncthreads();
  long long t1 = clock64();
  trtri_gj_inplace(A, ld, n);
  __syncthreads();
  long long t2 = clock64();
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) out[e] = A[(e / n) * ld + e % n];
  if (threadIdx.x == 0) { ts[0] = t1 - t0; ts[1] = t2 - t1; }
}

int main(int argc, char **argv) {
  int n = argc > 1 ? atoi(argv[1]) : 100;
  int nt = argc > 2 ? atoi(argv[2]) : 256;
  std::vector<double> A(n * n), B(n * n);
  srand(1);
  for (auto &x : B) x = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = (i == j) ? n : 0;
      for (int k = 0; k < n; k++) s += B[i * n + k] * B[j * n + k];
      A[i * n + j] = s;
    }
  double *dA, *dO;
  long long *dts;
  hipMalloc(&dA, 8 * n * n); hipMalloc(&dO, 8 * n * n); hipMalloc(&dts, 16);
  hipMemcpy(dA, A.data(), 8 * n * n, hipMemcpyHostToDevice);
  size_t bytes = dense_lds_bytes(n, n);
  hipFuncSetAttribute((const void *)k_test, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 3; it++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_test, dim3(1), dim3(nt), bytes, 0, dA, n, dO, dts);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long ts[2]; hipMemcpy(ts, dts, 16, hipMemcpyDeviceToHost);
    printf("nt=%d n=%d kernel %.1f us  chol %lld cyc  trtri %lld cyc\n", nt, n, ms * 1e3, ts[0], ts[1]);
  }
  // check: Linv * A * Linv^T = I
  std::vector<double> Li(n * n);
  hipMemcpy(Li.data(), dO, 8 * n * n, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      double s = 0;
      for (int a = 0; a <= i; a++)
        for (int b = 0; b <= j; b++) s += Li[i * n + a] * A[a * n + b] * Li[j * n + b];
      err = fmax(err, fabs(s - (i == j)));
    }
  printf("max |Linv A Linv^T - I| = %.3e\n", err);
  return 0;
}
