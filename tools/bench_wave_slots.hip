// Per-slot cycle split of dense_lds.h ldl_wave_inv on one workgroup (512 threads, matrix in LDS): wave 0's and
// wave 1's clock64 per 16-column slot (the routine's own `prof` hook), with and without the unit-lower inverse.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_wave_slots.hip -o build/bench_wave_slots
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "dense_lds.h"
using namespace uvhp;

template <int SMAX>
__global__ void __launch_bounds__(512) k_slots(const double *Ain, int r, int inv, long long *prof, long long *tot) {
  extern __shared__ double lds[];
  const int ld = r | 1;
  double *A = lds, *D = lds + (size_t)(r + 1) * ld;
  for (int e = threadIdx.x; e < r * r + r; e += blockDim.x) {
    const int a = e / r, b = e - a * r;
    if (b <= a || a == r) A[(size_t)a * ld + b] = Ain[e];
  }
  __syncthreads();
  const long long t0 = clock64();
  ldl_wave_inv<SMAX>(A, SqLayout{ld}, r, r + 1, D, inv != 0, nullptr, prof);
  if (threadIdx.x == 0) tot[0] = clock64() - t0;
}

int main() {
  for (int r : {40, 63, 100, 127}) {
    std::vector<double> A((size_t)r * r + r);
    for (int i = 0; i < r; i++)
      for (int j = 0; j < r; j++) A[(size_t)i * r + j] = (i == j ? r + 1.0 : 0.0) + 1.0 / (1 + i + j);
    for (int j = 0; j < r; j++) A[(size_t)r * r + j] = 0.1 * j;
    double *dA;
    long long *dp, *dt;
    hipMalloc(&dA, sizeof(double) * A.size());
    hipMalloc(&dp, sizeof(long long) * 64);
    hipMalloc(&dt, sizeof(long long));
    hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    const size_t bytes = (size_t)(r + 1) * (r | 1) * 8 + (size_t)(r + 1) * 8;
    auto *kf = (r + 1 <= 64) ? k_slots<1> : k_slots<2>;
    hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    for (int inv = 0; inv < 2; inv++) {
      long long best = -1, p[64];
      for (int rep = 0; rep < 5; rep++) {
        hipMemset(dp, 0, sizeof(long long) * 64);
        hipLaunchKernelGGL(kf, dim3(1), dim3(512), bytes, 0, dA, r, inv, dp, dt);
        hipDeviceSynchronize();
        long long t;
        hipMemcpy(&t, dt, sizeof(t), hipMemcpyDeviceToHost);
        if (best < 0 || t < best) {
          best = t;
          hipMemcpy(p, dp, sizeof(p), hipMemcpyDeviceToHost);
        }
      }
      printf("r=%3d inv=%d total %7lld cycles | wave0 slots:", r, inv, best);
      for (int j = 0; j < 10 && p[j]; j++) printf(" %lld", p[j]);
      printf(" | wave1:");
      for (int j = 0; j < 10 && p[32 + j]; j++) printf(" %lld", p[32 + j]);
      printf("\n");
    }
    hipFree(dA);
    hipFree(dp);
    hipFree(dt);
  }
  return 0;
}
