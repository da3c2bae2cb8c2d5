// Per-slot cycle split of dense_lds.h ldl_wave_inv on one workgroup (matrix in LDS): the first panel wave's and
// the first helper's clock64 per 16-column slot (the routine's own `prof` hook), with and without the
// unit-lower inverse, for the one-panel-wave form (SMAX rows per lane, 512 threads) and the W-panel-wave form
// (SMAX = 1, 512 or 1024 threads); the factors are checked bit-identical.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_wave_slots.hip -o build/bench_wave_slots
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "dense_lds.h"
using namespace uvhp;

template <int SMAX, int W>
__device__ void slots_body(const double *Ain, int r, int inv, long long *prof, long long *tot,
                           double *Aout) {
  extern __shared__ double lds[];
  const int ld = r | 1;
  double *A = lds, *D = lds + (size_t)(r + 1) * ld;
  for (int e = threadIdx.x; e < (r + 1) * ld + r + 1; e += blockDim.x) lds[e] = 0.0;  // no stale LDS in the output
  __syncthreads();
  for (int e = threadIdx.x; e < r * r + r; e += blockDim.x) {
    const int a = e / r, b = e - a * r;
    if (b <= a || a == r) A[(size_t)a * ld + b] = Ain[e];
  }
  __syncthreads();
  const long long t0 = clock64();
  ldl_wave_inv<SMAX, SqLayout, W>(A, SqLayout{ld}, r, r + 1, D, inv != 0, nullptr, prof);
  if (threadIdx.x == 0) tot[0] = clock64() - t0;
  __syncthreads();
  for (int e = threadIdx.x; e < (r + 1) * ld + r + 1; e += blockDim.x) Aout[e] = lds[e];
}

template <int SMAX, int W>
__global__ void __launch_bounds__(512) k_slots(const double *Ain, int r, int inv, long long *prof, long long *tot,
                                               double *Aout) {
  slots_body<SMAX, W>(Ain, r, inv, prof, tot, Aout);
}
template <int SMAX, int W>
__global__ void __launch_bounds__(1024) k_slots_1k(const double *Ain, int r, int inv, long long *prof, long long *tot,
                                                  double *Aout) {
  slots_body<SMAX, W>(Ain, r, inv, prof, tot, Aout);
}

typedef void (*KFn)(const double *, int, int, long long *, long long *, double *);

int main() {
  for (int r : {40, 63, 100, 127, 135}) {
    std::vector<double> A((size_t)r * r + r);
    for (int i = 0; i < r; i++)
      for (int j = 0; j < r; j++) A[(size_t)i * r + j] = (i == j ? r + 1.0 : 0.0) + 1.0 / (1 + i + j);
    for (int j = 0; j < r; j++) A[(size_t)r * r + j] = 0.1 * j;
    double *dA, *dO;
    long long *dp, *dt;
    const size_t bytes = (size_t)(r + 1) * (r | 1) * 8 + (size_t)(r + 1) * 8, nout = bytes / 8;
    (void)hipMalloc(&dA, sizeof(double) * A.size());
    (void)hipMalloc(&dp, sizeof(long long) * 64);
    (void)hipMalloc(&dt, sizeof(long long));
    (void)hipMalloc(&dO, bytes);
    (void)hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    const int rows = r + 1, wneed = (rows - 16 + 47) / 48;
    struct V {
      const char *name;
      KFn f;
      int threads;
    };
    KFn one = rows <= 64 ? k_slots<1, 1> : rows <= 128 ? k_slots<2, 1> : k_slots<3, 1>;
    KFn multi = wneed <= 1 ? k_slots<1, 1> : wneed == 2 ? k_slots<1, 2> : k_slots<1, 3>;
    KFn multi1k = wneed <= 1 ? k_slots_1k<1, 1> : wneed == 2 ? k_slots_1k<1, 2> : k_slots_1k<1, 3>;
    V vs[3] = {{"one panel wave, 512 ", one, 512}, {"W panel waves, 512  ", multi, 512}, {"W panel waves, 1024 ", multi1k, 1024}};
    std::vector<double> out[3];
    for (int v = 0; v < 3; v++) {
      (void)hipFuncSetAttribute((const void *)vs[v].f, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      for (int inv = 0; inv < 2; inv++) {
        long long best = -1, p[64];
        for (int rep = 0; rep < 5; rep++) {
          (void)hipMemset(dp, 0, sizeof(long long) * 64);
          hipLaunchKernelGGL(vs[v].f, dim3(1), dim3(vs[v].threads), bytes, 0, dA, r, inv, dp, dt, dO);
          (void)hipDeviceSynchronize();
          long long t;
          (void)hipMemcpy(&t, dt, sizeof(t), hipMemcpyDeviceToHost);
          if (best < 0 || t < best) {
            best = t;
            (void)hipMemcpy(p, dp, sizeof(p), hipMemcpyDeviceToHost);
          }
        }
        if (inv) {
          out[v].resize(nout);
          (void)hipMemcpy(out[v].data(), dO, bytes, hipMemcpyDeviceToHost);
        }
        printf("%s r=%3d W=%d inv=%d total %7lld cycles | panel slots:", vs[v].name, r, v ? wneed : 1, inv, best);
        for (int j = 0; j < 10 && p[j]; j++) printf(" %lld", p[j]);
        printf(" | helper:");
        for (int j = 0; j < 10 && p[32 + j]; j++) printf(" %lld", p[32 + j]);
        printf("\n");
      }
    }
    for (int v = 0; v < 3; v += 2) {  // to compare builds of dense_lds.h bit for bit
      unsigned long long h = 1469598103934665603ull;
      for (double d : out[v]) {
        unsigned long long u;
        std::memcpy(&u, &d, 8);
        h = (h ^ u) * 1099511628211ull;
      }
      printf("r=%3d variant %d factor + inverse digest %016llx\n", r, v, h);
    }
    for (int v = 1; v < 3; v++) {
      size_t nd = 0;
      for (size_t e = 0; e < nout; e++) nd += std::memcmp(&out[0][e], &out[v][e], 8) != 0;
      printf("r=%3d variant %d factor + inverse bit-identical to one panel wave: %s (%zu differing doubles)\n", r, v,
             nd ? "NO" : "yes", nd);
    }
    (void)hipFree(dA);
    (void)hipFree(dp);
    (void)hipFree(dt);
    (void)hipFree(dO);
  }
  return 0;
}
