// dense_lds.h ldl_wave_inv (the information-form factors' form: W panel waves, 1024 threads, no inverse, the
// diagonal-block inverses to Xd) in three LDS layouts: square (ld = n | 1, where it fits), packed lower triangle
// (k_info_cholP / Z mode 1) and 16 x 16 tiles of the lower triangle at row stride 17 (TlLayout below).  In-kernel
// cycles (best of 5) and the factor, pivots and block inverses compared bit for bit with the packed layout's.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_layouts.hip -o build/bench_layouts
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "dense_lds.h"
using namespace uvhp;

// lower 16 x 16 tiles (I, C), C <= I, stored tile after tile (I(I+1)/2 + C), rows of a tile at stride 17
struct TlLayout {
  static constexpr bool square = false;
  __device__ __forceinline__ size_t operator()(int i, int j) const {
    const int I = i >> 4, C = j >> 4;
    return (size_t)(I * (I + 1) / 2 + C) * 272 + (i & 15) * 17 + (j & 15);
  }
};
__host__ __device__ inline size_t tl_doubles(int nrows) {
  const int nb = (nrows + 15) / 16;
  return (size_t)nb * (nb + 1) / 2 * 272;
}

template <class LA, int W>
__global__ void __launch_bounds__(1024) k_fact(const double *Ain, int n, int nrows, LA la, size_t asz, long long *tot,
                                               double *Lout, double *Dout, double *Xd) {
  extern __shared__ double lds[];
  double *A = lds, *D = lds + asz;
  for (int e = threadIdx.x; e < nrows * n; e += blockDim.x) {
    const int a = e / n, b = e - a * n;
    if (b <= a) A[la(a, b)] = Ain[e];
  }
  __syncthreads();
  const long long t0 = clock64();
  ldl_wave_inv<1, LA, W>(A, la, n, nrows, D, false, Xd);
  if (threadIdx.x == 0) tot[0] = clock64() - t0;
  __syncthreads();
  for (int e = threadIdx.x; e < nrows * n; e += blockDim.x) {
    const int a = e / n, b = e - a * n;
    Lout[e] = (b < a) ? A[la(a, b)] : 0.0;
  }
  for (int k = threadIdx.x; k < n; k += blockDim.x) Dout[k] = D[k];
}

template <class LA, int W>
static void run(const char *name, const std::vector<double> &A, int n, int nrows, LA la, size_t asz,
                std::vector<double> *ref) {
  double *dA, *dL, *dD, *dX;
  long long *dt;
  const int nb = (n + 15) / 16;
  (void)hipMalloc(&dA, sizeof(double) * A.size());
  (void)hipMalloc(&dL, sizeof(double) * nrows * n);
  (void)hipMalloc(&dD, sizeof(double) * n);
  (void)hipMalloc(&dX, sizeof(double) * 256 * nb);
  (void)hipMalloc(&dt, sizeof(long long));
  (void)hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
  const size_t bytes = (asz + n) * sizeof(double);
  if (bytes > 152 * 1024) {
    std::printf("%-8s n %3d rows %3d: %zu B of LDS, does not fit\n", name, n, nrows, bytes);
    return;
  }
  auto fn = k_fact<LA, W>;
  (void)hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024);
  long long best = -1;
  for (int rep = 0; rep < 5; rep++) {
    hipLaunchKernelGGL(fn, dim3(1), dim3(1024), bytes, 0, dA, n, nrows, la, asz, dt, dL, dD, dX);
    (void)hipDeviceSynchronize();
    long long t;
    (void)hipMemcpy(&t, dt, sizeof(t), hipMemcpyDeviceToHost);
    if (best < 0 || t < best) best = t;
  }
  std::vector<double> out((size_t)nrows * n + n + 256 * nb);
  (void)hipMemcpy(out.data(), dL, sizeof(double) * nrows * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(out.data() + (size_t)nrows * n, dD, sizeof(double) * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(out.data() + (size_t)nrows * n + n, dX, sizeof(double) * 256 * nb, hipMemcpyDeviceToHost);
  size_t nd = 0;
  if (ref->empty())
    *ref = out;
  else
    for (size_t e = 0; e < out.size(); e++) nd += std::memcmp(&out[e], &(*ref)[e], 8) != 0;
  std::printf("%-8s n %3d rows %3d W %d: %7lld cycles, LDS %6zu B, differing doubles vs packed %zu\n", name, n, nrows, W,
              best, bytes, nd);
  (void)hipFree(dA);
  (void)hipFree(dL);
  (void)hipFree(dD);
  (void)hipFree(dX);
  (void)hipFree(dt);
}

template <int W>
static void case_n(int n) {
  const int nrows = n + 1;
  std::vector<double> A((size_t)nrows * n);
  for (int i = 0; i < nrows; i++)
    for (int j = 0; j < n; j++) A[(size_t)i * n + j] = (i == j ? n + 1.0 : 0.0) + 1.0 / (1 + i + j) + (i == n ? 0.1 * j : 0.0);
  std::vector<double> ref;
  run<PkLayout, W>("packed", A, n, nrows, PkLayout{}, packed_lds_doubles(nrows), &ref);
  run<TlLayout, W>("tiles", A, n, nrows, TlLayout{}, tl_doubles(nrows), &ref);
  run<SqLayout, W>("square", A, n, nrows, SqLayout{n | 1}, (size_t)nrows * (n | 1), &ref);
}

int main() {
  case_n<3>(134);
  case_n<3>(154);
  case_n<4>(172);
  case_n<4>(190);
  return 0;
}
