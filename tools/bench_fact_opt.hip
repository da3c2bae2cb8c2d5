// dense_lds.h ldl_wave_inv option bits (OPT) on one 1024-thread workgroup, matrix in LDS (the k_ekf_fact form:
// r x r SPD S with the residual row, W = panel_waves(r + 1) panel waves, unit-lower inverse on): in-kernel cycles
// (best of 5) per OPT and the largest difference of the factor / inverse / D / y against OPT = 0, relative to the
// largest magnitude of each output.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_fact_opt.hip -o build/bench_fact_opt
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "dense_lds.h"
using namespace uvhp;

template <int W, int OPT>
__global__ void __launch_bounds__(1024) k_opt(const double *Ain, int r, int inv, long long *tot, double *Aout) {
  extern __shared__ double lds[];
  const int ld = r | 1;
  double *A = lds, *D = lds + (size_t)(r + 1) * ld;
  for (int e = threadIdx.x; e < r * r + r; e += blockDim.x) {
    const int a = e / r, b = e - a * r;
    if (b <= a || a == r) A[(size_t)a * ld + b] = Ain[e];
  }
  __syncthreads();
  const long long t0 = clock64();
  ldl_wave_inv<1, SqLayout, W, OPT>(A, SqLayout{ld}, r, r + 1, D, inv != 0, nullptr, nullptr);
  if (threadIdx.x == 0) tot[0] = clock64() - t0;
  __syncthreads();
  for (int e = threadIdx.x; e < (r + 1) * ld + r + 1; e += blockDim.x) Aout[e] = lds[e];
}

typedef void (*KFn)(const double *, int, int, long long *, double *);

template <int W>
KFn pick(int opt) {
  switch (opt) {
    case 0: return k_opt<W, 0>;
    case 1: return k_opt<W, 1>;
    case 2: return k_opt<W, 2>;
    case 4: return k_opt<W, 4>;
    case 5: return k_opt<W, 5>;
    default: return k_opt<W, 7>;
  }
}

int main() {
  const int opts[] = {0, 1, 2, 4, 5, 7};
  for (int r : {40, 63, 81, 100, 127, 135}) {
    // a covariance-like SPD matrix (geometric spectrum over 6 decades) + residual row
    std::vector<double> A((size_t)r * r + r), Q((size_t)r * r);
    unsigned s = 12345u + r;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65535.0 - 0.5; };
    for (auto &q : Q) q = rnd();
    for (int i = 0; i < r; i++)
      for (int j = 0; j < r; j++) {
        double acc = 0.0;
        for (int k = 0; k < r; k++) acc += Q[(size_t)i * r + k] * Q[(size_t)j * r + k] * std::pow(10.0, -6.0 * k / r);
        A[(size_t)i * r + j] = acc + (i == j ? 1e-6 : 0.0);
      }
    for (int j = 0; j < r; j++) A[(size_t)r * r + j] = rnd();
    double *dA, *dO;
    long long *dt;
    const size_t bytes = (size_t)(r + 1) * (r | 1) * 8 + (size_t)(r + 1) * 8, nout = bytes / 8;
    (void)hipMalloc(&dA, sizeof(double) * A.size());
    (void)hipMalloc(&dt, sizeof(long long));
    (void)hipMalloc(&dO, bytes);
    (void)hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    const int w = panel_waves(r + 1);
    std::vector<double> ref;
    for (int opt : opts) {
      KFn f = w <= 1 ? pick<1>(opt) : w == 2 ? pick<2>(opt) : pick<3>(opt);
      (void)hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      long long best = -1;
      for (int rep = 0; rep < 5; rep++) {
        hipLaunchKernelGGL(f, dim3(1), dim3(1024), bytes, 0, dA, r, 1, dt, dO);
        (void)hipDeviceSynchronize();
        long long t;
        (void)hipMemcpy(&t, dt, sizeof(t), hipMemcpyDeviceToHost);
        if (best < 0 || t < best) best = t;
      }
      std::vector<double> out(nout);
      (void)hipMemcpy(out.data(), dO, bytes, hipMemcpyDeviceToHost);
      if (opt == 0) ref = out;
      double dmax = 0.0, vmax = 0.0;
      for (size_t e = 0; e < nout; e++) {
        if (!std::isfinite(out[e])) dmax = INFINITY;
        dmax = std::max(dmax, std::fabs(out[e] - ref[e]));
        vmax = std::max(vmax, std::fabs(ref[e]));
      }
      printf("r=%3d W=%d OPT=%d  %7lld cycles  max |diff| / max |value| vs OPT 0: %.2e\n", r, w, opt, best,
             dmax / vmax);
    }
    (void)hipFree(dA);
    (void)hipFree(dt);
    (void)hipFree(dO);
  }
  return 0;
}
