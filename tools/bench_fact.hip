// Single-workgroup factorizations on MI355X (512 threads, matrix in LDS): ldl_blk16 + ldl_to_chol (the
// previous core) against dense_lds.h ldl_wave_inv without and with the unit-lower inverse, in-kernel cycle
// counts, results checked against a CPU Cholesky / triangular inverse of [S ; b^T].  LDS requests are
// clamped to the CU's 160 KiB (static + dynamic) and every launch is checked.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I uvio_amd/csrc tools/bench_fact.hip -o build/bench_fact
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dense_lds.h"
using namespace uvhp;

// variant 0: ldl_blk16 + ldl_to_chol (L_c, y); 1: ldl_wave_inv (L_c, y); 2: ldl_wave_inv + inverse (L_c^-1, y)
template <int variant, int SMAX>
__global__ void __launch_bounds__(512) k_fact(const double *Ain, int r, double *out, long long *ts) {
  extern __shared__ double lds[];
  const int ld = r | 1;
  double *A = lds, *W = lds + (size_t)(r + 1) * ld;  // W: ldl_blk16's panel scratch / the D of ldl_wave_inv
  staged_copy(
      r * r + r, [&](int e) { return Ain[e]; },
      [&](int e, double v) {
        const int a = e / r, b = e - a * r;
        if (b <= a || a == r) A[(size_t)a * ld + b] = v;
      });
  __syncthreads();
  const long long t0 = clock64();
  if constexpr (variant == 0) {
    ldl_blk16(A, ld, r, r + 1, W);
    ldl_to_chol(A, ld, r, r + 1);
  } else {
    ldl_wave_inv<SMAX>(A, SqLayout{ld}, r, r + 1, W, variant == 2);
  }
  const long long t1 = clock64();
  for (int e = threadIdx.x; e < r * r + r; e += blockDim.x) {
    const int a = e / r, b = e - a * r;
    double v = 0.0;
    if constexpr (variant == 0) {
      v = (b <= a || a == r) ? A[(size_t)a * ld + b] : 0.0;
    } else {
      const double sd_b = sqrt(W[b]);
      if (a == r)
        v = A[(size_t)r * ld + b] * sd_b;
      else if (variant == 1)
        v = (b < a) ? A[(size_t)a * ld + b] * sd_b : (b == a ? sd_b : 0.0);
      else
        v = (b < a) ? A[(size_t)b * ld + a] / sqrt(W[a]) : (b == a ? 1.0 / sd_b : 0.0);
    }
    out[e] = v;
  }
  if (threadIdx.x == 0) ts[0] = t1 - t0;
}

int main() {
  int bad = 0;
  const void *kf[3][2] = {{(const void *)k_fact<0, 1>, (const void *)k_fact<0, 1>},
                          {(const void *)k_fact<1, 1>, (const void *)k_fact<1, 2>},
                          {(const void *)k_fact<2, 1>, (const void *)k_fact<2, 2>}};
  size_t lds_limit = 160 * 1024;
  for (int v = 0; v < 3; v++)
    for (int s = 0; s < 2; s++) {
      hipFuncAttributes fa{};
      (void)hipFuncGetAttributes(&fa, kf[v][s]);
      const size_t lim = 160 * 1024 - (size_t)fa.sharedSizeBytes;
      if (lim < lds_limit) lds_limit = lim;
    }
  for (int v = 0; v < 3; v++)
    for (int s = 0; s < 2; s++)
      if (hipFuncSetAttribute(kf[v][s], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_limit) != hipSuccess) {
        printf("dynamic LDS limit not granted\n");
        return 1;
      }
  const char *names[3] = {"blk16+chol ", "wave       ", "wave+inv   "};
  for (int r : {5, 16, 20, 33, 48, 100, 127}) {
    const size_t bytes = dense_lds_bytes(r + 1, r) + (size_t)(r + 1) * 4 * sizeof(double);
    if (bytes > lds_limit) {
      printf("r=%d needs %zu B > %zu: skipped\n", r, bytes, lds_limit);
      continue;
    }
    std::vector<double> Bm(r * r), A((r + 1) * r);
    srand(r);
    for (auto &x : Bm) x = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < r; i++)
      for (int j = 0; j < r; j++) {
        double s = (i == j) ? 0.1 : 0;
        for (int k = 0; k < r; k++) s += Bm[i * r + k] * Bm[j * r + k];
        A[i * r + j] = s;
      }
    for (int j = 0; j < r; j++) A[r * r + j] = (double)rand() / RAND_MAX - 0.5;
    std::vector<double> L(r * r, 0.0), Li(r * r, 0.0), y(r);
    for (int j = 0; j < r; j++) {
      double s = A[j * r + j];
      for (int k = 0; k < j; k++) s -= L[j * r + k] * L[j * r + k];
      L[j * r + j] = std::sqrt(s);
      for (int i = j + 1; i < r; i++) {
        double t = A[i * r + j];
        for (int k = 0; k < j; k++) t -= L[i * r + k] * L[j * r + k];
        L[i * r + j] = t / L[j * r + j];
      }
    }
    for (int i = 0; i < r; i++) {
      double t = A[r * r + i];
      for (int k = 0; k < i; k++) t -= L[i * r + k] * y[k];
      y[i] = t / L[i * r + i];
    }
    for (int c = 0; c < r; c++)
      for (int i = c; i < r; i++) {
        double t = (i == c) ? 1.0 : 0.0;
        for (int k = c; k < i; k++) t -= L[i * r + k] * Li[k * r + c];
        Li[i * r + c] = t / L[i * r + i];
      }
    double *dA, *dO;
    long long *dts;
    (void)hipMalloc(&dA, 8 * A.size());
    (void)hipMalloc(&dO, 8 * A.size());
    (void)hipMalloc(&dts, 64);
    (void)hipMemcpy(dA, A.data(), 8 * A.size(), hipMemcpyHostToDevice);
    for (int variant = 0; variant < 3; variant++) {
      long long best = 1LL << 60;
      for (int it = 0; it < 10; it++) {
        const double *cA = dA;
        void *args[] = {&cA, &r, &dO, &dts};
        if (hipLaunchKernel(kf[variant][r + 1 > 64 ? 1 : 0], dim3(1), dim3(512), args, bytes, 0) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) {
          printf("launch failed\n");
          return 1;
        }
        long long ts;
        (void)hipMemcpy(&ts, dts, 8, hipMemcpyDeviceToHost);
        if (ts < best) best = ts;
      }
      std::vector<double> O(A.size());
      (void)hipMemcpy(O.data(), dO, 8 * O.size(), hipMemcpyDeviceToHost);
      const std::vector<double> &R = (variant == 2) ? Li : L;
      double e = 0, m = 0, ey = 0, my = 0;
      for (int i = 0; i < r; i++)
        for (int j = 0; j <= i; j++) {
          e = fmax(e, fabs(O[i * r + j] - R[i * r + j]));
          m = fmax(m, fabs(R[i * r + j]));
        }
      for (int j = 0; j < r; j++) {
        ey = fmax(ey, fabs(O[r * r + j] - y[j]));
        my = fmax(my, fabs(y[j]));
      }
      printf("r=%3d %s %8lld cycles | rel err %s %.1e  y %.1e\n", r, names[variant], best,
             variant == 2 ? "Linv" : "L   ", e / m, ey / my);
      if (!(e / m < 1e-9) || !(ey / my < 1e-9)) bad++;
    }
    (void)hipFree(dA);
    (void)hipFree(dO);
    (void)hipFree(dts);
  }
  return bad;
}
