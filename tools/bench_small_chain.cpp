// Isolated timing of two update-chain launches at the cfg3 shapes, through the product library's own launch
// functions (libuvio_hp.so): launch_trsm_lt (X = V U^-T of the information form, N = 313, r = 148) and
// launch_ekf_phaseA (k_ekf_MS: M = P[:, I] H^T and S_up = H T^T, N = 313, n = 163, r = 100, T given).
// Prints the average µs per call over REPS back-to-back calls (HIP events, caches warm) and a checksum of the
// outputs, so two library builds or an A/B switch (UVIO_HP_MS_SPLIT: M and S as two launches) can be compared
// for speed and for bit-equality.  Results: profiles/r04t_small_chain.txt.
// Usage: bench_small_chain [REPS [N LDP n r LDH [TALL]]] (the k_ekf_MS / full-update shapes).
// Build: hipcc -O2 -std=c++17 -I uvio_amd/csrc -I include tools/bench_small_chain.cpp -L uvio_amd -l:libuvio_hp.so
//        -Wl,-rpath,'$ORIGIN/../uvio_amd' -o build/bench_small_chain
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "kernels.h"
using namespace uvhp;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double *dev(const std::vector<double> &h) {
  double *d;
  CK(hipMalloc(&d, h.size() * sizeof(double)));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  return d;
}
static uint64_t checksum(const double *d, size_t n) {
  std::vector<double> h(n);
  CK(hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost));
  uint64_t c = 1469598103934665603ull;
  for (double v : h) {
    uint64_t u;
    memcpy(&u, &v, 8);
    c = (c ^ u) * 1099511628211ull;
  }
  return c;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  // the direct-update shapes (k_ekf_MS / the full update): N ldp n r ldh, defaults the cfg3 SLAM batch's means
  const int uN = argc > 2 ? atoi(argv[2]) : 313, uldp = argc > 3 ? atoi(argv[3]) : uN;
  const int un = argc > 4 ? atoi(argv[4]) : 163, ur = argc > 5 ? atoi(argv[5]) : 100;
  const int uldh = argc > 6 ? atoi(argv[6]) : un;
  const bool utall = argc > 7 ? atoi(argv[7]) != 0 : true;  // 0: no T from a chi2 gate (delayed initialization)
  std::mt19937_64 rng(11);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int N = 313;
  {  // trsm: W = M L^-T, L unit-diagonal-dominant lower (r x r)
    const int r = 148;
    std::vector<double> M(N * r), L(r * r, 0.0);
    for (auto &v : M) v = U(rng);
    for (int i = 0; i < r; i++)
      for (int j = 0; j <= i; j++) L[i * r + j] = (i == j) ? 1.0 + 0.5 * std::abs(U(rng)) : 0.1 * U(rng);
    double *dM = dev(M), *dL = dev(L), *dW, *dDinv;
    CK(hipMalloc(&dW, sizeof(double) * N * r));
    CK(hipMalloc(&dDinv, sizeof(double) * 256 * (r / 16 + 2)));
    launch_trsm_lt(s, dM, r, nullptr, N, r, dL, r, dDinv, dW, true);  // forms Dinv
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int k = 0; k < reps; k++) launch_trsm_lt(s, dM, r, nullptr, N, r, dL, r, dDinv, dW, false);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("trsm_lt  N %d r %d: %.2f us/call  checksum %016llx\n", N, r, 1000.0 * ms / reps,
           (unsigned long long)checksum(dW, (size_t)N * r));
  }
  {  // k_ekf_MS: M = P[:, I] H^T, S_up = H T^T with T = H P_II (given)
    const int n = un, r = ur, N = uN, ldp = uldp, ldh = uldh;
    std::vector<double> P((size_t)N * ldp), H((size_t)r * ldh), T((size_t)r * ldh);
    for (int i = 0; i < N; i++)
      for (int j = 0; j <= i; j++) P[(size_t)i * ldp + j] = P[(size_t)j * ldp + i] = (i == j) ? 1.0 : 0.01 * U(rng);
    for (auto &v : H) v = U(rng);
    for (auto &v : T) v = U(rng);
    std::vector<int> hidx(n);
    for (int k = 0; k < n; k++) hidx[k] = (k * 37) % N;
    double *dP = dev(P), *dH = dev(H), *dT = dev(T);
    int *dI, *dneg;
    CK(hipMalloc(&dI, sizeof(int) * n));
    CK(hipMemcpy(dI, hidx.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    CK(hipMalloc(&dneg, sizeof(int) * 4));
    EkfScratch sc{};
    CK(hipMalloc(&sc.M, sizeof(double) * N * r));
    CK(hipMalloc(&sc.S, sizeof(double) * 4 * r * r));
    sc.neg = dneg;
    sc.Tall = utall ? dT : nullptr;
    sc.ldt = ldh;
    launch_ekf_phaseA(s, dP, ldp, N, dH, ldh, r, n, dI, 1e-4, sc);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int k = 0; k < reps; k++) launch_ekf_phaseA(s, dP, ldp, N, dH, ldh, r, n, dI, 1e-4, sc);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("ekf_MS   N %d ldp %d n %d r %d ldh %d: %.2f us/call  checksum M %016llx S %016llx\n", N, ldp, n, r, ldh, 1000.0 * ms / reps,
           (unsigned long long)checksum(sc.M, (size_t)N * r),
           (unsigned long long)checksum(sc.S + 2 * (size_t)r * r, (size_t)r * r));
  }
  {  // the whole direct update (k_ekf_MS -> k_ekf_fact -> k_ekf_WP) back to back: each k_ekf_MS reads the P that
     // the previous k_ekf_WP wrote (per-kernel times: run under rocprofv3 --kernel-trace --stats)
    const int n = un, r = ur, N = uN, ldp = uldp, ldh = uldh;
    std::vector<double> P((size_t)N * ldp), H((size_t)r * ldh), T((size_t)r * ldh), res(r);
    for (int i = 0; i < N; i++)
      for (int j = 0; j <= i; j++) P[(size_t)i * ldp + j] = P[(size_t)j * ldp + i] = (i == j) ? 1.0 : 0.01 * U(rng);
    for (auto &v : H) v = 0.05 * U(rng);
    for (auto &v : T) v = U(rng);
    for (auto &v : res) v = 0.01 * U(rng);
    std::vector<int> hidx(n);
    for (int k = 0; k < n; k++) hidx[k] = (k * 37) % N;
    double *dP = dev(P), *dH = dev(H), *dT = dev(T), *dres = dev(res);
    int *dI, *dneg;
    CK(hipMalloc(&dI, sizeof(int) * n));
    CK(hipMemcpy(dI, hidx.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    CK(hipMalloc(&dneg, sizeof(int) * 4));
    EkfScratch sc{};
    CK(hipMalloc(&sc.M, sizeof(double) * N * r));
    CK(hipMalloc(&sc.S, sizeof(double) * 6 * r * r));
    CK(hipMalloc(&sc.y, sizeof(double) * (r + 2)));
    CK(hipMalloc(&sc.dx, sizeof(double) * (N + 2)));
    CK(hipMalloc(&sc.Dinv, sizeof(double) * 256 * (r / 16 + 2)));
    sc.neg = dneg;
    sc.Tall = utall ? dT : nullptr;
    sc.ldt = ldh;
    const int reps2 = reps < 50 ? reps : 50;  // P shrinks with every update
    CK(hipEventRecord(e0, s));
    for (int k = 0; k < reps2; k++) launch_ekf_update(s, dP, ldp, N, dH, ldh, r, n, dI, dres, 1, 1.0, sc);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("ekf_update N %d n %d r %d: %.2f us/call (MS + fact + WP)\n", N, n, r, 1000.0 * ms / reps2);
  }
  return 0;
}
