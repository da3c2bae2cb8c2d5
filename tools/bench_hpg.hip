// Variants of the large-batch chi2 GEMM T = H P_can (kernels_chi2.hip k_gemm_HPg_tiled) at the TrackSIM workloads'
// shapes (cfg5: m 74568 x n 242, cfg4: 80691 x 172, cfg3t: 30184 x 154; ldh 512), timed with hip events, every
// variant's T compared bit for bit with the committed kernel's (every variant accumulates each element over k in
// the same ascending 4-wide MFMA steps, so the bits must agree).
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -ffp-contract=off tools/bench_hpg.hip -o build/bench_hpg
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef double dbl4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)

__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int per = nwg / 8, rem = nwg % 8, x = orig % 8, k = orig / 8;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
}

// ---- V0: the committed kernel (64 x 64 tile, 4 waves of 32 x 32, K slabs of 16 through LDS, two barriers)
template <int BK>
__global__ void __launch_bounds__(256) k_v0(const double *__restrict__ H, int m, int n, int ldh,
                                            const double *__restrict__ P, int ldp, double *__restrict__ T, int ldt) {
  constexpr int HPB = 64, HPK = BK, NL = HPK / 4;
  __shared__ double As[HPB][HPK + 1];
  __shared__ double Bs[HPK][HPB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int tc = (n + HPB - 1) / HPB;
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), ti = wid / tc;
  const int i0 = ti * HPB, j0 = (wid - ti * tc) * HPB;
  double ra[NL], rb[NL];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NL; u++) {
      const int e = tid + 256 * u;
      const int ar = i0 + e / HPK, ak = k0 + e % HPK;
      ra[u] = (ar < m && ak < n) ? H[(size_t)ar * ldh + ak] : 0.0;
      const int bk = k0 + (e >> 6), bc = j0 + (e & 63);
      rb[u] = (bk < n && bc < n) ? P[(size_t)bk * ldp + bc] : 0.0;
    }
  };
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(0);
  for (int k0 = 0; k0 < n; k0 += HPK) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NL; u++) {
      const int e = tid + 256 * u;
      As[e / HPK][e % HPK] = ra[u];
      Bs[e >> 6][e & 63] = rb[u];
    }
    __syncthreads();
    if (k0 + HPK < n) load(k0 + HPK);
#pragma unroll
    for (int kk = 0; kk < HPK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[t] = As[32 * wr + 16 * t + r16][kk + kq];
        b[t] = Bs[kk + kq][32 * wc + 16 * t + r16];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ta++)
#pragma unroll
        for (int tb = 0; tb < 2; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 2; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 32 * wr + 16 * ta + kq + 4 * q, col = j0 + 32 * wc + 16 * tb + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}

// ---- V2: LDS double buffer (one barrier per slab): slab s + 1 is written into the other stage while slab s is
// multiplied; tile 64 x 64, 4 waves of 32 x 32
template <int BK>
__global__ void __launch_bounds__(256) k_v2(const double *__restrict__ H, int m, int n, int ldh,
                                            const double *__restrict__ P, int ldp, double *__restrict__ T, int ldt) {
  constexpr int HPB = 64, HPK = BK, NL = HPK / 4;
  __shared__ double As[2][HPB][HPK + 1];
  __shared__ double Bs[2][HPK][HPB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int tc = (n + HPB - 1) / HPB;
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), ti = wid / tc;
  const int i0 = ti * HPB, j0 = (wid - ti * tc) * HPB;
  double ra[NL], rb[NL];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NL; u++) {
      const int e = tid + 256 * u;
      const int ar = i0 + e / HPK, ak = k0 + e % HPK;
      ra[u] = (ar < m && ak < n) ? H[(size_t)ar * ldh + ak] : 0.0;
      const int bk = k0 + (e >> 6), bc = j0 + (e & 63);
      rb[u] = (bk < n && bc < n) ? P[(size_t)bk * ldp + bc] : 0.0;
    }
  };
  auto store = [&](int s) {
#pragma unroll
    for (int u = 0; u < NL; u++) {
      const int e = tid + 256 * u;
      As[s][e / HPK][e % HPK] = ra[u];
      Bs[s][e >> 6][e & 63] = rb[u];
    }
  };
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(0);
  store(0);
  __syncthreads();
  int s = 0;
  for (int k0 = 0; k0 < n; k0 += HPK) {
    const bool more = k0 + HPK < n;
    if (more) load(k0 + HPK);
#pragma unroll
    for (int kk = 0; kk < HPK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[t] = As[s][32 * wr + 16 * t + r16][kk + kq];
        b[t] = Bs[s][kk + kq][32 * wc + 16 * t + r16];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ta++)
#pragma unroll
        for (int tb = 0; tb < 2; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
    if (more) store(s ^ 1);
    __syncthreads();
    s ^= 1;
  }
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 2; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 32 * wr + 16 * ta + kq + 4 * q, col = j0 + 32 * wc + 16 * tb + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}

// ---- V4: no LDS and no barriers: each wave owns a 32 x 32 block of T (2 x 2 MFMA tiles), its A rows and B
// columns read straight from global memory in the MFMA operand layout (register double buffer of KC k-steps);
// four waves per workgroup cover a 64 x 64 tile, the workgroups XCD-swizzled as in V0
template <int KC>
__global__ void __launch_bounds__(256) k_v4(const double *__restrict__ H, int m, int n, int ldh,
                                            const double *__restrict__ P, int ldp, double *__restrict__ T, int ldt) {
  constexpr int HPB = 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int tc = (n + HPB - 1) / HPB;
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), ti = wid / tc;
  const int i0 = ti * HPB + 32 * wr, j0 = (wid - ti * tc) * HPB + 32 * wc;
  const double *Ar[2];
  bool av[2], bv[2];
  int bc[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int row = i0 + 16 * t + r16;
    av[t] = row < m;
    Ar[t] = H + (size_t)min(row, m - 1) * ldh;
    bc[t] = min(j0 + 16 * t + r16, n - 1);
    bv[t] = j0 + 16 * t + r16 < n;
  }
  double a0[KC][2], b0[KC][2], a1[KC][2], b1[KC][2];
  auto load = [&](int k0, double (&a)[KC][2], double (&b)[KC][2]) {
#pragma unroll
    for (int u = 0; u < KC; u++) {
      const int k = k0 + 4 * u + kq;
      const bool kin = k < n;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[u][t] = (av[t] && kin) ? Ar[t][k] : 0.0;
        b[u][t] = (bv[t] && kin) ? P[(size_t)k * ldp + bc[t]] : 0.0;
      }
    }
  };
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  auto mma = [&](double (&a)[KC][2], double (&b)[KC][2], int k0) {
#pragma unroll
    for (int u = 0; u < KC; u++)
      if (k0 + 4 * u < n)
#pragma unroll
        for (int ta = 0; ta < 2; ta++)
#pragma unroll
          for (int tb = 0; tb < 2; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][ta], b[u][tb], acc[ta][tb], 0, 0, 0);
  };
  load(0, a0, b0);
  for (int k0 = 0; k0 < n; k0 += 8 * KC) {
    if (k0 + 4 * KC < n) load(k0 + 4 * KC, a1, b1);
    mma(a0, b0, k0);
    if (k0 + 4 * KC >= n) break;
    if (k0 + 8 * KC < n) load(k0 + 8 * KC, a0, b0);
    mma(a1, b1, k0 + 4 * KC);
  }
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 2; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 16 * ta + kq + 4 * q, col = j0 + 16 * tb + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}

// ---- V5: V4 with 32 x 64 per wave (2 x 4 MFMA tiles): each A operand feeds 4 MFMAs, each B operand 2; a workgroup
// of 4 waves covers 128 x 64
template <int KC>
__global__ void __launch_bounds__(256) k_v5(const double *__restrict__ H, int m, int n, int ldh,
                                            const double *__restrict__ P, int ldp, double *__restrict__ T, int ldt) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int tc = (n + 63) / 64;
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), ti = wid / tc;
  const int i0 = ti * 128 + 32 * w, j0 = (wid - ti * tc) * 64;
  const double *Ar[2];
  bool av[2], bv[4];
  int bc[4];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int row = i0 + 16 * t + r16;
    av[t] = row < m;
    Ar[t] = H + (size_t)min(row, m - 1) * ldh;
  }
#pragma unroll
  for (int t = 0; t < 4; t++) {
    bc[t] = min(j0 + 16 * t + r16, n - 1);
    bv[t] = j0 + 16 * t + r16 < n;
  }
  double a0[KC][2], b0[KC][4], a1[KC][2], b1[KC][4];
  auto load = [&](int k0, double (&a)[KC][2], double (&b)[KC][4]) {
#pragma unroll
    for (int u = 0; u < KC; u++) {
      const int k = k0 + 4 * u + kq;
      const bool kin = k < n;
#pragma unroll
      for (int t = 0; t < 2; t++) a[u][t] = (av[t] && kin) ? Ar[t][k] : 0.0;
#pragma unroll
      for (int t = 0; t < 4; t++) b[u][t] = (bv[t] && kin) ? P[(size_t)k * ldp + bc[t]] : 0.0;
    }
  };
  dbl4 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 4; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  auto mma = [&](double (&a)[KC][2], double (&b)[KC][4], int k0) {
#pragma unroll
    for (int u = 0; u < KC; u++)
      if (k0 + 4 * u < n)
#pragma unroll
        for (int ta = 0; ta < 2; ta++)
#pragma unroll
          for (int tb = 0; tb < 4; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][ta], b[u][tb], acc[ta][tb], 0, 0, 0);
  };
  load(0, a0, b0);
  for (int k0 = 0; k0 < n; k0 += 8 * KC) {
    if (k0 + 4 * KC < n) load(k0 + 4 * KC, a1, b1);
    mma(a0, b0, k0);
    if (k0 + 4 * KC >= n) break;
    if (k0 + 8 * KC < n) load(k0 + 8 * KC, a0, b0);
    mma(a1, b1, k0 + 4 * KC);
  }
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 4; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 16 * ta + kq + 4 * q, col = j0 + 16 * tb + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}

// ---- V6: one workgroup per 64-row strip of T over ALL its columns (n <= 256): the H slab is staged once per strip
// (V0 stages it once per 64-column tile, i.e. ceil(n / 64) times), wave w owns the w-th quarter of the 16-column
// MFMA tiles (NT of them) for all 4 row tiles, so a 16-wide K slab is 16 NT MFMAs per wave per barrier pair
template <int NT>
__global__ void __launch_bounds__(256) k_v6(const double *__restrict__ H, int m, int n, int ldh,
                                            const double *__restrict__ P, int ldp, double *__restrict__ T, int ldt) {
  constexpr int HPK = 16, BW = 64 * NT;  // staged B width: 4 waves x NT tiles x 16 columns
  __shared__ double As[64][HPK + 1];
  __shared__ double Bs[HPK][BW + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int i0 = xcd_swizzle(blockIdx.x, gridDim.x) * 64;
  double ra[4], rb[NT * 4];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      const int ar = i0 + (e >> 4), ak = k0 + (e & 15);
      ra[u] = (ar < m && ak < n) ? H[(size_t)ar * ldh + ak] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < NT * 4; u++) {
      const int e = tid + 256 * u;
      const int bk = k0 + e / BW, bc = e % BW;
      rb[u] = (bk < n && bc < n) ? P[(size_t)bk * ldp + bc] : 0.0;
    }
  };
  dbl4 acc[4][NT];
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < NT; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(0);
  for (int k0 = 0; k0 < n; k0 += HPK) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      As[e >> 4][e & 15] = ra[u];
    }
#pragma unroll
    for (int u = 0; u < NT * 4; u++) {
      const int e = tid + 256 * u;
      Bs[e / BW][e % BW] = rb[u];
    }
    __syncthreads();
    if (k0 + HPK < n) load(k0 + HPK);
#pragma unroll
    for (int kk = 0; kk < HPK; kk += 4) {
      double a[4], b[NT];
#pragma unroll
      for (int t = 0; t < 4; t++) a[t] = As[16 * t + r16][kk + kq];
#pragma unroll
      for (int t = 0; t < NT; t++) b[t] = Bs[kk + kq][16 * (NT * w + t) + r16];
#pragma unroll
      for (int ta = 0; ta < 4; ta++)
#pragma unroll
        for (int tb = 0; tb < NT; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int ta = 0; ta < 4; ta++)
#pragma unroll
    for (int tb = 0; tb < NT; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 16 * ta + kq + 4 * q, col = 16 * (NT * w + tb) + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}

// ---- V7: the library's kernel as committed (kernels_chi2.hip k_gemm_HPg_tiled, hidx and zero parameters kept), run
// with hidx = nullptr as the pipeline runs it
__global__ void __launch_bounds__(256) k_lib(const double *__restrict__ H, int m, int n, int ldh,
                                             const double *__restrict__ P, int ldp, const int *__restrict__ hidx,
                                             double *__restrict__ T, int ldt, int *zero) {
  constexpr int HPB = 64, HPK = 16;
  __shared__ double As[HPB][HPK + 1];
  __shared__ double Bs[HPK][HPB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  if (zero && tid == 0 && blockIdx.x == 0) *zero = 0;
  const int tc = (n + HPB - 1) / HPB;
  const int wid = xcd_swizzle(blockIdx.x, gridDim.x), ti = wid / tc;
  const int i0 = ti * HPB, j0 = (wid - ti * tc) * HPB;
  int pcol[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int c = j0 + ((tid + 256 * u) & 63);
    pcol[u] = (c < n) ? (hidx ? hidx[c] : c) : 0;
  }
  double ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      const int ar = i0 + (e >> 4), ak = k0 + (e & 15);
      ra[u] = (ar < m && ak < n) ? H[(size_t)ar * ldh + ak] : 0.0;
      const int bk = k0 + (e >> 6), bc = j0 + (e & 63);
      rb[u] = (bk < n && bc < n) ? P[(size_t)(hidx ? hidx[bk] : bk) * ldp + pcol[u]] : 0.0;
    }
  };
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(0);
  for (int k0 = 0; k0 < n; k0 += HPK) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      As[e >> 4][e & 15] = ra[u];
      Bs[e >> 6][e & 63] = rb[u];
    }
    __syncthreads();
    if (k0 + HPK < n) load(k0 + HPK);
#pragma unroll
    for (int kk = 0; kk < HPK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[t] = As[32 * wr + 16 * t + r16][kk + kq];
        b[t] = Bs[kk + kq][32 * wc + 16 * t + r16];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ta++)
#pragma unroll
        for (int tb = 0; tb < 2; tb++) acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int ta = 0; ta < 2; ta++)
#pragma unroll
    for (int tb = 0; tb < 2; tb++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + 32 * wr + 16 * ta + kq + 4 * q, col = j0 + 32 * wc + 16 * tb + r16;
        if (row < m && col < n) T[(size_t)row * ldt + col] = acc[ta][tb][q];
      }
}
typedef void (*KFn)(const double *, int, int, int, const double *, int, double *, int);

int main(int argc, char **argv) {
  const int ldh = argc > 1 ? std::atoi(argv[1]) : 512;
  const int cold = argc > 2 ? std::atoi(argv[2]) : 0;
  // argv[4] = 1: fragment device memory first (8192 blocks of 256 KiB, every other one freed), as a process that
  // already allocated and freed many buffers (the bench's torch + engine) would have it
  if (argc > 4 && std::atoi(argv[4]) == 1) {
    std::vector<void *> blk(8192);
    for (auto &b : blk) CK(hipMalloc(&b, 256 << 10));
    for (size_t i = 0; i < blk.size(); i += 2) CK(hipFree(blk[i]));
  }
  const size_t scrub_bytes = (size_t)1 << 30;
  void *scrub = nullptr;
  if (cold) CK(hipMalloc(&scrub, scrub_bytes));
  struct Shape {
    const char *name;
    int m, n;
  } shapes[] = {{"cfg5", 74568, 242}, {"cfg4", 80691, 172}, {"cfg3t", 30184, 154}};
  for (const Shape &sh : shapes) {
    const int m = sh.m, n = sh.n;
    std::vector<double> hH((size_t)m * ldh), hP((size_t)n * n);
    unsigned s = 12345;
    auto rnd = [&]() {
      s = s * 1664525u + 1013904223u;
      return ((s >> 8) & 0xffff) / 65536.0 - 0.5;
    };
    for (auto &x : hH) x = rnd();
    for (auto &x : hP) x = rnd();
    // data patterns (argv[3]): 0 random in [-0.5, 0.5); 1 H with 60 % of each row's columns exactly zero, P a
    // covariance-like matrix (1e-2 diagonal, 1e-8 off-diagonal); 2 as 1 with 1e-310 (subnormal) in 5 % of P; 3 all zero
    const int pat = argc > 3 ? std::atoi(argv[3]) : 0;
    if (pat >= 1 && pat <= 2) {
      for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++)
          if ((unsigned)(i * 7 + j * 13) % 10 < 6) hH[(size_t)i * ldh + j] = 0.0;
          else hH[(size_t)i * ldh + j] *= 400.0;
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) hP[(size_t)i * n + j] = (i == j) ? 1e-2 * (1.0 + rnd()) : 1e-8 * rnd();
      if (pat == 2)
        for (int i = 0; i < n; i++)
          for (int j = 0; j < n; j++)
            if ((i * 31 + j * 17) % 20 == 0) hP[(size_t)i * n + j] = 1e-310;
    } else if (pat == 3) {
      for (auto &x : hH) x = 0.0;
      for (auto &x : hP) x = 0.0;
    }
    double *H, *P, *T0, *T1;
    CK(hipMalloc(&H, sizeof(double) * hH.size()));
    CK(hipMalloc(&P, sizeof(double) * hP.size()));
    CK(hipMalloc(&T0, sizeof(double) * (size_t)m * ldh));
    CK(hipMalloc(&T1, sizeof(double) * (size_t)m * ldh));
    CK(hipMemcpy(H, hH.data(), sizeof(double) * hH.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(P, hP.data(), sizeof(double) * hP.size(), hipMemcpyHostToDevice));
    double *Hsrc = nullptr;
    if (cold) {
      CK(hipMalloc(&Hsrc, sizeof(double) * hH.size()));
      CK(hipMemcpy(Hsrc, H, sizeof(double) * hH.size(), hipMemcpyDeviceToDevice));
    }
    const int tc = (n + 63) / 64, g64 = tc * ((m + 63) / 64), g128 = tc * ((m + 127) / 128);
    struct Var {
      const char *name;
      KFn f;
      int grid;
    } vars[] = {{"v0 committed (64x64, K16, 2 barriers)", k_v0<16>, g64},
                {"v0 K32", k_v0<32>, g64},
                {"v2 LDS double buffer K16", k_v2<16>, g64},
                {"v2 LDS double buffer K32", k_v2<32>, g64},
                {"v4 no LDS 32x32/wave KC4", k_v4<4>, g64},
                {"v4 no LDS 32x32/wave KC8", k_v4<8>, g64},
                {"v5 no LDS 32x64/wave KC4", k_v5<4>, g128},
                {"v5 no LDS 32x64/wave KC2", k_v5<2>, g128},
                {"v6 64-row strips, all columns", (n + 15) / 16 <= 12 ? k_v6<3> : k_v6<4>, (m + 63) / 64}};
    std::vector<double> ref((size_t)m * ldh), out((size_t)m * ldh);
    {
      int *zero = nullptr;
      CK(hipMalloc(&zero, sizeof(int)));
      hipEvent_t a0, a1;
      CK(hipEventCreate(&a0));
      CK(hipEventCreate(&a1));
      for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k_lib, dim3(g64), dim3(256), 0, 0, H, m, n, ldh, P, n, (const int *)nullptr, T1, ldh, zero);
      CK(hipEventRecord(a0, 0));
      for (int r = 0; r < 20; r++) hipLaunchKernelGGL(k_lib, dim3(g64), dim3(256), 0, 0, H, m, n, ldh, P, n, (const int *)nullptr, T1, ldh, zero);
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a0, a1));
      std::printf("%-6s m %6d n %3d  %-40s %8.1f us\n", sh.name, m, n, "library kernel (hidx = nullptr)", 1e3 * ms / 20);
      CK(hipFree(zero));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int v = 0; v < (int)(sizeof(vars) / sizeof(vars[0])); v++) {
      double *Tv = v ? T1 : T0;
      CK(hipMemset(Tv, 0, sizeof(double) * (size_t)m * ldh));
      for (int r = 0; r < 3; r++) hipLaunchKernelGGL(vars[v].f, dim3(vars[v].grid), dim3(256), 0, 0, H, m, n, ldh, P, n, Tv, ldh);
      CK(hipDeviceSynchronize());
      const int reps = 20;
      double us = 0;
      if (!cold) {
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(vars[v].f, dim3(vars[v].grid), dim3(256), 0, 0, H, m, n, ldh, P, n, Tv, ldh);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        us = 1e3 * ms / reps;
      } else {  // H rewritten (as k_feature does) and a 1 GB scrub between launches: cold caches
        for (int r = 0; r < reps; r++) {
          if (cold == 1) {  // H rewritten last: fresh in the caches, everything else evicted
            CK(hipMemsetAsync(scrub, r & 0xff, scrub_bytes, 0));
            CK(hipMemcpyAsync(H, Hsrc, sizeof(double) * (size_t)m * ldh, hipMemcpyDeviceToDevice, 0));
          } else {  // cold == 2: H rewritten, then 1 GB scrubbed: H and P from HBM
            CK(hipMemcpyAsync(H, Hsrc, sizeof(double) * (size_t)m * ldh, hipMemcpyDeviceToDevice, 0));
            CK(hipMemsetAsync(scrub, r & 0xff, scrub_bytes, 0));
          }
          CK(hipEventRecord(e0, 0));
          hipLaunchKernelGGL(vars[v].f, dim3(vars[v].grid), dim3(256), 0, 0, H, m, n, ldh, P, n, Tv, ldh);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          us += 1e3 * ms / reps;
        }
      }
      CK(hipMemcpy((v ? out : ref).data(), Tv, sizeof(double) * (size_t)m * ldh, hipMemcpyDeviceToHost));
      long long diff = 0;
      if (v)
        for (int i = 0; i < m; i++)
          for (int j = 0; j < n; j++)
            if (std::memcmp(&out[(size_t)i * ldh + j], &ref[(size_t)i * ldh + j], 8) != 0) diff++;
      std::printf("frag %d pat %d %s ldh %d %-6s m %6d n %3d  %-40s %8.1f us  %5.1f TFLOP/s  differing %lld\n", argc > 4 ? std::atoi(argv[4]) : 0, pat, cold == 2 ? "cold-hbm" : cold ? "cold" : "warm", ldh, sh.name, m, n, vars[v].name, us,
                  2.0 * m * n * n / us * 1e-6, diff);
      std::fflush(stdout);
    }
    CK(hipFree(H));
    CK(hipFree(P));
    CK(hipFree(T0));
    CK(hipFree(T1));
    if (Hsrc) CK(hipFree(Hsrc));
  }
  return 0;
}
