// Dependent-chain latencies of the primitives the single-wave factorization steps are made of (one wave,
// clock64 around 256 chained operations).  Build: hipcc -x hip --offload-arch=gfx950 -O3 tools/bench_lat.hip -o build/bench_lat
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(double *io, long long *out) {
  __shared__ double sh[64];
  double x = io[threadIdx.x], y = io[64 + threadIdx.x];
  long long t0, t1;
  // 1) dependent f64 FMA
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) x = fma(x, y, 0.5);
  t1 = clock64();
  out[0] = t1 - t0;
  // 2) dependent v_rcp_f64
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) x = __builtin_amdgcn_rcp(x + 1.0);
  t1 = clock64();
  out[1] = t1 - t0;
  // 3) dependent IEEE division
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) x = 1.0 / (x + 1.0);
  t1 = clock64();
  out[2] = t1 - t0;
  // 4) LDS store -> broadcast load round trip
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) {
    if (threadIdx.x == (i & 15)) sh[i & 15] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    x = sh[i & 15] + 1.0;
  }
  t1 = clock64();
  out[3] = t1 - t0;
  // 5) v_readlane round trip (double)
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) {
    unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    unsigned lo = __builtin_amdgcn_readlane((unsigned)u, 5), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), 5);
    x = __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo) + 1.0;
  }
  t1 = clock64();
  out[4] = t1 - t0;
  // 6) independent f64 FMAs (issue rate): 8 chains
  double z[8];
  for (int k = 0; k < 8; k++) z[k] = x + k;
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 32; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) z[k] = fma(z[k], y, 0.5);
  t1 = clock64();
  out[5] = t1 - t0;
  // 7) dependent MFMA f64 16x16x4
  typedef double dbl4 __attribute__((ext_vector_type(4)));
  dbl4 acc = {x, y, x, y};
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  t1 = clock64();
  out[6] = t1 - t0;
  // 8) s_barrier alone (one wave per block here: 8 waves in the 512 launch)
  t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < 256; i++) __syncthreads();
  t1 = clock64();
  out[7] = t1 - t0;
  double s = x + acc[0] + acc[1] + acc[2] + acc[3];
  for (int k = 0; k < 8; k++) s += z[k];
  io[128 + threadIdx.x] = s;
}

int main() {
  double *io;
  long long *out;
  (void)hipMalloc(&io, 8 * 1024);
  (void)hipMalloc(&out, 8 * 16);
  (void)hipMemset(io, 0, 8 * 1024);
  const char *names[] = {"dep v_fma_f64", "dep v_rcp_f64", "dep 1.0/x (IEEE)", "LDS store->bcast load", "readlane pair",
                         "indep fma_f64 (per instr)", "dep mfma_f64_16x16x4", "__syncthreads (8 waves)"};
  for (int threads : {64, 512}) {
    for (int it = 0; it < 3; it++) {
      hipLaunchKernelGGL(k_lat, dim3(1), dim3(threads), 0, 0, io, out);
      if (hipDeviceSynchronize() != hipSuccess) return 1;
    }
    long long h[8];
    (void)hipMemcpy(h, out, 64, hipMemcpyDeviceToHost);
    printf("block %d threads:\n", threads);
    for (int k = 0; k < 8; k++) printf("  %-28s %7.1f cycles\n", names[k], h[k] / 256.0);
  }
  return 0;
}
