// Host round-trip costs on one MI355X: what a launch -> readback -> wait cycle costs the host and how long
// the device sits idle around it.  Variants: D2H through hipMemcpyAsync into pinned memory vs the kernel
// writing pinned host memory itself; H2D staging copy vs the kernel reading pinned memory; blocking vs
// spinning synchronization.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 tools/bench_sync.hip -o build/bench_sync
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void k_work(const double *in, double *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 2.0 + 1.0;
}

// the last block to finish raises a flag in mapped host memory (system-scope release)
__global__ void k_work_flag(const double *in, double *out, int n, unsigned *count, volatile int *flag, int seq) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 2.0 + 1.0;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    if (atomicAdd(count, 1u) == gridDim.x - 1) {
      *count = 0;
      __threadfence_system();
      __hip_atomic_store((int *)flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main(int argc, char **argv) {
  const int spin = argc > 1 ? atoi(argv[1]) : 0;
  if (spin == 1) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  if (spin == 2) CK(hipSetDeviceFlags(hipDeviceScheduleYield));
  if (spin == 3) CK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = 1024;  // 8 KB
  double *din, *dout, *hpin, *hmap;
  CK(hipMalloc(&din, n * 8));
  CK(hipMalloc(&dout, n * 8));
  CK(hipHostMalloc(&hpin, n * 8, hipHostMallocDefault));
  CK(hipHostMalloc(&hmap, n * 8, hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < n; i++) hpin[i] = hmap[i] = i;
  double *hmap_dev = nullptr;
  CK(hipHostGetDevicePointer((void **)&hmap_dev, hmap, 0));
  const int iters = 2000;
  const char *names[] = {"launch only (no wait)", "launch+sync", "launch+D2H copy+sync", "launch writes pinned+sync",
                         "H2D copy+launch+D2H copy+sync", "launch reads+writes pinned+sync", "3 launches+sync",
                         "hipMemcpyAsync H2D only (no wait)", "launch raises host flag + host polls"};
  unsigned *dcount;
  CK(hipMalloc(&dcount, 4));
  CK(hipMemset(dcount, 0, 4));
  int *hflag, *hflag_dev;
  CK(hipHostMalloc(&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  *hflag = 0;
  CK(hipHostGetDevicePointer((void **)&hflag_dev, hflag, 0));
  int seq = 0;
  for (int v = 0; v < 9; v++) {
    for (int w = 0; w < 2; w++) {  // warm-up pass, then the timed pass
      CK(hipStreamSynchronize(s));
      auto t0 = clk::now();
      double host_launch = 0;
      for (int it = 0; it < iters; it++) {
        auto a = clk::now();
        switch (v) {
          case 0: k_work<<<n / 256, 256, 0, s>>>(din, dout, n); break;
          case 1: k_work<<<n / 256, 256, 0, s>>>(din, dout, n); break;
          case 2:
            k_work<<<n / 256, 256, 0, s>>>(din, dout, n);
            CK(hipMemcpyAsync(hpin, dout, n * 8, hipMemcpyDeviceToHost, s));
            break;
          case 3: k_work<<<n / 256, 256, 0, s>>>(din, hmap_dev, n); break;
          case 4:
            CK(hipMemcpyAsync(din, hpin, n * 8, hipMemcpyHostToDevice, s));
            k_work<<<n / 256, 256, 0, s>>>(din, dout, n);
            CK(hipMemcpyAsync(hpin, dout, n * 8, hipMemcpyDeviceToHost, s));
            break;
          case 5: k_work<<<n / 256, 256, 0, s>>>(hmap_dev, hmap_dev, n); break;
          case 6:
            k_work<<<n / 256, 256, 0, s>>>(din, dout, n);
            k_work<<<n / 256, 256, 0, s>>>(dout, din, n);
            k_work<<<n / 256, 256, 0, s>>>(din, dout, n);
            break;
          case 7: CK(hipMemcpyAsync(din, hpin, n * 8, hipMemcpyHostToDevice, s)); break;
          case 8: k_work_flag<<<n / 256, 256, 0, s>>>(din, hmap_dev, n, dcount, hflag_dev, ++seq); break;
        }
        auto b = clk::now();
        host_launch += us(a, b);
        if (v == 8) {
          long spins = 0;
          while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq)
            if (++spins > 2000000000L) {
              printf("flag never raised\n");
              return 1;
            }
        } else if (v != 0 && v != 7) {
          CK(hipStreamSynchronize(s));
        }
      }
      CK(hipStreamSynchronize(s));
      auto t1 = clk::now();
      if (w == 1)
        printf("sched %d  %-36s  %7.2f us/iter  (host enqueue %6.2f us)\n", spin, names[v], us(t0, t1) / iters,
               host_launch / iters);
    }
  }
  return 0;
}
