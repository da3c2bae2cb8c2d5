// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the tracker kernels use
// (MI355X_MICROARCH.md "HBM": FETCH_SIZE reads half of a 16 B/lane streaming read; other widths uncalibrated).
// Each kernel moves a known byte count once over a 256 MiB buffer: coalesced loads / stores of 1, 2, 4, 8 and
// 16 bytes per lane, and the LK / pyramid patterns (a byte and a dword gather of 4 bilinear taps per pixel over
// 16 x 16 windows).  Run one PMC counter per pass:
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o run -- build/bench_fetch
//   rocprofv3 --pmc WRITE_SIZE ...
// then tools/fetch_calib.py joins the kernel names with the byte counts printed here.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 tools/bench_fetch.hip -o build/bench_fetch
#include <hip/hip_runtime.h>

#include <cstdint>
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

template <class T>
__global__ void k_read(const T *__restrict__ a, size_t n, unsigned long long *sink) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  for (; i < n; i += stride) {
    const T v = a[i];
    unsigned long long w = 0;
    __builtin_memcpy(&w, &v, sizeof(T) < 8 ? sizeof(T) : 8);
    acc = acc * 31 + w;
  }
  if (acc == 0x1234567ull) sink[0] = acc;  // keeps the loads
}

template <class T>
__global__ void k_write(T *__restrict__ a, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  T v;
  unsigned char *b = reinterpret_cast<unsigned char *>(&v);
  for (size_t k = 0; k < sizeof(T); k++) b[k] = (unsigned char)k;
  for (; i < n; i += stride) a[i] = v;
}

// LK-like: one 64-lane block per window, 16 x 16 window of 1-byte pixels and 4-byte derivatives, 4 bilinear taps
// each (img[o], img[o+1], img[o+w], img[o+w+1]); windows tile the image without overlap, so the unique bytes are
// the windows plus one extra row / column of taps
__global__ void k_gather_lk(const uint8_t *__restrict__ img, const int *__restrict__ der, int w, int h,
                            unsigned long long *sink) {
  const int wx = w / 17, bx = blockIdx.x % wx, by = blockIdx.x / wx;
  const int x0 = bx * 17, y0 = by * 17;
  unsigned long long acc = 0;
  for (int e = threadIdx.x; e < 256; e += 64) {
    const int x = x0 + (e & 15), y = y0 + (e >> 4);
    const size_t o = (size_t)y * w + x;
    acc += img[o] + img[o + 1] + img[o + w] + img[o + w + 1];
    acc += (unsigned)(der[o] + der[o + 1] + der[o + w] + der[o + w + 1]);
  }
  if (acc == 0x1234567ull) sink[0] = acc;
}

int main() {
  const size_t bytes = 256ull << 20;
  void *buf;
  unsigned long long *sink;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, bytes));
  const int grid = 256 * 16, block = 256;
  printf("kernel,bytes\n");
#define RD(T, NAME)                                                                                    \
  hipLaunchKernelGGL(k_read<T>, dim3(grid), dim3(block), 0, 0, (const T *)buf, bytes / sizeof(T), sink); \
  printf("k_read<%s>,%zu\n", NAME, bytes);
#define WR(T, NAME)                                                                       \
  hipLaunchKernelGGL(k_write<T>, dim3(grid), dim3(block), 0, 0, (T *)buf, bytes / sizeof(T)); \
  printf("k_write<%s>,%zu\n", NAME, bytes);
  // names as the trace demangles them
  RD(uint8_t, "unsigned char") RD(uint16_t, "unsigned short") RD(uint32_t, "unsigned int")
  RD(uint64_t, "unsigned long") RD(uint4, "HIP_vector_type<unsigned int, 4u>")
  WR(uint8_t, "unsigned char") WR(uint16_t, "unsigned short") WR(uint32_t, "unsigned int")
  WR(uint64_t, "unsigned long") WR(uint4, "HIP_vector_type<unsigned int, 4u>")
  // LK-like gathers over a 8192 x 4096 image (32 MiB of pixels, 128 MiB of derivatives)
  const int w = 8192, h = 4096;
  uint8_t *img = (uint8_t *)buf;
  int *der = (int *)((char *)buf + (size_t)w * h);
  const int nwin = (w / 17) * ((h - 1) / 17);
  hipLaunchKernelGGL(k_gather_lk, dim3(nwin), dim3(64), 0, 0, img, der, w, h, sink);
  // unique bytes: per window 17 x 17 pixels (taps) of 1 + 4 bytes
  printf("k_gather_lk,%zu\n", (size_t)nwin * 17 * 17 * 5);
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
