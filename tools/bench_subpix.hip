// Microbenchmark of k_subpix (cornerSubPix, kernels_track.hip) on a synthetic 752x480 tiled image: corners
// near the tile junctions (where the refinement iterates) plus flat-area starts (where it stops at once), per-launch
// time over repetitions (HIP events) and a digest of the refined points to compare kernel versions bit for bit.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I uvio_amd/csrc \
//          tools/bench_subpix.hip -o build/bench_subpix
#include "../uvio_amd/csrc/kernels_track.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace uvhp;

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

static unsigned hsh(unsigned a, unsigned b) {
  unsigned h = a * 73856093u ^ b * 19349663u;
  h = (h ^ (h >> 13)) * 1274126177u;
  return h ^ (h >> 16);
}
static float scene(float x, float y) {  // 18-pixel tiles + value noise
  int tx = (int)floorf(x / 18.f), ty = (int)floorf(y / 18.f);
  float base = 35.f + 185.f * (hsh(tx, ty) & 0xffff) / 65535.f;
  int nx = (int)floorf(x / 4.5f), ny = (int)floorf(y / 4.5f);
  return base + 36.f * ((hsh(nx + 7, ny) & 0xffff) / 65535.f - 0.5f);
}

int main(int argc, char **argv) {
  const int W = 752, H = 480, reps = argc > 1 ? atoi(argv[1]) : 50;
  std::vector<uint8_t> im(W * H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++)
      im[y * W + x] = (uint8_t)std::min(255.f, std::max(0.f, scene(x, y) + (hsh(x, y + 999) % 5) - 2.f));
  uint8_t *dimg;
  CK(hipMalloc(&dimg, W * H));
  CK(hipMemcpy(dimg, im.data(), W * H, hipMemcpyHostToDevice));
  std::vector<float> mk(121);
  for (int i = 0; i < 11; i++)
    for (int j = 0; j < 11; j++) {
      float y = (float)(i - 5) / 5, x = (float)(j - 5) / 5;
      mk[i * 11 + j] = (float)(std::exp(-y * y) * std::exp(-x * x));
    }
  float *mask, *dp;
  CK(hipMalloc(&mask, 121 * 4));
  CK(hipMemcpy(mask, mk.data(), 121 * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&dp, 8 * 4096));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int n : {100, 300, 800}) {
    std::vector<float> pts;
    for (int i = 0; pts.size() < 2 * (size_t)n; i++) {
      const unsigned r = hsh(i, n);
      const int tx = 1 + (int)(r % 40), ty = 1 + (int)((r >> 8) % 25);
      const float jx = (float)((r >> 16) % 7) - 3.f + 0.25f * ((r >> 20) & 3), jy = (float)((r >> 24) % 7) - 3.f;
      pts.push_back(std::min(W - 8.f, 18.f * tx + jx));
      pts.push_back(std::min(H - 8.f, 18.f * ty + jy));
    }
    CK(hipMemcpy(dp, pts.data(), n * 8, hipMemcpyHostToDevice));
    launch_subpix(s, dimg, W, H, dp, n, mask, 5, 20, 1e-6);
    CK(hipStreamSynchronize(s));
    float tot = 0;
    for (int r = 0; r < reps; r++) {
      CK(hipMemcpyAsync(dp, pts.data(), n * 8, hipMemcpyHostToDevice, s));
      CK(hipEventRecord(e0, s));
      launch_subpix(s, dimg, W, H, dp, n, mask, 5, 20, 1e-6);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
    }
    std::vector<unsigned> out(2 * n);
    CK(hipMemcpy(out.data(), dp, n * 8, hipMemcpyDeviceToHost));
    unsigned long long hsum = 1469598103934665603ull;
    for (unsigned u : out) hsum = (hsum ^ u) * 1099511628211ull;
    int moved = 0;
    for (int i = 0; i < 2 * n; i++) moved += ((const float *)out.data())[i] != pts[i];
    printf("subpix n %4d  %8.1f us/launch  digest %016llx  moved coords %d\n", n, 1e3 * tot / reps, hsum, moved);
  }
  return 0;
}
