// Microbenchmark of the KLT front-end kernels (kernels_track.hip) on a synthetic 752x480 stereo-like
// pair: per-kernel average time over repetitions (HIP events).
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include tools/bench_track.hip -o build/bench_track
#include "../uvio_amd/csrc/kernels_track.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace uvhp;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static unsigned hsh(unsigned a, unsigned b) {
  unsigned h = a * 73856093u ^ b * 19349663u;
  h = (h ^ (h >> 13)) * 1274126177u;
  return h ^ (h >> 16);
}
static float scene(float x, float y) {  // tiles + value noise
  int tx = (int)floorf(x / 18.f), ty = (int)floorf(y / 18.f);
  float base = 35.f + 185.f * (hsh(tx, ty) & 0xffff) / 65535.f;
  int nx = (int)floorf(x / 4.5f), ny = (int)floorf(y / 4.5f);
  return base + 36.f * ((hsh(nx + 7, ny) & 0xffff) / 65535.f - 0.5f);
}

struct Pyr {
  DPyr p{};
  void alloc(int w, int h) {
    int lw = w, lh = h;
    for (int l = 0; l < 5; l++) {
      p.w[l] = lw;
      p.h[l] = lh;
      uint8_t *a;
      int16_t *d;
      CK(hipMalloc(&a, lw * lh));
      CK(hipMalloc(&d, lw * lh * 4));
      p.img[l] = a;
      p.der[l] = d;
      p.levels = l + 1;
      lw = (lw + 1) / 2;
      lh = (lh + 1) / 2;
      if (lw <= 15 || lh <= 15) break;
    }
  }
};

int main(int argc, char **argv) {
  const int W = 752, H = 480, reps = argc > 1 ? atoi(argv[1]) : 20;
  std::vector<uint8_t> i0(W * H), i1(W * H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      i0[y * W + x] = (uint8_t)std::min(255.f, std::max(0.f, scene(x, y) + (hsh(x, y + 999) % 5) - 2.f));
      i1[y * W + x] = (uint8_t)std::min(255.f, std::max(0.f, scene(x + 2.3f, y - 1.7f) + (hsh(x + 5, y) % 5) - 2.f));
    }
  uint8_t *d0, *d1;
  unsigned *hist;
  CK(hipMalloc(&d0, W * H));
  CK(hipMalloc(&d1, W * H));
  CK(hipMalloc(&hist, 1024));
  CK(hipMemcpy(d0, i0.data(), W * H, hipMemcpyHostToDevice));
  CK(hipMemcpy(d1, i1.data(), W * H, hipMemcpyHostToDevice));
  Pyr A, B;
  A.alloc(W, H);
  B.alloc(W, H);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto fn) {
    fn();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; r++) fn();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %9.1f us\n", name, 1e3 * ms / reps);
  };
  timeit("equalize+pyramid (1 img)", [&] {
    launch_equalize(s, d0, W, H, W, 1, hist, (uint8_t *)A.p.img[0]);
    launch_pyramid(s, A.p);
  });
  launch_equalize(s, d1, W, H, W, 1, hist, (uint8_t *)B.p.img[0]);
  launch_pyramid(s, B.p);
  // FAST on all 25 cells of 150 x 96
  const int gx = 5, gy = 5, sw = W / gx, sh = H / gy, kmax = 9;
  std::vector<int> cells;
  for (int x = 0; x < gx; x++)
    for (int y = 0; y < gy; y++) {
      cells.push_back(x * sw);
      cells.push_back(y * sh);
    }
  int *dcells, *dn;
  uint8_t *dscore;
  CK(hipMalloc(&dscore, W * H));
  float *dout;
  CK(hipMalloc(&dcells, cells.size() * 4));
  CK(hipMalloc(&dn, 25 * 4));
  CK(hipMalloc(&dout, 25 * kmax * 3 * 4));
  CK(hipMemcpy(dcells, cells.data(), cells.size() * 4, hipMemcpyHostToDevice));
  for (int thr : {10, 20, 40}) {
    char nm[64];
    snprintf(nm, 64, "fast 25 cells thr %d", thr);
    timeit(nm, [&] { launch_fast_cells(s, A.p.img[0], W, H, dcells, 25, sw, sh, thr, kmax, dout, dn, dscore); });
  }
  timeit("fast score only thr 20", [&] {
    hipLaunchKernelGGL(k_fast_score, dim3(25, (sh + kFastBand - 1) / kFastBand), dim3(256), 0, s, A.p.img[0], W, dcells,
                       sw, sh, 20, dscore);
  });
  timeit("fast select only", [&] {
    hipLaunchKernelGGL(k_fast_select, dim3(25), dim3(kFastThreads), fast_lds_bytes(sw, sh), s, dscore, W, dcells, sw, sh,
                       kmax, dout, dn);
  });
  timeit("empty kernel", [&] { hipLaunchKernelGGL(k_hist, dim3(1), dim3(256), 0, s, d0, 1, 1, 1, hist); });
  launch_fast_cells(s, A.p.img[0], W, H, dcells, 25, sw, sh, 20, kmax, dout, dn, dscore);
  std::vector<float> fo(25 * kmax * 3);
  std::vector<int> fn(25);
  CK(hipMemcpy(fo.data(), dout, fo.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(fn.data(), dn, 100, hipMemcpyDeviceToHost));
  std::vector<float> pts;
  for (int c = 0; c < 25; c++)
    for (int i = 0; i < fn[c]; i++) {
      pts.push_back(fo[(c * kmax + i) * 3]);
      pts.push_back(fo[(c * kmax + i) * 3 + 1]);
    }
  int n = (int)pts.size() / 2;
  printf("fast points: %d\n", n);
  float *dp, *dq, *mask;
  uint8_t *st;
  CK(hipMalloc(&dp, 8 * 4096));
  CK(hipMalloc(&dq, 8 * 4096));
  CK(hipMalloc(&st, 4096));
  CK(hipMalloc(&mask, 121 * 4));
  std::vector<float> mk(121);
  for (int i = 0; i < 11; i++)
    for (int j = 0; j < 11; j++) {
      float y = (float)(i - 5) / 5, x = (float)(j - 5) / 5;
      mk[i * 11 + j] = (float)(std::exp(-y * y) * std::exp(-x * x));
    }
  CK(hipMemcpy(mask, mk.data(), 121 * 4, hipMemcpyHostToDevice));
  timeit("subpix", [&] {
    CK(hipMemcpyAsync(dp, pts.data(), n * 8, hipMemcpyHostToDevice, s));
    launch_subpix(s, A.p.img[0], W, H, dp, n, mask, 5, 20, 1e-6);
  });
  // LK on a 200-point grid
  std::vector<float> g;
  for (int i = 0; i < 200; i++) {
    g.push_back(40.f + (i % 20) * 34.f + 0.37f);
    g.push_back(40.f + (i / 20) * 40.f + 0.61f);
  }
  CK(hipMemcpy(dp, g.data(), g.size() * 4, hipMemcpyHostToDevice));
  timeit("lk 200 pts", [&] {
    LkSlots lk{};
    lk.prev[0] = A.p;
    lk.next[0] = B.p;
    lk.p0[0] = dp;
    lk.p1[0] = dq;
    lk.st[0] = st;
    lk.n[0] = 200;
    launch_lk(s, lk, 1, 15, 5, 30, 0.01f, true);
  });
  std::vector<float> q(400);
  std::vector<uint8_t> sv(200);
  CK(hipMemcpy(q.data(), dq, 1600, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sv.data(), st, 200, hipMemcpyDeviceToHost));
  double ex = 0, ey = 0;
  int ok = 0;
  for (int i = 0; i < 200; i++)
    if (sv[i]) {
      ok++;
      ex += q[2 * i] - g[2 * i];
      ey += q[2 * i + 1] - g[2 * i + 1];
    }
  printf("lk ok %d mean flow (%.3f, %.3f) (expect -2.3, 1.7)\n", ok, ex / ok, ey / ok);
  return 0;
}
