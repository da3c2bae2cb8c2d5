// Cycle breakdown of the pyramidal LK kernel (kernels_track.hip lk_point, built with UVHP_LK_PROF) on a
// synthetic 752x480 pair shifted by (2.3, -1.7) px: per point the cycles of the level setups (prev window
// gather + gradient matrix), the J staging rounds and the iterations, and the kernel time (HIP events).
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DUVHP_LK_PROF -I include
//        tools/bench_lk.hip -o build/bench_lk
#include "../uvio_amd/csrc/kernels_track.hip"

#include <algorithm>
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
static float scene(float x, float y) {  // tiles + value noise
  int tx = (int)floorf(x / 18.f), ty = (int)floorf(y / 18.f);
  float base = 35.f + 185.f * (hsh(tx, ty) & 0xffff) / 65535.f;
  int nx = (int)floorf(x / 4.5f), ny = (int)floorf(y / 4.5f);
  return base + 36.f * ((hsh(nx + 7, ny) & 0xffff) / 65535.f - 0.5f);
}

static DPyr alloc_pyr(int w, int h, int levels) {
  DPyr p{};
  for (int l = 0; l < levels; l++) {
    uint8_t *a;
    int16_t *d;
    CK(hipMalloc(&a, (size_t)w * h));
    CK(hipMalloc(&d, (size_t)w * h * 4));
    p.img[l] = a;
    p.der[l] = d;
    p.w[l] = w;
    p.h[l] = h;
    p.levels = l + 1;
    w = (w + 1) / 2;
    h = (h + 1) / 2;
  }
  return p;
}

int main(int argc, char **argv) {
  const int W = 752, H = 480, L = 6, npts = argc > 1 ? atoi(argv[1]) : 400, reps = 20;
  std::vector<uint8_t> i0(W * H), i1(W * H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      i0[y * W + x] = (uint8_t)std::min(255.f, std::max(0.f, scene(x, y) + (hsh(x, y + 999) % 5) - 2.f));
      i1[y * W + x] = (uint8_t)std::min(255.f, std::max(0.f, scene(x + 2.3f, y - 1.7f) + (hsh(x + 5, y) % 5) - 2.f));
    }
  uint8_t *s0, *s1;
  CK(hipMalloc(&s0, W * H));
  CK(hipMalloc(&s1, W * H));
  CK(hipMemcpy(s0, i0.data(), W * H, hipMemcpyHostToDevice));
  CK(hipMemcpy(s1, i1.data(), W * H, hipMemcpyHostToDevice));
  unsigned *hist;
  CK(hipMalloc(&hist, 2 * 256 * 4));
  PyrJob pj{};
  pj.p[0] = alloc_pyr(W, H, L);
  pj.p[1] = alloc_pyr(W, H, L);
  pj.src[0] = s0;
  pj.src[1] = s1;
  pj.stride[0] = pj.stride[1] = W;
  pj.hist[0] = hist;
  pj.hist[1] = hist + 256;
  pj.ncam = 2;
  pj.equalize = 1;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  launch_pyramids(s, pj);
  std::vector<float> g;
  for (int i = 0; i < npts; i++) {
    g.push_back(20.f + (i % 25) * 28.7f + 0.37f);
    g.push_back(20.f + (i / 25) * (440.f / ((npts + 24) / 25)) + 0.61f);
  }
  float *dp, *dq;
  uint8_t *st;
  CK(hipMalloc(&dp, 8 * npts));
  CK(hipMalloc(&dq, 8 * npts));
  CK(hipMalloc(&st, npts));
  CK(hipMemcpy(dp, g.data(), g.size() * 4, hipMemcpyHostToDevice));
  LkSlots lk{};
  lk.prev[0] = pj.p[0];
  lk.next[0] = pj.p[1];
  lk.p0[0] = dp;
  lk.p1[0] = dq;
  lk.st[0] = st;
  lk.n[0] = npts;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f, sum = 0.f;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(e0, s));
    launch_lk(s, lk, 1, 15, L - 1, 30, 0.01f, true);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
    sum += ms;
  }
  printf("k_lk %d points, %d levels: best %.1f us, mean %.1f us\n", npts, L, 1e3f * best, 1e3f * sum / reps);
  {  // results digest (FNV-1a over the tracked points and statuses): equal digests = bit-identical results
    std::vector<float> q(2 * npts);
    std::vector<uint8_t> sv(npts);
    CK(hipMemcpy(q.data(), dq, 8 * npts, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sv.data(), st, npts, hipMemcpyDeviceToHost));
    unsigned long long hsum = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
      for (size_t i = 0; i < n; i++) hsum = (hsum ^ ((const uint8_t *)p)[i]) * 1099511628211ull;
    };
    mix(q.data(), q.size() * 4);
    mix(sv.data(), sv.size());
    int ok = 0;
    for (auto v : sv) ok += v;
    printf("results digest %016llx  tracked %d of %d\n", hsum, ok, npts);
  }
#ifdef UVHP_LK_PROF
  std::vector<LkProf> pr(npts);
  CK(hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(g_lk_prof), npts * sizeof(LkProf)));
  std::vector<int> idx(npts);
  for (int i = 0; i < npts; i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](int a, int b) { return pr[a].total > pr[b].total; });
  double ms = 0, mst = 0, mi = 0, mt = 0, ni = 0, nst = 0;
  for (auto &q : pr) {
    ms += q.setup, mst += q.stage, mi += q.iter, mt += q.total, ni += q.n_iter, nst += q.n_stage;
  }
  printf("mean cycles: total %.0f  setup %.0f  stage %.0f (%.2f rounds)  iter %.0f (%.1f iterations, %.0f per iteration)\n",
         mt / npts, ms / npts, mst / npts, nst / npts, mi / npts, ni / npts, mi / std::max(ni, 1.0));
  printf("slowest points: total  setup  stage(n)  iter(n)  levels\n");
  for (int k = 0; k < 8 && k < npts; k++) {
    const LkProf &q = pr[idx[k]];
    printf("  %5d  %8llu %6llu %6llu(%d) %7llu(%d) %d  per-iter %.0f\n", idx[k], q.total, q.setup, q.stage, q.n_stage,
           q.iter, q.n_iter, q.n_level, q.n_iter ? (double)q.iter / q.n_iter : 0.0);
  }
#endif
  return 0;
}
