// ORACLE — test infrastructure only (see la.h header).  KLT front-end restatement, see tracker.h.
#include "tracker.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>

#include "feat.h"

namespace orc {

// cv::parallel_for_ stand-in for the CPU baseline: the reference's configs run OpenCV with
// num_opencv_threads 4 (config/*/estimator_config.yaml:87-89), and calcOpticalFlowPyrLK (per point),
// pyrDown and the Scharr derivatives (per row) are the parallel OpenCV calls of the KLT front-end.
// Work items are independent, so the results do not depend on the thread count (tests compare 1 vs 4).
namespace {
struct CvPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  const std::function<void(size_t, size_t)> *job = nullptr;
  size_t n = 0, chunks = 0, next = 0, done = 0;
  long gen = 0;
  bool stop = false;
  ~CvPool() { resize(0); }
  void resize(int k) {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
    th.clear();
    stop = false;
    for (int i = 0; i < k; i++) th.emplace_back([this] { loop(); });
  }
  void loop() {
    long seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> l(mu);
      cv.wait(l, [&] { return stop || (job && gen != seen); });
      if (stop) return;
      seen = gen;
      work(l);
    }
  }
  // claims chunks until none is left (called with the lock held)
  void work(std::unique_lock<std::mutex> &l) {
    while (next < chunks) {
      const size_t c = next++;
      const auto *f = job;
      const size_t lo = n * c / chunks, hi = n * (c + 1) / chunks;
      l.unlock();
      (*f)(lo, hi);
      l.lock();
      if (++done == chunks) done_cv.notify_all();
    }
  }
  void run(size_t count, const std::function<void(size_t, size_t)> &f) {
    std::unique_lock<std::mutex> l(mu);
    job = &f;
    n = count;
    chunks = std::min(count, (size_t)(4 * (th.size() + 1)));
    next = done = 0;
    gen++;
    cv.notify_all();
    work(l);
    done_cv.wait(l, [&] { return done == chunks; });
    job = nullptr;
  }
};
CvPool g_pool;
int g_threads = 1;
}  // namespace

void set_cv_threads(int k) {
  k = std::max(1, k);
  if (k == g_threads) return;
  g_pool.resize(k - 1);
  g_threads = k;
}
int cv_threads() { return g_threads; }
void cv_parallel_for(size_t n, const std::function<void(size_t, size_t)> &f) {
  if (g_threads <= 1 || n < 2) {
    if (n) f(0, n);
    return;
  }
  g_pool.run(n, f);
}

static inline int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = (p < 0) ? -p : 2 * n - 2 - p;
  return p;
}
static inline uint8_t sat_u8_round(float v) {
  int r = (int)std::nearbyint(v);  // cvRound: round half to even
  return (uint8_t)std::min(255, std::max(0, r));
}

// cv::equalizeHist (histogram.cpp EqualizeHistLut_Invoker)
GrayImg equalize_hist(const GrayImg &src) {
  int hist[256] = {0};
  for (uint8_t v : src.d) hist[v]++;
  GrayImg dst = src;
  int i = 0;
  while (!hist[i]) ++i;
  int total = (int)src.d.size();
  if (hist[i] == total) {
    std::fill(dst.d.begin(), dst.d.end(), (uint8_t)i);
    return dst;
  }
  float scale = (256 - 1.f) / (total - hist[i]);
  int lut[256];
  int sum = 0;
  for (lut[i++] = 0; i < 256; ++i) {
    sum += hist[i];
    lut[i] = sat_u8_round(sum * scale);
  }
  for (auto &v : dst.d) v = (uint8_t)lut[v];
  return dst;
}

// cv::pyrDown (pyramids.cpp pyrDown_): 5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101, rounding (+128)>>8
GrayImg pyr_down(const GrayImg &src) {
  GrayImg dst;
  dst.w = (src.w + 1) / 2;
  dst.h = (src.h + 1) / 2;
  dst.d.resize((size_t)dst.w * dst.h);
  static const int k[5] = {1, 4, 6, 4, 1};
  cv_parallel_for((size_t)dst.h, [&](size_t y0, size_t y1) {
    for (int y = (int)y0; y < (int)y1; y++)
      for (int x = 0; x < dst.w; x++) {
        int acc = 0;
        for (int i = 0; i < 5; i++) {
          int sy = reflect101(2 * y + i - 2, src.h);
          int row = 0;
          for (int j = 0; j < 5; j++) row += k[j] * src.at(reflect101(2 * x + j - 2, src.w), sy);
          acc += k[i] * row;
        }
        dst.d[(size_t)y * dst.w + x] = (uint8_t)((acc + 128) >> 8);
      }
  });
  return dst;
}

// calcSharrDeriv (lkpyramid.cpp): dx = [3 10 3]^T (x) [-1 0 1], dy = its transpose, reflect-101 borders
std::vector<int16_t> scharr_deriv(const GrayImg &s) {
  std::vector<int16_t> d((size_t)s.w * s.h * 2);
  cv_parallel_for((size_t)s.h, [&](size_t ya, size_t yb) {
    for (int y = (int)ya; y < (int)yb; y++) {
      int y0 = reflect101(y - 1, s.h), y2 = reflect101(y + 1, s.h);
      auto t0 = [&](int x) { return (s.at(x, y0) + s.at(x, y2)) * 3 + s.at(x, y) * 10; };
      auto t1 = [&](int x) { return s.at(x, y2) - s.at(x, y0); };
      for (int x = 0; x < s.w; x++) {
        int xm = reflect101(x - 1, s.w), xp = reflect101(x + 1, s.w);
        d[((size_t)y * s.w + x) * 2] = (int16_t)(t0(xp) - t0(xm));
        d[((size_t)y * s.w + x) * 2 + 1] = (int16_t)((t1(xp) + t1(xm)) * 3 + t1(x) * 10);
      }
    }
  });
  return d;
}

Pyramid build_pyramid(const GrayImg &img, int win, int max_level) {
  Pyramid p;
  GrayImg cur = img;
  int w = img.w, h = img.h;
  for (int level = 0; level <= max_level; level++) {
    if (level != 0) cur = pyr_down(cur);
    p.img.push_back(cur);
    p.deriv.push_back(scharr_deriv(cur));
    w = (w + 1) / 2;
    h = (h + 1) / 2;
    if (w <= win || h <= win) break;
  }
  return p;
}

// ---- FAST-9 (fast.cpp FAST_t<16> + cornerScore<16>) ----
static const int kFastOff[16][2] = {{0, 3},  {1, 3},  {2, 2},  {3, 1},  {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

static int fast_score(const GrayImg &img, int x, int y, int threshold) {
  int v = img.at(x, y);
  int d[25];
  for (int k = 0; k < 25; k++) {
    int kk = k % 16;
    d[k] = v - img.at(x + kFastOff[kk][0], y + kFastOff[kk][1]);
  }
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = std::min(d[k + 1], d[k + 2]);
    a = std::min(a, d[k + 3]);
    if (a <= a0) continue;
    a = std::min(a, d[k + 4]);
    a = std::min(a, d[k + 5]);
    a = std::min(a, d[k + 6]);
    a = std::min(a, d[k + 7]);
    a = std::min(a, d[k + 8]);
    a0 = std::max(a0, std::min(a, d[k]));
    a0 = std::max(a0, std::min(a, d[k + 9]));
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = std::max(d[k + 1], d[k + 2]);
    b = std::max(b, d[k + 3]);
    b = std::max(b, d[k + 4]);
    b = std::max(b, d[k + 5]);
    if (b >= b0) continue;
    b = std::max(b, d[k + 6]);
    b = std::max(b, d[k + 7]);
    b = std::max(b, d[k + 8]);
    b0 = std::min(b0, std::max(b, d[k]));
    b0 = std::min(b0, std::max(b, d[k + 9]));
  }
  return -b0 - 1;
}

static bool fast_is_corner(const GrayImg &img, int x, int y, int threshold) {
  int v = img.at(x, y);
  for (int pass = 0; pass < 2; pass++) {
    int count = 0;
    for (int k = 0; k < 25; k++) {
      int kk = k % 16;
      int p = img.at(x + kFastOff[kk][0], y + kFastOff[kk][1]);
      bool ok = (pass == 0) ? (p < v - threshold) : (p > v + threshold);
      if (ok) {
        if (++count > 8) return true;
      } else {
        count = 0;
      }
    }
  }
  return false;
}

std::vector<KeyPt> fast_roi(const GrayImg &img, int x0, int y0, int w, int h, int thr) {
  std::vector<int> score((size_t)w * h, 0);
  for (int i = 3; i < h - 3; i++)
    for (int j = 3; j < w - 3; j++)
      if (fast_is_corner(img, x0 + j, y0 + i, thr)) score[(size_t)i * w + j] = fast_score(img, x0 + j, y0 + i, thr);
  std::vector<KeyPt> kp;
  for (int i = 3; i < h - 3; i++)
    for (int j = 3; j < w - 3; j++) {
      int s = score[(size_t)i * w + j];
      if (s == 0) continue;
      bool keep = true;
      for (int di = -1; di <= 1 && keep; di++)
        for (int dj = -1; dj <= 1; dj++) {
          if (!di && !dj) continue;
          if (s <= score[(size_t)(i + di) * w + j + dj]) {
            keep = false;
            break;
          }
        }
      if (keep) kp.push_back(KeyPt{(float)j, (float)i, (float)s});
    }
  return kp;
}

// ---- Grider_GRID.h:128: std::sort(pts_new, Grider_FAST::compare_response) ----
// libstdc++'s own std::sort on the cv::FAST sequence (raster order): the permutation of equal responses is
// the reference's (see tracker.h).
void grid_sort(std::vector<KeyPt> &kp) {
  std::sort(kp.begin(), kp.end(), [](const KeyPt &a, const KeyPt &b) { return a.response > b.response; });
}

// ---- cornerSubPix (cornersubpix.cpp) over getRectSubPix (u8 -> float, replicated border) ----
static void rect_subpix(const GrayImg &img, int ww, int hh, float cx, float cy, float *dst) {
  cx -= (ww - 1) * 0.5f;
  cy -= (hh - 1) * 0.5f;
  int ix = (int)std::floor(cx), iy = (int)std::floor(cy);
  float a = cx - ix, b = cy - iy;
  float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
  auto px = [&](int x, int y) {
    x = std::min(std::max(x, 0), img.w - 1);
    y = std::min(std::max(y, 0), img.h - 1);
    return (float)img.at(x, y);
  };
  for (int i = 0; i < hh; i++)
    for (int j = 0; j < ww; j++) {
      int x = ix + j, y = iy + i;
      dst[i * ww + j] = px(x, y) * a11 + px(x + 1, y) * a12 + px(x, y + 1) * a21 + px(x + 1, y + 1) * a22;
    }
}

void corner_subpix(const GrayImg &img, std::vector<KeyPt> &pts, int win, int max_iters, double eps) {
  const int win_w = 2 * win + 1, win_h = 2 * win + 1;
  std::vector<float> mask((size_t)win_w * win_h), buf((size_t)(win_w + 2) * (win_h + 2));
  for (int i = 0; i < win_h; i++) {
    float y = (float)(i - win) / win;
    float vy = std::exp(-y * y);
    for (int j = 0; j < win_w; j++) {
      float x = (float)(j - win) / win;
      mask[(size_t)i * win_w + j] = (float)(vy * std::exp(-x * x));
    }
  }
  eps *= eps;
  for (auto &p : pts) {
    float cTx = p.x, cTy = p.y, cIx = cTx, cIy = cTy;
    int iter = 0;
    double err = 0;
    do {
      double a = 0, b = 0, c = 0, bb1 = 0, bb2 = 0;
      rect_subpix(img, win_w + 2, win_h + 2, cIx, cIy, buf.data());
      const float *sp = buf.data() + (win_w + 2) + 1;
      for (int i = 0, k = 0; i < win_h; i++, sp += win_w + 2) {
        double py = i - win;
        for (int j = 0; j < win_w; j++, k++) {
          double m = mask[k];
          double tgx = sp[j + 1] - sp[j - 1];
          double tgy = sp[j + win_w + 2] - sp[j - win_w - 2];
          double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
          double pxv = j - win;
          a += gxx;
          b += gxy;
          c += gyy;
          bb1 += gxx * pxv + gxy * py;
          bb2 += gxy * pxv + gyy * py;
        }
      }
      double det = a * c - b * b;
      if (std::fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
      double scale = 1.0 / det;
      float nx = (float)(cIx + c * scale * bb1 - b * scale * bb2);
      float ny = (float)(cIy - b * scale * bb1 + a * scale * bb2);
      err = (double)(nx - cIx) * (nx - cIx) + (double)(ny - cIy) * (ny - cIy);
      cIx = nx;
      cIy = ny;
      if (cIx < 0 || cIx >= img.w || cIy < 0 || cIy >= img.h) break;
    } while (++iter < max_iters && err > eps);
    if (std::fabs(cIx - cTx) > win || std::fabs(cIy - cTy) > win) {
      cIx = cTx;
      cIy = cTy;
    }
    p.x = cIx;
    p.y = cIy;
  }
}

// ---- pyramidal LK (lkpyramid.cpp LKTrackerInvoker) ----
static inline int img_px(const GrayImg &g, int x, int y) {  // BORDER_REFLECT_101 pad
  return g.at(reflect101(x, g.w), reflect101(y, g.h));
}
static inline int der_px(const std::vector<int16_t> &d, const GrayImg &g, int x, int y, int c) {  // BORDER_CONSTANT 0
  if (x < 0 || y < 0 || x >= g.w || y >= g.h) return 0;
  return d[((size_t)y * g.w + x) * 2 + c];
}
static inline int descale(int64_t x, int n) { return (int)((x + ((int64_t)1 << (n - 1))) >> n); }

void lk_track(const Pyramid &prev, const Pyramid &next, const std::vector<KeyPt> &p0, std::vector<KeyPt> &p1,
              std::vector<uint8_t> &status, int win, int max_level, int max_iters, float eps) {
  int maxL = std::min(max_level, std::min(prev.levels(), next.levels()) - 1);
  size_t n = p0.size();
  status.assign(n, 1);
  const float halfw = (win - 1) * 0.5f;
  const int W_BITS = 14;
  const float FLT_SCALE = 1.f / (1 << 20);
  const float crit_eps = eps * eps;
  for (int level = maxL; level >= 0; level--) {
    const GrayImg &I = prev.img[level], &J = next.img[level];
    const auto &dI = prev.deriv[level];
    // calcOpticalFlowPyrLK: parallel_for_ over the points of each level (lkpyramid.cpp LKTrackerInvoker)
    cv_parallel_for(n, [&](size_t plo, size_t phi) {
    std::vector<int> Iw((size_t)win * win), dIx((size_t)win * win), dIy((size_t)win * win);
    for (size_t pi = plo; pi < phi; pi++) {
      float sc = (float)(1. / (1 << level));
      float prx = p0[pi].x * sc, pry = p0[pi].y * sc;
      float nx, ny;
      if (level == maxL) {
        nx = p1[pi].x * sc;
        ny = p1[pi].y * sc;
      } else {
        nx = p1[pi].x * 2.f;
        ny = p1[pi].y * 2.f;
      }
      p1[pi].x = nx;
      p1[pi].y = ny;
      prx -= halfw;
      pry -= halfw;
      int ipx = (int)std::floor(prx), ipy = (int)std::floor(pry);
      if (ipx < -win || ipx >= I.w || ipy < -win || ipy >= I.h) {
        if (level == 0) status[pi] = 0;
        continue;
      }
      float a = prx - ipx, b = pry - ipy;
      int iw00 = (int)std::nearbyint((1.f - a) * (1.f - b) * (1 << W_BITS));
      int iw01 = (int)std::nearbyint(a * (1.f - b) * (1 << W_BITS));
      int iw10 = (int)std::nearbyint((1.f - a) * b * (1 << W_BITS));
      int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
      int64_t iA11 = 0, iA12 = 0, iA22 = 0;
      for (int y = 0; y < win; y++)
        for (int x = 0; x < win; x++) {
          int X = ipx + x, Y = ipy + y;
          int ival = descale((int64_t)img_px(I, X, Y) * iw00 + img_px(I, X + 1, Y) * iw01 + img_px(I, X, Y + 1) * iw10 +
                                 img_px(I, X + 1, Y + 1) * iw11,
                             W_BITS - 5);
          int ixv = descale((int64_t)der_px(dI, I, X, Y, 0) * iw00 + der_px(dI, I, X + 1, Y, 0) * iw01 +
                                der_px(dI, I, X, Y + 1, 0) * iw10 + der_px(dI, I, X + 1, Y + 1, 0) * iw11,
                            W_BITS);
          int iyv = descale((int64_t)der_px(dI, I, X, Y, 1) * iw00 + der_px(dI, I, X + 1, Y, 1) * iw01 +
                                der_px(dI, I, X, Y + 1, 1) * iw10 + der_px(dI, I, X + 1, Y + 1, 1) * iw11,
                            W_BITS);
          Iw[y * win + x] = (int16_t)ival;
          dIx[y * win + x] = (int16_t)ixv;
          dIy[y * win + x] = (int16_t)iyv;
          iA11 += (int64_t)ixv * ixv;
          iA12 += (int64_t)ixv * iyv;
          iA22 += (int64_t)iyv * iyv;
        }
      float A11 = (float)iA11 * FLT_SCALE, A12 = (float)iA12 * FLT_SCALE, A22 = (float)iA22 * FLT_SCALE;
      float D = A11 * A22 - A12 * A12;
      float minEig = (A22 + A11 - std::sqrt((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (2 * win * win);
      if (minEig < 1e-4f || D < FLT_EPSILON) {
        if (level == 0) status[pi] = 0;
        continue;
      }
      D = 1.f / D;
      nx -= halfw;
      ny -= halfw;
      float pdx = 0.f, pdy = 0.f;
      for (int j = 0; j < max_iters; j++) {
        int inx = (int)std::floor(nx), iny = (int)std::floor(ny);
        if (inx < -win || inx >= J.w || iny < -win || iny >= J.h) {
          if (level == 0) status[pi] = 0;
          break;
        }
        a = nx - inx;
        b = ny - iny;
        iw00 = (int)std::nearbyint((1.f - a) * (1.f - b) * (1 << W_BITS));
        iw01 = (int)std::nearbyint(a * (1.f - b) * (1 << W_BITS));
        iw10 = (int)std::nearbyint((1.f - a) * b * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        int64_t ib1 = 0, ib2 = 0;
        for (int y = 0; y < win; y++)
          for (int x = 0; x < win; x++) {
            int X = inx + x, Y = iny + y;
            int diff = descale((int64_t)img_px(J, X, Y) * iw00 + img_px(J, X + 1, Y) * iw01 + img_px(J, X, Y + 1) * iw10 +
                                   img_px(J, X + 1, Y + 1) * iw11,
                               W_BITS - 5) -
                       Iw[y * win + x];
            ib1 += (int64_t)diff * dIx[y * win + x];
            ib2 += (int64_t)diff * dIy[y * win + x];
          }
        float b1 = (float)ib1 * FLT_SCALE, b2 = (float)ib2 * FLT_SCALE;
        float dx = (A12 * b2 - A22 * b1) * D;
        float dy = (A12 * b1 - A11 * b2) * D;
        nx += dx;
        ny += dy;
        p1[pi].x = nx + halfw;
        p1[pi].y = ny + halfw;
        if ((double)dx * dx + (double)dy * dy <= crit_eps) break;
        if (j > 0 && std::fabs(dx + pdx) < 0.01f && std::fabs(dy + pdy) < 0.01f) {
          p1[pi].x -= dx * 0.5f;
          p1[pi].y -= dy * 0.5f;
          break;
        }
        pdx = dx;
        pdy = dy;
      }
    }
    });
  }
}

// ---- RANSAC fundamental (fundam.cpp run7Point / FMEstimatorCallback, ptsetreg.cpp) ----
struct CvRng {  // cv::RNG (multiply-with-carry, CV_RNG_COEFF 4164903690)
  uint64_t state;
  explicit CvRng(uint64_t s) : state(s ? s : (uint64_t)(int64_t)-1) {}
  unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
    return (unsigned)state;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

void ransac_subsets(int count, int max_iters, std::vector<int> &idx) {
  CvRng rng((uint64_t)(int64_t)-1);
  idx.assign((size_t)max_iters * 7, 0);
  for (int it = 0; it < max_iters; it++) {
    int *s = &idx[(size_t)it * 7];
    for (int i = 0; i < 7; i++) {
      for (;;) {
        int v = rng.uniform(0, count);
        int j;
        for (j = 0; j < i; j++)
          if (s[j] == v) break;
        if (j == i) {
          s[i] = v;
          break;
        }
      }
    }
  }
}

// cv::solveCubic (coeffs c[0] x^3 + c[1] x^2 + c[2] x + c[3])
static int solve_cubic(const double *co, double *x) {
  double a = co[0], b = co[1], c = co[2], d = co[3];
  if (a == 0) {
    if (b == 0) {
      if (c == 0) return d == 0 ? -1 : 0;
      x[0] = -d / c;
      return 1;
    }
    double D = c * c - 4 * b * d;
    if (D >= 0) {
      D = std::sqrt(D);
      x[0] = (-c - D) / (2 * b);
      x[1] = (-c + D) / (2 * b);
      return 2;
    }
    return 0;
  }
  a = 1. / a;
  b *= a;
  c *= a;
  d *= a;
  double Q = (b * b - c * 3) * (1. / 9);
  double R = (b * b * b * 2 - b * c * 9 + d * 27) * (1. / 54);
  double Qcubed = Q * Q * Q;
  double dd = Qcubed - R * R;
  if (dd > 0) {
    double theta = std::acos(R / std::sqrt(Qcubed));
    double sqrtQ = std::sqrt(Q);
    double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = b * (1. / 3);
    x[0] = t0 * std::cos(t1) - t2;
    x[1] = t0 * std::cos(t1 + (2. * M_PI / 3)) - t2;
    x[2] = t0 * std::cos(t1 + (4. * M_PI / 3)) - t2;
    return 3;
  } else if (dd == 0) {
    if (R >= 0) {
      x[0] = -2 * std::pow(R, 1. / 3) - a / 3;
      x[1] = std::pow(R, 1. / 3) - a / 3;
    } else {
      x[0] = 2 * std::pow(-R, 1. / 3) - a / 3;
      x[1] = -std::pow(-R, 1. / 3) - a / 3;
    }
    int n = x[0] == x[1] ? 1 : 2;
    return n;
  }
  dd = std::sqrt(-dd);
  double e = std::pow(dd + std::fabs(R), 1. / 3);
  if (R > 0) e = -e;
  x[0] = (e + Q / e) - b * (1. / 3);
  return 1;
}

// null space of the 7x9 epipolar system by Householder QR of A^T (any orthonormal basis of the
// 2-D null space gives the same singular members of the pencil after F(2,2) normalization)
int fundamental_7pt(const double *x0, const double *y0, const double *x1, const double *y1, double *F) {
  double At[9][7];
  for (int i = 0; i < 7; i++) {
    double a[9] = {x1[i] * x0[i], x1[i] * y0[i], x1[i], y1[i] * x0[i], y1[i] * y0[i], y1[i], x0[i], y0[i], 1.0};
    for (int k = 0; k < 9; k++) At[k][i] = a[k];
  }
  // Q = H_0 H_1 ... H_6 (9x9); null space = Q[:, 7], Q[:, 8]
  double Vh[7][9], beta[7];
  for (int c = 0; c < 7; c++) {
    double ss = 0;
    for (int r = c; r < 9; r++) ss += At[r][c] * At[r][c];
    double x0v = At[c][c], alpha = (x0v > 0) ? -std::sqrt(ss) : std::sqrt(ss);
    for (int r = 0; r < 9; r++) Vh[c][r] = (r < c) ? 0.0 : (r == c ? x0v - alpha : At[r][c]);
    double vn = ss - x0v * x0v + (x0v - alpha) * (x0v - alpha);
    beta[c] = vn > 0 ? 2.0 / vn : 0.0;
    for (int j = c; j < 7; j++) {
      double s = 0;
      for (int r = c; r < 9; r++) s += Vh[c][r] * At[r][j];
      s *= beta[c];
      for (int r = c; r < 9; r++) At[r][j] -= s * Vh[c][r];
    }
  }
  double f[2][9];
  for (int q = 0; q < 2; q++) {
    double e[9] = {0};
    e[7 + q] = 1.0;
    for (int c = 6; c >= 0; c--) {  // Q e = H_0 (H_1 (... H_6 e))
      double s = 0;
      for (int r = c; r < 9; r++) s += Vh[c][r] * e[r];
      s *= beta[c];
      for (int r = c; r < 9; r++) e[r] -= s * Vh[c][r];
    }
    for (int k = 0; k < 9; k++) f[q][k] = e[k];
  }
  double *f1 = f[0], *f2 = f[1];
  for (int i = 0; i < 9; i++) f1[i] -= f2[i];
  double t0, t1, t2, c[4], r[3] = {0, 0, 0};
  t0 = f2[4] * f2[8] - f2[5] * f2[7];
  t1 = f2[3] * f2[8] - f2[5] * f2[6];
  t2 = f2[3] * f2[7] - f2[4] * f2[6];
  c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
  c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
         f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
         f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
         f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
  t0 = f1[4] * f1[8] - f1[5] * f1[7];
  t1 = f1[3] * f1[8] - f1[5] * f1[6];
  t2 = f1[3] * f1[7] - f1[4] * f1[6];
  c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
         f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
         f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
         f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
  c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
  int n = solve_cubic(c, r);
  if (n < 1 || n > 3) return 0;
  for (int k = 0; k < n; k++) {
    double lambda = r[k], mu = 1.;
    double s = f1[8] * r[k] + f2[8];
    double *Fm = F + 9 * k;
    if (std::fabs(s) > DBL_EPSILON) {
      mu = 1. / s;
      lambda *= mu;
      Fm[8] = 1.;
    } else {
      Fm[8] = 0.;
    }
    for (int i = 0; i < 8; i++) Fm[i] = f1[i] * lambda + f2[i] * mu;
  }
  return n;
}

static int ransac_update_iters(double p, double ep, int model_points, int max_iters) {
  p = std::max(p, 0.);
  p = std::min(p, 1.);
  ep = std::max(ep, 0.);
  ep = std::min(ep, 1.);
  double num = std::max(1. - p, DBL_MIN);
  double denom = 1. - std::pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = std::log(num);
  denom = std::log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)std::nearbyint(num / denom);
}

void ransac_fundamental_mask(const std::vector<float> &x0, const std::vector<float> &y0, const std::vector<float> &x1,
                             const std::vector<float> &y1, double thr, double conf, int max_iters,
                             std::vector<uint8_t> &mask) {
  int count = (int)x0.size();
  mask.assign(count, 0);
  if (count < 7) return;
  std::vector<int> subs;
  ransac_subsets(count, max_iters, subs);
  std::vector<uint8_t> cur(count);
  float t = (float)(thr * thr);
  int niters = max_iters, best = 0;
  for (int it = 0; it < niters && it < max_iters; it++) {
    double sx0[7], sy0[7], sx1[7], sy1[7];
    for (int i = 0; i < 7; i++) {
      int k = subs[(size_t)it * 7 + i];
      sx0[i] = x0[k];
      sy0[i] = y0[k];
      sx1[i] = x1[k];
      sy1[i] = y1[k];
    }
    double F[27];
    int nm = fundamental_7pt(sx0, sy0, sx1, sy1, F);
    for (int m = 0; m < nm; m++) {
      const double *f = F + 9 * m;
      int good = 0;
      for (int i = 0; i < count; i++) {
        double a = f[0] * x0[i] + f[1] * y0[i] + f[2];
        double b = f[3] * x0[i] + f[4] * y0[i] + f[5];
        double c = f[6] * x0[i] + f[7] * y0[i] + f[8];
        double s2 = 1. / (a * a + b * b);
        double d2 = x1[i] * a + y1[i] * b + c;
        a = f[0] * x1[i] + f[3] * y1[i] + f[6];
        b = f[1] * x1[i] + f[4] * y1[i] + f[7];
        c = f[2] * x1[i] + f[5] * y1[i] + f[8];
        double s1 = 1. / (a * a + b * b);
        double d1 = x0[i] * a + y0[i] * b + c;
        float err = (float)std::max(d1 * d1 * s1, d2 * d2 * s2);
        cur[i] = err <= t;
        good += cur[i];
      }
      if (good > std::max(best, 7 - 1)) {
        mask = cur;
        best = good;
        niters = ransac_update_iters(conf, (double)(count - good) / count, 7, niters);
      }
    }
  }
}

}  // namespace orc
