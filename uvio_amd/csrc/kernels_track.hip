// KLT front-end kernels (TrackKLT.cpp:34-886, Grider_GRID.h:74-180 over the OpenCV primitives they
// call; restated in oracle/src/tracker.cpp).  Byte / integer work throughout
// except cornerSubPix (double) and the LK float tail; every result is bit-identical to the oracle:
//   k_hist_multi + k_pyr_pair  equalizeHist (LDS histogram, LUT per workgroup from the global counts),
//                            pyrDown 5x5 (sum + 128) >> 8 and Scharr dx/dy int16 (calcSharrDeriv), reflect-101,
//                            two pyramid levels per launch
//   k_fast_score/_select     FAST-9 + 3x3 NMS + top-k per grid cell in std::sort's tie order (one workgroup per cell)
//   k_subpix<WIN>            cornerSubPix, one wavefront per point (five raster-order sums, one lane each = oracle
//                            order; window size a template constant)
//   k_lk                     pyramidal LK, one wavefront per point, exact integer window sums
//   k_undistort              cv::undistortPoints restatement (hp_math.h)
//   k_ransac_hyp / _select   7-point RANSAC: all hypotheses in parallel, then the sequential
//                            adaptive-iteration scan of RANSACPointSetRegistrator::run on one lane
#include <cstdlib>
#include <stdexcept>
#include <utility>

#include "kernels.h"

namespace uvhp {

// The dispatcher deals workgroups round robin to the 8 XCDs, each with its own L2: workgroup w of nwg is
// given the index that puts a contiguous range of indices on each XCD (a bijection on [0, nwg))
__device__ __forceinline__ int xcd_contiguous(int w, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = w % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
}

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = (p < 0) ? -p : 2 * n - 2 - p;
  return p;
}

// ---------------------------------------------------------------- fused multi-camera pyramid
// All cameras of a frame in one launch per stage (blockIdx.z = camera), TWO pyramid levels per launch:
//   k_hist_multi              histograms of the input images
//   k_pyr_pair<true>  (l = 0) level 0 = LUT(src) (the LUT from the histogram scan) and level 1
//   k_pyr_pair<false> (l = 2) level 2 = pyrDown(level 1) and level 3; (l = 4) level 4
// A workgroup owns a 64 x 16 tile of level l and the 32 x 8 tile of level l+1 below it.  Level l is built in
// LDS over the tile plus a 4-pixel margin (each cell the value at the reflect-101 coordinate, so the margin
// holds exactly the neighbours calcSharrDeriv and the next pyrDown read); level l's pixels and Scharr
// derivatives are written from LDS four pixels per thread (one 4-byte image store, one 16-byte derivative
// store), then level l+1 (+1 halo, reflect-101 in its own size) is reduced from the same LDS block and
// written with its derivatives.  Level l+1 is never read back for level l+2's margin inside the launch, and
// level l is not re-read from memory for level l+1: 4 launches per frame (with the histogram) instead of 6,
// same bits as one pyrDown + Scharr per level.
constexpr int kPM = 4;  // LDS margin of the level-l window
// tile geometry of one pair launch: the level-l tile PW x PH (PW * PH / 256 pixels per thread), its window with
// the margin, the level-(l+1) tile under it and the level l-1 source of the window's pyrDown taps
template <int PW, int PH>
struct PairTile {
  static constexpr int WW = PW + 2 * kPM, WH = PH + 2 * kPM, QW = PW / 2, QH = PH / 2;
  static constexpr int SW = 2 * WW + 4, SH = 2 * WH + 4, PPT = PW * PH / 256;
};
__device__ __forceinline__ void scharr_at(const uint8_t *t, int ld, int x, int y, int16_t &dx, int16_t &dy) {
  // (x, y): the pixel's cell; the 3x3 neighbourhood is in t
  const uint8_t *rm = t + (y - 1) * ld, *r0 = t + y * ld, *rp = t + (y + 1) * ld;
  const int t0m = (rm[x - 1] + rp[x - 1]) * 3 + r0[x - 1] * 10, t0p = (rm[x + 1] + rp[x + 1]) * 3 + r0[x + 1] * 10;
  const int t1m = rp[x - 1] - rm[x - 1], t1p = rp[x + 1] - rm[x + 1], t1 = rp[x] - rm[x];
  dx = (int16_t)(t0p - t0m);
  dy = (int16_t)((t1p + t1m) * 3 + t1 * 10);
}

// level `l`'s owned pixels (PPT consecutive per thread) and derivatives from the LDS window
template <int PW, int PH>
__device__ __forceinline__ void write_level(const uint8_t *win, int x0, int y0, int w, int h, uint8_t *img,
                                            int16_t *der) {
  using T = PairTile<PW, PH>;
  constexpr int PPT = T::PPT, TPR = PW / PPT;  // pixels per thread, threads per tile row
  const int t = threadIdx.x, ty = t / TPR, tx = (t % TPR) * PPT;
  const int gy = y0 + ty, gx = x0 + tx;
  if (ty >= PH || gy >= h || gx >= w) return;
  const int cy = ty + kPM, cx = tx + kPM;
  uint8_t v[PPT];
  int16_t d[2 * PPT];
#pragma unroll
  for (int k = 0; k < PPT; k++) {
    v[k] = win[cy * T::WW + cx + k];
    scharr_at(win, T::WW, cx + k, cy, d[2 * k], d[2 * k + 1]);
  }
  const size_t o = (size_t)gy * w + gx;
  if constexpr (PPT == 4) {
    if (gx + 3 < w && (w & 3) == 0) {
      *(uchar4 *)(img + o) = make_uchar4(v[0], v[1], v[2], v[3]);
      int4 pk;
      pk.x = (int)(((unsigned)(uint16_t)d[1] << 16) | (uint16_t)d[0]);
      pk.y = (int)(((unsigned)(uint16_t)d[3] << 16) | (uint16_t)d[2]);
      pk.z = (int)(((unsigned)(uint16_t)d[5] << 16) | (uint16_t)d[4]);
      pk.w = (int)(((unsigned)(uint16_t)d[7] << 16) | (uint16_t)d[6]);
      *(int4 *)(der + 2 * o) = pk;
      return;
    }
  }
  for (int k = 0; k < PPT && gx + k < w; k++) {
    img[o + k] = v[k];
    *(int *)(der + 2 * (o + k)) = (int)(((unsigned)(uint16_t)d[2 * k + 1] << 16) | (uint16_t)d[2 * k]);
  }
}

template <bool EQ, int PW, int PH>
__global__ void __launch_bounds__(256) k_pyr_pair(PyrJob job, int l) {
  using T = PairTile<PW, PH>;
  __shared__ uint8_t lut[256];
  __shared__ int scan[256];
  __shared__ int first;
  __shared__ uint8_t win[T::WH * T::WW];
  __shared__ uint8_t q[(T::QH + 2) * (T::QW + 2)];
  __shared__ uint8_t srcs[EQ ? 1 : T::SH * T::SW];
  // tiles of one camera in raster order, a contiguous range of them per XCD (neighbouring tiles share their
  // margin rows / columns through that XCD's L2)
  const int idx = xcd_contiguous(blockIdx.x + blockIdx.z * gridDim.x, gridDim.x * gridDim.z);
  const int c = idx / gridDim.x, tile = idx - c * gridDim.x, t = threadIdx.x;
  // the levels 2-3 launch runs after level 0's has read the histogram: it clears it for the next frame (the
  // tracker zeroes it once at allocation), which saves a fill per camera and frame
  if (!EQ && l == 2 && job.equalize && tile == 0) job.hist[c][t] = 0u;
  const DPyr &p = job.p[c];
  if (l >= p.levels) return;
  const int w = p.w[l], h = p.h[l];
  const int ntx = (w + PW - 1) / PW;
  const int x0 = (tile % ntx) * PW, y0 = (tile / ntx) * PH;
  if (y0 >= h) return;
  if constexpr (EQ) {
    // LUT of EqualizeHistLut_Invoker from an inclusive LDS scan of the counts (blockDim == 256)
    if (!job.equalize) {
      lut[t] = (uint8_t)t;
    } else {
      const unsigned *hist = job.hist[c];
      const int hv = (int)hist[t];
      scan[t] = hv;
      if (t == 0) first = 256;
      __syncthreads();
      if (hv) atomicMin(&first, t);
      for (int o = 1; o < 256; o <<= 1) {
        int v = (t >= o) ? scan[t - o] : 0;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
      }
      const int i0 = first, total = w * h, h0 = (int)hist[i0];
      if (h0 == total) {
        lut[t] = (uint8_t)i0;
      } else if (t <= i0) {
        lut[t] = 0;
      } else {
        float scale = __fdiv_rn(256 - 1.f, (float)(total - h0));
        int sum = scan[t] - scan[i0];
        int r = (int)rintf(__fmul_rn((float)sum, scale));
        lut[t] = (uint8_t)min(255, max(0, r));
      }
    }
    __syncthreads();
  }
  // level l over the window (reflect-101 coordinates)
  const uint8_t *src = EQ ? job.src[c] : p.img[l - 1];
  const int sld = EQ ? job.stride[c] : p.w[l - 1];
  // All of a thread's source bytes are loaded before any is used (a load consumed in the same loop iteration
  // made one memory round trip per iteration); a window inside the image takes plain loads, one touching an
  // edge the reflect-101 coordinates.
  if constexpr (EQ) {
    constexpr int NW = T::WH * T::WW, NWP = (NW + 255) / 256;
    uint8_t v[NWP];
    const int bx = x0 - kPM, by = y0 - kPM;
    if (bx >= 0 && bx + T::WW <= w && by >= 0 && by + T::WH <= h) {
#pragma unroll
      for (int k = 0; k < NWP; k++) {
        const int e = min(t + 256 * k, NW - 1), wy = e / T::WW, wx = e - wy * T::WW;
        v[k] = src[(size_t)(by + wy) * sld + bx + wx];
      }
    } else {
#pragma unroll
      for (int k = 0; k < NWP; k++) {
        const int e = min(t + 256 * k, NW - 1), wy = e / T::WW, wx = e - wy * T::WW;
        v[k] = src[(size_t)reflect101(by + wy, h) * sld + reflect101(bx + wx, w)];
      }
    }
#pragma unroll
    for (int k = 0; k < NWP; k++)
      if (t + 256 * k < NW) win[t + 256 * k] = lut[v[k]];
  } else {
    // level l-1 over every pyrDown tap of the window, at virtual coordinates (each cell the value at its
    // reflect-101 coordinate in level l-1).  Every window cell that is read later (rows / columns up to one
    // past the level's edge: reflected by at most 3) has its taps inside this block; the deeper-reflected
    // margin cells nothing reads are clamped into it
    const int sw = p.w[l - 1], sh = p.h[l - 1], sx0 = 2 * (x0 - kPM) - 2, sy0 = 2 * (y0 - kPM) - 2;
    constexpr int NS = T::SH * T::SW, NSP = (NS + 255) / 256;
    uint8_t v[NSP];
    if (sx0 >= 0 && sx0 + T::SW <= sw && sy0 >= 0 && sy0 + T::SH <= sh) {
#pragma unroll
      for (int k = 0; k < NSP; k++) {
        const int e = min(t + 256 * k, NS - 1), sy = e / T::SW, sx = e - sy * T::SW;
        v[k] = src[(size_t)(sy0 + sy) * sld + sx0 + sx];
      }
    } else {
#pragma unroll
      for (int k = 0; k < NSP; k++) {
        const int e = min(t + 256 * k, NS - 1), sy = e / T::SW, sx = e - sy * T::SW;
        v[k] = src[(size_t)reflect101(sy0 + sy, sh) * sld + reflect101(sx0 + sx, sw)];
      }
    }
#pragma unroll
    for (int k = 0; k < NSP; k++)
      if (t + 256 * k < NS) srcs[t + 256 * k] = v[k];
    __syncthreads();
    const int k5[5] = {1, 4, 6, 4, 1};
    for (int e = t; e < T::WH * T::WW; e += 256) {
      const int wy = e / T::WW, wx = e - wy * T::WW;
      const int gx = reflect101(x0 + wx - kPM, w), gy = reflect101(y0 + wy - kPM, h);
      const int ry = min(max(2 * gy - 2 - sy0, 0), T::SH - 5), rx = min(max(2 * gx - 2 - sx0, 0), T::SW - 5);
      int acc = 0;
#pragma unroll
      for (int i = 0; i < 5; i++) {
        const uint8_t *row = srcs + (ry + i) * T::SW + rx;
        int r = 0;
#pragma unroll
        for (int j = 0; j < 5; j++) r += k5[j] * row[j];
        acc += k5[i] * r;
      }
      win[e] = (uint8_t)((acc + 128) >> 8);
    }
  }
  __syncthreads();
  write_level<PW, PH>(win, x0, y0, w, h, (uint8_t *)p.img[l], (int16_t *)p.der[l]);
  if (l + 1 >= p.levels) return;
  // level l+1: the 32 x 8 tile + 1 halo, each cell pyrDown of the window at its reflect-101 coordinate
  const int dw = p.w[l + 1], dh = p.h[l + 1], qx0 = x0 / 2, qy0 = y0 / 2;
  if (qy0 >= dh || qx0 >= dw) return;
  const int k5[5] = {1, 4, 6, 4, 1};
  for (int e = t; e < (T::QH + 2) * (T::QW + 2); e += 256) {
    const int ty = e / (T::QW + 2), tx = e - ty * (T::QW + 2);
    const int x = reflect101(qx0 + tx - 1, dw), y = reflect101(qy0 + ty - 1, dh);
    int acc = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      // level-l row 2y + i - 2 (the window cell holds its reflect-101 value)
      const uint8_t *row = win + (2 * y + i - 2 - (y0 - kPM)) * T::WW - (x0 - kPM);
      int r = 0;
#pragma unroll
      for (int j = 0; j < 5; j++) r += k5[j] * row[2 * x + j - 2];
      acc += k5[i] * r;
    }
    q[e] = (uint8_t)((acc + 128) >> 8);
  }
  __syncthreads();
  const int tx = t % T::QW, ty = t / T::QW, gx = qx0 + tx, gy = qy0 + ty;
  if (ty < T::QH && gx < dw && gy < dh) {
    const size_t o = (size_t)gy * dw + gx;
    ((uint8_t *)p.img[l + 1])[o] = q[(ty + 1) * (T::QW + 2) + tx + 1];
    int16_t dx, dy;
    scharr_at(q, T::QW + 2, tx + 1, ty + 1, dx, dy);
    *(int *)((int16_t *)p.der[l + 1] + 2 * o) = (int)(((unsigned)(uint16_t)dy << 16) | (uint16_t)dx);
  }
}

// Histogram of each camera's input: a packed, 16-byte aligned image is read 16 pixels per load (one load per
// thread at 752 x 480 with the launch below); otherwise eight byte loads are issued before their counts.
__global__ void __launch_bounds__(256) k_hist_multi(PyrJob job) {
  __shared__ unsigned hs[256];
  const int c = blockIdx.z;
  const DPyr &p = job.p[c];
  const int w = p.w[0], h = p.h[0], stride = job.stride[c], n = w * h;
  const uint8_t *img = job.src[c];
  hs[threadIdx.x] = 0;
  __syncthreads();
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  if (stride == w && (reinterpret_cast<uintptr_t>(img) & 15) == 0) {
    for (int e = 16 * tid; e < n; e += 16 * nth) {
      if (e + 16 <= n) {
        const uint4 q = *reinterpret_cast<const uint4 *>(img + e);
        const unsigned wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 16; k++) atomicAdd(&hs[(wd[k >> 2] >> (8 * (k & 3))) & 0xff], 1u);
      } else {
        for (int k = e; k < n; k++) atomicAdd(&hs[img[k]], 1u);
      }
    }
  } else {
    for (int e0 = tid; e0 < n; e0 += 8 * nth) {
      int v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int e = min(e0 + k * nth, n - 1), y = e / w, x = e - y * w;
        v[k] = img[(size_t)y * stride + x];
      }
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (e0 + k * nth < n) atomicAdd(&hs[v[k]], 1u);
    }
  }
  __syncthreads();
  if (hs[threadIdx.x]) atomicAdd(&job.hist[c][threadIdx.x], hs[threadIdx.x]);
}

void launch_pyramids(hipStream_t s, const PyrJob &job) {
  if (job.ncam <= 0) return;
  int maxl = 0;
  for (int c = 0; c < job.ncam; c++) maxl = max(maxl, job.p[c].levels);
  auto tiles = [&](int l) {
    int wl = 0, hl = 0;
    for (int c = 0; c < job.ncam; c++)
      if (l < job.p[c].levels) {
        wl = max(wl, job.p[c].w[l]);
        hl = max(hl, job.p[c].h[l]);
      }
    return std::make_pair(wl, hl);
  };
  auto grid = [&](int l, int pw, int ph) {
    auto [wl, hl] = tiles(l);
    return ((wl + pw - 1) / pw) * ((hl + ph - 1) / ph);
  };
  if (job.equalize) {
    int w0 = 0, h0 = 0;
    for (int c = 0; c < job.ncam; c++) w0 = max(w0, job.p[c].w[0]), h0 = max(h0, job.p[c].h[0]);
    // the histograms are zero here: cleared by the previous frame's levels 2-3 launch (below), or at allocation
    if (maxl <= 2)
      for (int c = 0; c < job.ncam; c++)
        if (hipMemsetAsync(job.hist[c], 0, 256 * sizeof(unsigned), s) != hipSuccess) throw std::runtime_error("hipMemsetAsync");
    hipLaunchKernelGGL(k_hist_multi, dim3(min(256, (w0 * h0 + 4095) / 4096), 1, job.ncam), dim3(256), 0, s, job);
  }
  // level 0 (the big image): 64 x 16 tiles, four pixels per thread; levels >= 2 (<= 188 x 120 at 752 x 480):
  // 32 x 8 tiles, so each workgroup's serial staging and reduction stay short
  hipLaunchKernelGGL((k_pyr_pair<true, 64, 16>), dim3(grid(0, 64, 16), 1, job.ncam), dim3(256), 0, s, job, 0);
  for (int l = 2; l < maxl; l += 2)
    hipLaunchKernelGGL((k_pyr_pair<false, 32, 8>), dim3(grid(l, 32, 8), 1, job.ncam), dim3(256), 0, s, job, l);
}

double pyramid_bytes(const PyrJob &job) {
  // histogram pass reads the input; every pair launch reads its source (the input, or level l-1) once and
  // writes its two levels' images and derivatives
  double b = 0.0;
  for (int c = 0; c < job.ncam; c++) {
    const DPyr &p = job.p[c];
    const double a0 = (double)p.w[0] * p.h[0];
    b += (job.equalize ? a0 : 0.0) + a0;
    for (int l = 0; l < p.levels; l++) b += 5.0 * p.w[l] * p.h[l];
    for (int l = 2; l < p.levels; l += 2) b += (double)p.w[l - 1] * p.h[l - 1];
  }
  return b;
}

// downsample_cameras: cv::pyrDown of the raw 2w x 2h camera image before tracking (VioManager.cpp:270-278),
// the same 5x5 binomial and rounding as the pyramid levels; one output pixel per thread, 64 x 4 blocks
// (coalesced rows), blockIdx.z = camera
__global__ void __launch_bounds__(256) k_decimate_multi(DecimateJob job) {
  const int c = blockIdx.z;
  const int dw = job.w[c], dh = job.h[c], sw = 2 * dw, sh = 2 * dh, ld = job.stride[c];
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= dw || y >= dh) return;
  const uint8_t *src = job.src[c];
  const int k5[5] = {1, 4, 6, 4, 1};
  int xs[5];
#pragma unroll
  for (int j = 0; j < 5; j++) xs[j] = reflect101(2 * x + j - 2, sw);
  int acc = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint8_t *row = src + (size_t)reflect101(2 * y + i - 2, sh) * ld;
    int r = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) r += k5[j] * row[xs[j]];
    acc += k5[i] * r;
  }
  job.dst[c][(size_t)y * dw + x] = (uint8_t)((acc + 128) >> 8);
}

void launch_decimate(hipStream_t s, const DecimateJob &job) {
  if (job.ncam <= 0) return;
  int w = 0, h = 0;
  for (int c = 0; c < job.ncam; c++) w = max(w, job.w[c]), h = max(h, job.h[c]);
  hipLaunchKernelGGL(k_decimate_multi, dim3((w + 63) / 64, (h + 3) / 4, job.ncam), dim3(256), 0, s, job);
}

// ---------------------------------------------------------------- FAST-9 on grid cells
// ring offsets (dx, dy) of cv::makeOffsets(pattern 16)
__constant__ int c_fast_off[16][2] = {{0, 3},  {1, 3},  {2, 2},  {3, 1},  {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                      {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// true iff the 16-bit circular mask holds a run of >= 9 set bits (FAST_t's consecutive count over the
// 25-long ring walk): bit i of r is set iff bits i..i+8 of the doubled mask all are
__device__ __forceinline__ bool has_arc9(unsigned m) {
  m |= m << 16;
  unsigned r = m & (m >> 1);
  r &= r >> 2;  // 4 consecutive
  r &= r >> 4;  // 8 consecutive
  r &= m >> 8;  // 9 consecutive
  return (r & 0xFFFFu) != 0;
}

// FAST-9 test + cornerScore<16> of a pixel from its value v and Bresenham ring; 0 = not a corner
__device__ __forceinline__ void fast_ring(const uint8_t *p, int ld, int &v, int (&ring)[16]) {
  v = p[0];
#pragma unroll
  for (int k = 0; k < 16; k++) ring[k] = p[c_fast_off[k][1] * ld + c_fast_off[k][0]];
}
__device__ int fast_corner_score(const int v, const int (&ring)[16], int thr) {
  unsigned dk = 0, br = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    dk |= (unsigned)(ring[k] < v - thr) << k;
    br |= (unsigned)(ring[k] > v + thr) << k;
  }
  if (!has_arc9(dk) && !has_arc9(br)) return 0;
  int d[25];
#pragma unroll
  for (int k = 0; k < 25; k++) d[k] = v - ring[k & 15];
  int a0 = thr;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int a = min(d[k + 1], d[k + 2]);
    a = min(a, d[k + 3]);
    if (a <= a0) continue;
    a = min(a, d[k + 4]);
    a = min(a, d[k + 5]);
    a = min(a, d[k + 6]);
    a = min(a, d[k + 7]);
    a = min(a, d[k + 8]);
    a0 = max(a0, min(a, d[k]));
    a0 = max(a0, min(a, d[k + 9]));
  }
  int b0 = -a0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int b = max(d[k + 1], d[k + 2]);
    b = max(b, d[k + 3]);
    b = max(b, d[k + 4]);
    b = max(b, d[k + 5]);
    if (b >= b0) continue;
    b = max(b, d[k + 6]);
    b = max(b, d[k + 7]);
    b = max(b, d[k + 8]);
    b0 = min(b0, max(b, d[k]));
    b0 = min(b0, max(b, d[k + 9]));
  }
  return -b0 - 1;
}

// Phase 1: scores of every interior pixel of every cell (cv::FAST on the cell ROI: ring reads of an
// interior pixel stay inside the cell) into an image-sized u8 map.  Grid (cell, band of kFastBand rows)
// so a few cells still spread over many CUs.
constexpr int kFastBand = 8;
__device__ __forceinline__ int fast_cam(const FastJob &job, int c) {
  int k = 0;
  while (k < job.ncam - 1 && c >= job.cell_end[k]) k++;
  return k;
}
__global__ void __launch_bounds__(256) k_fast_score(FastJob job, const int *__restrict__ cells, int thr) {
  const int c = blockIdx.x, i0 = blockIdx.y * kFastBand;
  const int k = fast_cam(job, c);
  const uint8_t *__restrict__ img = job.img[k];
  uint8_t *__restrict__ score = job.score[k];
  const int w = job.w[k], sw = job.sw[k], sh = job.sh[k];
  const int x0 = cells[2 * c], y0 = cells[2 * c + 1];
  const int rows = min(kFastBand, sh - i0), np = rows * sw;
  // two pixels per thread and round: both rings' loads are in flight before either is scored
  for (int e0 = threadIdx.x; e0 < np; e0 += 2 * blockDim.x) {
    int v[2], ring[2][16], ii[2], jj[2];
    bool in[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int e = min(e0 + u * (int)blockDim.x, np - 1);
      ii[u] = i0 + e / sw;
      jj[u] = e % sw;
      in[u] = ii[u] >= 3 && ii[u] < sh - 3 && jj[u] >= 3 && jj[u] < sw - 3;
      // a pixel of the cell's 3-pixel border reads its own (interior-clamped) ring and is not scored
      const int ci = min(max(ii[u], 3), sh - 4), cj = min(max(jj[u], 3), sw - 4);
      if (sh >= 7 && sw >= 7) fast_ring(img + (size_t)(y0 + ci) * w + x0 + cj, w, v[u], ring[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; u++)
      if (e0 + u * (int)blockDim.x < np)
        score[(size_t)(y0 + ii[u]) * w + x0 + jj[u]] = (uint8_t)(in[u] ? fast_corner_score(v[u], ring[u], thr) : 0);
  }
}

// ---- Grider_GRID.h:128 std::sort(pts_new, Grider_FAST::compare_response), emulated ----
// A cell's cv::FAST keypoints come in raster order (fast.cpp pushes row by row, x ascending) and are sorted by
// response only, with libstdc++'s introsort (stl_algo.h: __introsort_loop with _S_threshold 16,
// __unguarded_partition_pivot's median of three moved to the front, recursion on the right part, heap sort
// (__partial_sort) once 2 lg n levels are used up, then __final_insertion_sort).  std::sort is not stable: its
// tie order is observable in which corners a cell keeps and in the order they get ids (TrackKLT.cpp:483-520).
// The final insertion sort moves an element only past strictly smaller responses, so the sorted order is the
// STABLE order of the arrangement the introsort loop leaves; the device reproduces that arrangement and then
// selects by (response desc, arrangement position asc).  Candidates are packed as raster index | response << 16.
__device__ __forceinline__ int cand_resp(int v) { return v >> 16; }
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// std::__adjust_heap + std::__push_heap (stl_heap.h) with comp(x, y) = resp(x) > resp(y); one lane.
__device__ void heap_adjust(int *a, int hole, int len, int v) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (cand_resp(a[second]) > cand_resp(a[second - 1])) second--;
    a[hole] = a[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    a[hole] = a[second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && cand_resp(a[parent]) > cand_resp(v)) {
    a[hole] = a[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a[hole] = v;
}
// std::__partial_sort(first, last, last) = __make_heap + __sort_heap: introsort's depth-limit fallback; one lane
// (rare: it needs 2 lg n unbalanced partitions in a row).
__device__ void heap_sort_seg(int *a, int len) {
  if (len >= 2)
    for (int parent = (len - 2) / 2;; parent--) {
      heap_adjust(a, parent, len, a[parent]);
      if (parent == 0) break;
    }
  for (int last = len; last > 1;) {
    --last;
    const int v = a[last];
    a[last] = a[0];
    heap_adjust(a, 0, last, v);
  }
}

// __introsort_loop over arr[0, n) on ONE wavefront (every lane calls it; control is uniform).  One partition
// step __unguarded_partition(first + 1, last, first) is computed in parallel: its left scan stops at the
// positions L_1 < L_2 < ... holding response <= p, its right scan at R_1 > R_2 > ... holding response >= p
// (p the pivot's response).  Before the scans cross they only pass unmodified positions, so the k-th swap
// exchanges L_k and R_k for every k with L_k < R_k (a monotone condition), K swaps in all, and the cut is
// min(L_{K+1}, R_K) (R_K holds L_K's element after the swap, where the left scan stops when no L lies
// between).  The positions come from ballot prefix counts (pl ascending, pr ascending: R_k = pr[cr - k]).
// Segments whose responses are all below t (the cell's k-th largest) are not refined: their order never
// reaches the selection.  depth < 0: 2 lg n, the reference's limit.
__device__ void grid_introsort(int *arr, int n, int t, int depth, unsigned short *pl, unsigned short *pr, int *stk,
                               int lane) {
  if (n <= 16) return;
  if (depth < 0) depth = 2 * (31 - __clz(n));
  const unsigned long long lt = (1ull << lane) - 1ull;
  if (lane == 0) stk[0] = 0, stk[1] = n, stk[2] = depth, stk[3] = 255;
  int sp = 1;
  wave_lds_sync();
  while (sp > 0) {
    sp--;
    int f = uni(stk[4 * sp]), l = uni(stk[4 * sp + 1]), d = uni(stk[4 * sp + 2]);
    const int ub = uni(stk[4 * sp + 3]);
    wave_lds_sync();
    while (l - f > 16 && ub >= t) {
      if (d == 0) {
        if (lane == 0) heap_sort_seg(arr + f, l - f);
        wave_lds_sync();
        break;
      }
      d--;
      // __move_median_to_first(first, first + 1, mid, last - 1)
      const int mid = f + (l - f) / 2;
      const int ra = uni(cand_resp(arr[f + 1])), rb = uni(cand_resp(arr[mid])), rc = uni(cand_resp(arr[l - 1]));
      int m;
      if (ra > rb)
        m = rb > rc ? mid : (ra > rc ? l - 1 : f + 1);
      else if (ra > rc)
        m = f + 1;
      else if (rb > rc)
        m = l - 1;
      else
        m = mid;
      const int vf = uni(arr[f]), vm = uni(arr[m]);
      const int p = cand_resp(vm);
      wave_lds_sync();
      if (lane == 0) arr[f] = vm, arr[m] = vf;
      wave_lds_sync();
      // scan stops of [f + 1, l)
      int cl = 0, cr = 0;
      for (int b = f + 1; b < l; b += 64) {
        const int i = b + lane;
        const int r = i < l ? cand_resp(arr[i]) : 0;
        const bool isl = i < l && r <= p, isr = i < l && r >= p;
        const unsigned long long bl = __ballot(isl), br = __ballot(isr);
        if (isl) pl[cl + __popcll(bl & lt)] = (unsigned short)i;
        if (isr) pr[cr + __popcll(br & lt)] = (unsigned short)i;
        cl += __popcll(bl);
        cr += __popcll(br);
      }
      wave_lds_sync();
      const int mn = min(cl, cr);
      int K = 0;
      for (int k0 = 0; k0 < mn; k0 += 64) {
        const int k = k0 + lane;
        const unsigned long long b = __ballot(k < mn && pl[k] < pr[cr - 1 - k]);
        K += __popcll(b);
        if (b != ~0ull) break;
      }
      const int cut = min(K < cl ? uni(pl[K < cl ? K : 0]) : l, K > 0 ? uni(pr[K > 0 ? cr - K : 0]) : l);
      for (int k0 = 0; k0 < K; k0 += 64) {
        const int k = k0 + lane;
        if (k < K) {
          const int a = pl[k], c = pr[cr - 1 - k];
          const int va = arr[a], vc = arr[c];
          arr[a] = vc;
          arr[c] = va;
        }
      }
      // the right part [cut, l) holds responses <= p; the left part [f, cut) continues here
      if (l - cut > 16 && p >= t) {
        if (lane == 0) stk[4 * sp] = cut, stk[4 * sp + 1] = l, stk[4 * sp + 2] = d, stk[4 * sp + 3] = p;
        sp++;
      }
      wave_lds_sync();
      l = cut;
    }
  }
}

// Phase 2: one workgroup per cell stages the cell's scores in LDS, keeps strict 3x3 maxima, arranges them in
// raster order (cv::FAST's), runs the introsort emulation above and writes the top kmax by (response desc,
// arrangement position asc) -- Grider_GRID.h:128's std::sort order -- as (x, y, response) in image coordinates.
// Strict NMS leaves no two adjacent survivors, so a cell has at most ceil(sw/2) ceil(sh/2) candidates.
constexpr int kFastThreads = 1024, kFastMaxK = 64, kSortStack = 64;
__host__ __device__ inline int fast_max_cand(int sw, int sh) { return ((sw + 1) / 2) * ((sh + 1) / 2); }
__host__ __device__ inline size_t fast_lds_bytes(int sw, int sh) {
  return (size_t)fast_max_cand(sw, sh) * 8 + (((size_t)sw * sh + 15) & ~(size_t)15);
}
__device__ __forceinline__ void fast_select_top(const int *arr, int n, int m, int t, int need, int lane, int wid,
                                                unsigned *sel, int *s_cut, int *s_nsel);
// (the selection tail shared with the probe kernel, below)
__global__ void __launch_bounds__(kFastThreads) k_fast_select(FastJob job, const int *__restrict__ cells, int kmax,
                                                              float *__restrict__ out, int *__restrict__ out_n,
                                                              int *__restrict__ sort_stats) {
  extern __shared__ int lds_fast[];
  const int c = blockIdx.x;
  const int cam = fast_cam(job, c);
  const uint8_t *__restrict__ scmap = job.score[cam];
  const int w = job.w[cam], sw = job.sw[cam], sh = job.sh[cam];
  const int kFastMaxCand = fast_max_cand(sw, sh);
  const int area = sw * sh;
  int *cand = lds_fast, *arr = lds_fast + kFastMaxCand;
  uint8_t *score = (uint8_t *)(arr + kFastMaxCand);
  __shared__ int ncand;
  __shared__ int stk[4 * kSortStack];
  const int x0 = cells[2 * c], y0 = cells[2 * c + 1];
  if (threadIdx.x == 0) ncand = 0;
  // eight loads in flight per thread before their LDS stores (a store right behind its load made one memory
  // round trip per pixel row of the loop)
  for (int e0 = threadIdx.x; e0 < area; e0 += 8 * blockDim.x) {
    uint8_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int e = min(e0 + k * (int)blockDim.x, area - 1), i = e / sw, j = e - i * sw;
      v[k] = scmap[(size_t)(y0 + i) * w + x0 + j];
    }
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (e0 + k * (int)blockDim.x < area) score[e0 + k * blockDim.x] = v[k];
  }
  __syncthreads();
  // survivors are appended with one LDS atomic per wavefront (ballot + prefix popcount): a per-thread
  // atomic on one counter serializes thousands of candidates
  const int lane = threadIdx.x & 63;
  for (int e0 = 0; e0 < area; e0 += blockDim.x) {
    const int e = e0 + threadIdx.x;
    const int sc = (e < area) ? score[e] : 0;
    bool keep = sc != 0;
    if (keep) {
      const int i = e / sw, j = e - i * sw;
      for (int di = -1; di <= 1 && keep; di++)
        for (int dj = -1; dj <= 1; dj++) {
          if (!di && !dj) continue;
          if (sc <= score[(i + di) * sw + j + dj]) {
            keep = false;
            break;
          }
        }
    }
    const unsigned long long bal = __ballot(keep);
    int base = 0;
    if (lane == 0 && bal) base = atomicAdd(&ncand, __popcll(bal));
    base = __shfl(base, 0, 64);
    if (keep) {
      const int slot = base + __popcll(bal & ((1ull << lane) - 1ull));
      if (slot < kFastMaxCand) cand[slot] = e | (sc << 16);
    }
  }
  __syncthreads();
  const int n = min(ncand, kFastMaxCand);
  const int m = min(n, kmax);
  // raster order: a bitmap of the candidates over the cell and its per-word prefix (in the score map's LDS, no
  // longer needed) place candidate e at #{candidates before e}; the response histogram gives the threshold t
  // (the m-th largest response) and above = #{response > t}
  __shared__ int hist[256];
  __shared__ int s_t, s_above, s_cut, s_nsel;
  __shared__ unsigned sel[kFastMaxK];
  const int nwords = (area + 31) >> 5;
  unsigned *bm = reinterpret_cast<unsigned *>(score);
  int *wpre = reinterpret_cast<int *>(bm + nwords);
  for (int a = threadIdx.x; a < 256; a += blockDim.x) hist[a] = 0;
  for (int a = threadIdx.x; a < nwords; a += blockDim.x) bm[a] = 0u;
  if (threadIdx.x == 0) s_cut = -1, s_nsel = 0, s_t = 256, s_above = 0;
  __syncthreads();
  for (int a = threadIdx.x; a < n; a += blockDim.x) {
    const int v = cand[a];
    atomicOr(&bm[(v & 0xFFFF) >> 5], 1u << (v & 31));
    atomicAdd(&hist[cand_resp(v)], 1);
  }
  __syncthreads();
  const int wid = threadIdx.x >> 6;
  if (wid == 0) {
    // exclusive popcount prefix over the bitmap's words: per-lane word ranges, prefix over lanes
    const int per = (nwords + 63) / 64, q0 = lane * per, q1 = min(nwords, q0 + per);
    int cnt = 0;
    for (int q = q0; q < q1; q++) cnt += __popc(bm[q]);
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    int run = incl - cnt;
    for (int q = q0; q < q1; q++) {
      wpre[q] = run;
      run += __popc(bm[q]);
    }
  } else if (wid == 1) {
    // t = the largest response with count(response >= t) >= m; above = count(response > t).  Lane l holds
    // bins 255 - 4l .. 252 - 4l; an inclusive prefix over lanes walks the responses downward.
    int cnt4[4], tot = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      cnt4[q] = hist[255 - 4 * lane - q];
      tot += cnt4[q];
    }
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    int cum = incl - tot;
    if (m > 0 && cum < m && incl >= m) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (cum + cnt4[q] >= m) {
          s_t = 255 - 4 * lane - q;
          s_above = cum;
          break;
        }
        cum += cnt4[q];
      }
    }
  }
  __syncthreads();
  for (int a = threadIdx.x; a < n; a += blockDim.x) {
    const int v = cand[a], e = v & 0xFFFF;
    arr[wpre[e >> 5] + __popc(bm[e >> 5] & ((1u << (e & 31)) - 1u))] = v;
  }
  __syncthreads();
  const int t = s_t, need = m > 0 ? m - s_above : 0;  // tied candidates to take (>= 1 when m > 0)
  if (wid == 0 && m > 0) {
    unsigned short *pl = reinterpret_cast<unsigned short *>(cand), *pr = pl + kFastMaxCand;
    grid_introsort(arr, n, t, -1, pl, pr, stk, lane);
    if (sort_stats && lane == 0 && n > 16) atomicAdd(sort_stats, 1);
  }
  __syncthreads();
  fast_select_top(arr, n, m, t, need, lane, wid, sel, &s_cut, &s_nsel);
  if (wid == 0) {
    // the <= 64 selected keys (255 - response) << 16 | position are sorted across the wavefront's lanes
    unsigned key = lane < min(s_nsel, kFastMaxK) ? sel[lane] : 0xFFFFFFFFu;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const unsigned other = (unsigned)__shfl_xor((int)key, j, 64);
        const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
        key = keep_min ? min(key, other) : max(key, other);
      }
    if (lane < m) {
      const int ia = arr[key & 0xFFFFu] & 0xFFFF;
      float *o = out + ((size_t)c * kmax + lane) * 3;
      o[0] = (float)(x0 + ia % sw);
      o[1] = (float)(y0 + ia / sw);
      o[2] = (float)(255 - (int)(key >> 16));
    }
    if (lane == 0) out_n[c] = m;
  }
}

// Every response above t, and the `need` tied ones at the lowest arrangement positions (found by wave 0 with a
// ballot walk over the arrangement), become keys (255 - response) << 16 | position in sel.  Ends with a barrier.
__device__ __forceinline__ void fast_select_top(const int *arr, int n, int m, int t, int need, int lane, int wid,
                                                unsigned *sel, int *s_cut, int *s_nsel) {
  if (wid == 0 && need > 0) {
    int seen = 0;
    for (int b = 0; b < n; b += 64) {
      const int i = b + lane;
      const unsigned long long bal = __ballot(i < n && cand_resp(arr[i]) == t);
      const int pc = __popcll(bal);
      if (seen + pc >= need) {
        unsigned long long x = bal;
        for (int r = need - seen; r > 1; r--) x &= x - 1ull;
        if (lane == 0) *s_cut = b + __ffsll((long long)x) - 1;
        break;
      }
      seen += pc;
    }
  }
  __syncthreads();
  const int cut = *s_cut;
  for (int a = threadIdx.x; a < n; a += blockDim.x) {
    const int sc = cand_resp(arr[a]);
    if (sc > t || (sc == t && a <= cut)) {
      const int slot = atomicAdd(s_nsel, 1);
      if (slot < kFastMaxK) sel[slot] = ((unsigned)(255 - sc) << 16) | (unsigned)a;
    }
  }
  (void)m;
  __syncthreads();
}

// Test probe of the emulation (uvio_hp_debug_grid_order): one workgroup per cell, the cell's responses in raster
// order; writes the arrangement's raster indices and, for kmax > 0, the cell's top-min(n, kmax) raster indices in
// the selection's order.  depth < 0: the reference's 2 lg n; depth 0 forces the heap-sort fallback.
__global__ void __launch_bounds__(kFastThreads) k_grid_order_probe(const uint8_t *__restrict__ resp,
                                                                   const int *__restrict__ off, int kmax, int depth,
                                                                   int *__restrict__ arrangement,
                                                                   int *__restrict__ top) {
  extern __shared__ int lds_probe[];
  __shared__ int stk[4 * kSortStack];
  __shared__ int hist[256];
  __shared__ int s_t, s_above, s_cut, s_nsel;
  __shared__ unsigned sel[kFastMaxK];
  const int c = blockIdx.x, o0 = off[c], n = off[c + 1] - o0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int *arr = lds_probe;
  unsigned short *pl = reinterpret_cast<unsigned short *>(arr + n), *pr = pl + n;
  const int m = kmax > 0 ? min(n, kmax) : n;
  for (int a = threadIdx.x; a < 256; a += blockDim.x) hist[a] = 0;
  if (threadIdx.x == 0) s_cut = -1, s_nsel = 0, s_t = 256, s_above = 0;
  __syncthreads();
  for (int a = threadIdx.x; a < n; a += blockDim.x) {
    arr[a] = a | ((int)resp[o0 + a] << 16);
    atomicAdd(&hist[resp[o0 + a]], 1);
  }
  __syncthreads();
  if (wid == 0 && m > 0) {
    int cum = 0;
    for (int r = 255; r >= 0; r--) {
      if (cum + hist[r] >= m) {
        s_t = r;
        s_above = cum;
        break;
      }
      cum += hist[r];
    }
  }
  __syncthreads();
  const int t = kmax > 0 ? s_t : -1, need = m > 0 ? m - s_above : 0;
  if (wid == 0 && m > 0) grid_introsort(arr, n, t, depth, pl, pr, stk, lane);
  __syncthreads();
  for (int a = threadIdx.x; a < n; a += blockDim.x) arrangement[o0 + a] = arr[a] & 0xFFFF;
  if (kmax <= 0) return;
  fast_select_top(arr, n, m, s_t, need, lane, wid, sel, &s_cut, &s_nsel);
  if (wid == 0) {
    unsigned key = lane < min(s_nsel, kFastMaxK) ? sel[lane] : 0xFFFFFFFFu;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const unsigned other = (unsigned)__shfl_xor((int)key, j, 64);
        const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
        key = keep_min ? min(key, other) : max(key, other);
      }
    if (lane < m) top[(size_t)c * kmax + lane] = arr[key & 0xFFFFu] & 0xFFFF;
  }
}

// ---------------------------------------------------------------- cornerSubPix
__device__ __forceinline__ float px_clamped(const uint8_t *img, int w, int h, int x, int y) {
  x = min(max(x, 0), w - 1);
  y = min(max(y, 0), h - 1);
  return (float)img[(size_t)y * w + x];
}

// One 64-lane workgroup (one wave) per point.  Lanes build the (win_w + 2)^2 bilinear patch and the
// per-pixel terms in LDS; lanes 0..4 then accumulate the five series, each in the oracle's raster order
// (the double sums are order-sensitive), so the result is bit-identical to the sequential cornerSubPix.
// The window is a template constant: the five raster sums unroll completely, so the LDS reads of each series
// stream ahead of its dependent add chain instead of stalling on every group of eight.  The five sums reach
// every lane by v_readlane and every lane runs the 2x2 solve on the same values: the position stays in
// registers and the iteration needs two barriers, not four.
constexpr int kSubpixMaxWin = 5, kSubpixMargin = 3;
__device__ __forceinline__ double lane_f64(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int WIN>
__global__ void __launch_bounds__(64) k_subpix(SubpixJob job, float *__restrict__ pts, const float *__restrict__ mask,
                                               int max_iters, double eps2) {
  constexpr int WW = 2 * WIN + 1, BW = WW + 2, NT = WW * WW, NTP = NT + (NT & 1);
  constexpr int S = BW + 1 + 2 * kSubpixMargin, NL = (S * S + 63) / 64, NB = (BW * BW + 63) / 64, NK = (NT + 63) / 64;
  __shared__ float tile[S * S];  // clamped image neighbourhood (u8 as float)
  __shared__ float buf[BW * BW];
  __shared__ double tg[5 * NTP];
  const int p = xcd_contiguous(blockIdx.x, gridDim.x), lane = threadIdx.x;  // neighbouring corners on one XCD
  int cam = 0;
  while (cam < job.ncam - 1 && p >= job.end[cam]) cam++;
  if (p >= job.end[cam]) return;
  const uint8_t *__restrict__ img = job.img[cam];
  const int w = job.w[cam], h = job.h[cam];
  const float cTx = pts[2 * p], cTy = pts[2 * p + 1];
  double mk[NK];  // this lane's mask weights, read once
#pragma unroll
  for (int r = 0; r < NK; r++) mk[r] = lane + 64 * r < NT ? (double)mask[lane + 64 * r] : 0.0;
  float cIx = cTx, cIy = cTy;
  int ox = -(1 << 28), oy = -(1 << 28);
  for (int iter = 0; iter < max_iters; iter++) {
    const float cx = cIx - (BW - 1) * 0.5f, cy = cIy - (BW - 1) * 0.5f;
    const int ix = (int)floorf(cx), iy = (int)floorf(cy);
    const float a = cx - ix, b = cy - iy;
    const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
    if (ix - ox < 0 || ix - ox > 2 * kSubpixMargin || iy - oy < 0 || iy - oy > 2 * kSubpixMargin) {
      ox = ix - kSubpixMargin;
      oy = iy - kSubpixMargin;
      float v[NL];  // all of a lane's loads in flight before the LDS stores
#pragma unroll
      for (int k = 0; k < NL; k++) {
        const int e = min(lane + 64 * k, S * S - 1), ty = e / S;
        v[k] = px_clamped(img, w, h, ox + e - ty * S, oy + ty);
      }
#pragma unroll
      for (int k = 0; k < NL; k++)
        if (lane + 64 * k < S * S) tile[lane + 64 * k] = v[k];
      __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < NB; r++) {
      const int e = lane + 64 * r;
      if (e < BW * BW) {
        const int i = e / BW, j = e - i * BW;
        const float *t = tile + (iy - oy + i) * S + (ix - ox + j);
        buf[e] = t[0] * a11 + t[1] * a12 + t[S] * a21 + t[S + 1] * a22;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NK; r++) {
      const int k = lane + 64 * r;
      if (k < NT) {
        const int i = k / WW, j = k - i * WW;
        const float *sp = buf + (i + 1) * BW + 1;
        const double m = mk[r];
        const double tgx = sp[j + 1] - sp[j - 1];
        const double tgy = sp[j + BW] - sp[j - BW];
        const double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
        const double pxv = j - WIN, py = i - WIN;
        tg[k] = gxx;
        tg[NTP + k] = gxy;
        tg[2 * NTP + k] = gyy;
        tg[3 * NTP + k] = gxx * pxv + gxy * py;
        tg[4 * NTP + k] = gxy * pxv + gyy * py;
      }
    }
    __syncthreads();
    double acc = 0;
    if (lane < 5) {  // one series per lane, each in raster order
      // double-buffered chunks of 12: the next chunk's LDS reads are in flight while this one is added (the
      // scheduler would otherwise keep one read ahead of the dependent add chain)
      constexpr int C = 12, NC = (NT + C - 1) / C;
      const double *row = tg + lane * NTP;
      double q[2][C];
#pragma unroll
      for (int i = 0; i < C; i++)
        if (i < NT) q[0][i] = row[i];
#pragma unroll
      for (int c = 0; c < NC; c++) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < C; i++)
          if ((c + 1) * C + i < NT) q[(c + 1) & 1][i] = row[(c + 1) * C + i];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < C; i++)
          if (c * C + i < NT) acc += q[c & 1][i];
      }
    }
    const double sa = lane_f64(acc, 0), sb = lane_f64(acc, 1), sc = lane_f64(acc, 2), bb1 = lane_f64(acc, 3),
                 bb2 = lane_f64(acc, 4);
    const double det = sa * sc - sb * sb;
    if (fabs(det) <= 4.930380657631324e-32) break;  // DBL_EPSILON^2
    const double scale = 1.0 / det;
    const float nx = (float)(cIx + sc * scale * bb1 - sb * scale * bb2);
    const float ny = (float)(cIy - sb * scale * bb1 + sa * scale * bb2);
    const double err = (double)(nx - cIx) * (nx - cIx) + (double)(ny - cIy) * (ny - cIy);
    cIx = nx;
    cIy = ny;
    if (nx < 0 || nx >= w || ny < 0 || ny >= h || !(err > eps2)) break;
    __syncthreads();  // tg and buf are rewritten by the next iteration
  }
  if (lane == 0) {
    if (fabsf(cIx - cTx) > WIN || fabsf(cIy - cTy) > WIN) {
      cIx = cTx;
      cIy = cTy;
    }
    pts[2 * p] = cIx;
    pts[2 * p + 1] = cIy;
  }
}

// ---------------------------------------------------------------- pyramidal LK
// The LK fixed-point products in 32 bits: the reference's CV_DESCALE sums are at most 255 * 2^14 (image) and
// 4080 * 2^14 (Scharr derivative, |d| <= 16 * 255) in magnitude, so int32 holds them exactly.
__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
// a . w over four bilinear taps on the full-rate 24-bit multipliers (v_mad_i32_i24 instead of the quarter-rate
// v_mul_lo_u32): pixels (<= 255), derivatives (|d| <= 4080) and weights (-1 .. 2^14) are far inside the signed
// 24-bit range, and every product and sum stays below 2^31.
__device__ __forceinline__ int dot4_i24(int a0, int a1, int a2, int a3, int w0, int w1, int w2, int w3) {
  return __mul24(a0, w0) + __mul24(a1, w1) + __mul24(a2, w2) + __mul24(a3, w3);
}
// Exact wave sums of the LK window partials through DPP instead of six ds_bpermute rounds.  Per lane at most
// 4 window pixels (win <= 16): |diff * dI| <= 8161 * 4080, so a lane's partial is below 2^27 and a 16-lane row
// sum below 2^31 -- quad_perm xor 1, xor 2, row_half_mirror, row_mirror add in int32 (each lane then holds its
// row's sum), and the four rows are added in int64 from v_readlane.  The whole wave must be active.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
// Wave sums of int32 lane partials whose 16-lane row sums still fit in int32 (the LK bounds below): the row
// stages are 32-bit integer adds, the four row sums are read into scalar registers and added as int64.
template <int N>
__device__ __forceinline__ void wave_sum_rows_i32(const int (&v)[N], long long (&out)[N]) {
  int d[N];
#pragma unroll
  for (int k = 0; k < N; k++) d[k] = v[k];
#pragma unroll
  for (int k = 0; k < N; k++) d[k] += dpp_i32<0xB1>(d[k]);
#pragma unroll
  for (int k = 0; k < N; k++) d[k] += dpp_i32<0x4E>(d[k]);
#pragma unroll
  for (int k = 0; k < N; k++) d[k] += dpp_i32<0x141>(d[k]);
#pragma unroll
  for (int k = 0; k < N; k++) d[k] += dpp_i32<0x140>(d[k]);
#pragma unroll
  for (int k = 0; k < N; k++)
    out[k] = ((long long)__builtin_amdgcn_readlane(d[k], 0) + (long long)__builtin_amdgcn_readlane(d[k], 16)) +
             ((long long)__builtin_amdgcn_readlane(d[k], 32) + (long long)__builtin_amdgcn_readlane(d[k], 48));
}
constexpr int kLkMargin = 4, kLkMaxWin = 16, kLkMaxTile = kLkMaxWin + 1 + 2 * kLkMargin;
static_assert(kLkMaxWin * kLkMaxWin <= 4 * 64, "wave_sum_rows_i32 bound: at most 4 window pixels per lane");
// one 64-lane workgroup per point; lanes own window pixels lane, lane+64, ... (225 for win 15).  (Round 6, measured
// and dropped: the point on four wavefronts, one window pixel per thread and the wave partials summed through LDS
// behind one barrier per sum -- bit-identical, 76.4 against 68 us per launch at cfg3, gpurun_out/r06h.)
// (qx, qy) is nextPts[ptidx] of LKTrackerInvoker: it carries the result between levels, and an
// early exit leaves it at its last written value, exactly as the oracle's p1[pi].
#ifdef UVHP_LK_PROF
// tools/bench_lk.hip: per-point cycle breakdown (level setup, J staging, iterations) of lk_point
struct LkProf {
  unsigned long long setup, stage, iter, total;
  int n_iter, n_stage, n_level, pad;
};
__device__ LkProf g_lk_prof[4096];
#define LKP_T(v) const unsigned long long v = clock64()
#else
#define LKP_T(v)
#endif
__device__ __forceinline__ float2 lk_point(const DPyr &prev, const DPyr &next, const float *__restrict__ p0,
                                         float *__restrict__ p1, uint8_t *__restrict__ status, int pi, int win,
                                         int max_level, int max_iters, float crit_eps, int init_from_p0,
                                         unsigned long long *bytes) {
  const int lane = threadIdx.x;
  const int maxL = min(max_level, min(prev.levels, next.levels) - 1);
  const float halfw = (win - 1) * 0.5f;
  const float FLT_SCALE = 1.f / (1 << 20);
  const float WSCALE = (float)(1 << 14);
  const int area = win * win;
  constexpr int kPer = 4;  // ceil(225 / 64)
  int Iw[kPer], dIx[kPer], dIy[kPer];
  // J neighbourhood of the window staged in LDS (reflect-101 applied while staging); restaged only when
  // an iteration moves the window more than kLkMargin pixels from where it was staged
  __shared__ uint8_t Jt[kLkMaxTile * kLkMaxTile];
  const int S = win + 1 + 2 * kLkMargin;
  // Every gather below is unconditional, so the loads of all of a lane's pixels are in flight together (a
  // per-pixel branch makes one load round per pixel): a lane past the window reads the last pixel's
  // location and carries zero derivatives and template value.  Window pixel (wx, wy) of this lane's slot q
  // and its offset in the staged J tile are the same on every level.
  int wx[kPer], wy[kPer], jo[kPer];
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const int e = min(lane + 64 * q, area - 1);
    wy[q] = e / win;
    wx[q] = e - wy[q] * win;
    jo[q] = wy[q] * S + wx[q];
  }
  constexpr int kStageN = (kLkMaxTile * kLkMaxTile + 63) / 64;
  int sx[kStageN], sy[kStageN];
#pragma unroll
  for (int k = 0; k < kStageN; k++) {
    const int e = min(lane + 64 * k, S * S - 1);
    sy[k] = e / S;
    sx[k] = e - sy[k] * S;
  }
  float qx = init_from_p0 ? p0[2 * pi] : p1[2 * pi], qy = init_from_p0 ? p0[2 * pi + 1] : p1[2 * pi + 1];
  uint8_t st = 1;
  int nlev = 0, nit = 0;  // levels with a prev window gathered, iterations (algorithmic bytes, LkSlots::bytes)
#ifdef UVHP_LK_PROF
  unsigned long long c_setup = 0, c_stage = 0, c_iter = 0;
  int n_stage = 0;
  LKP_T(c_begin);
#endif
  const float p0x = p0[2 * pi], p0y = p0[2 * pi + 1];
  // The template window of level l and its derivatives: the four bilinear taps of each pixel, image at
  // reflect-101 coordinates, derivatives zero outside the level (both channels in one 32-bit load).  The
  // template depends only on p0, so level l - 1's taps are gathered as soon as level l's are consumed and
  // their latency overlaps level l's iterations.  The window corner is clamped into the level's valid range
  // for the gather only: a level whose window is outside is skipped below and its taps are not used.
  int gi[kPer][4], gd[kPer][4], gm[kPer];  // gm: bit k set = derivative tap k inside the level
  auto gather = [&](int l) {
    const uint8_t *I = prev.img[l];
    const int *d32 = reinterpret_cast<const int *>(prev.der[l]);
    const int Iw_ = prev.w[l], Ih_ = prev.h[l];
    const float sc = (float)(1. / (1 << l));
    float prx = p0x * sc, pry = p0y * sc;
    prx -= halfw;
    pry -= halfw;
    const int ipx = min(max((int)floorf(prx), -win), Iw_ - 1), ipy = min(max((int)floorf(pry), -win), Ih_ - 1);
    if (ipx >= 0 && ipx + win < Iw_ && ipy >= 0 && ipy + win < Ih_) {  // window and taps inside: plain loads
#pragma unroll
      for (int q = 0; q < kPer; q++) {
        const size_t o = (size_t)(ipy + wy[q]) * Iw_ + ipx + wx[q];
        gi[q][0] = I[o];
        gi[q][1] = I[o + 1];
        gi[q][2] = I[o + Iw_];
        gi[q][3] = I[o + Iw_ + 1];
        gd[q][0] = d32[o];
        gd[q][1] = d32[o + 1];
        gd[q][2] = d32[o + Iw_];
        gd[q][3] = d32[o + Iw_ + 1];
        gm[q] = 0xf;
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < kPer; q++) {
      const int X = ipx + wx[q], Y = ipy + wy[q];
      const int rx0 = reflect101(X, Iw_), rx1 = reflect101(X + 1, Iw_);
      const size_t ry0 = (size_t)reflect101(Y, Ih_) * Iw_, ry1 = (size_t)reflect101(Y + 1, Ih_) * Iw_;
      gi[q][0] = I[ry0 + rx0];
      gi[q][1] = I[ry0 + rx1];
      gi[q][2] = I[ry1 + rx0];
      gi[q][3] = I[ry1 + rx1];
      const int cx0 = min(max(X, 0), Iw_ - 1), cx1 = min(max(X + 1, 0), Iw_ - 1);
      const size_t cy0 = (size_t)min(max(Y, 0), Ih_ - 1) * Iw_, cy1 = (size_t)min(max(Y + 1, 0), Ih_ - 1) * Iw_;
      gd[q][0] = d32[cy0 + cx0];
      gd[q][1] = d32[cy0 + cx1];
      gd[q][2] = d32[cy1 + cx0];
      gd[q][3] = d32[cy1 + cx1];
      // the masks are applied where the taps are consumed: a select right after a load would wait for it here
      const bool vx0 = X >= 0 && X < Iw_, vx1 = X + 1 >= 0 && X + 1 < Iw_;
      const bool vy0 = Y >= 0 && Y < Ih_, vy1 = Y + 1 >= 0 && Y + 1 < Ih_;
      gm[q] = (vx0 && vy0) | (vx1 && vy0) << 1 | (vx0 && vy1) << 2 | (vx1 && vy1) << 3;
    }
  };
  if (maxL >= 0) gather(maxL);
  for (int level = maxL; level >= 0; level--) {
    const uint8_t *J = next.img[level];
    const int Iw_ = prev.w[level], Ih_ = prev.h[level], Jw_ = next.w[level], Jh_ = next.h[level];
    const float sc = (float)(1. / (1 << level));
    float prx = p0x * sc, pry = p0y * sc;
    if (level == maxL) {
      qx = qx * sc;
      qy = qy * sc;
    } else {
      qx = qx * 2.f;
      qy = qy * 2.f;
    }
    prx -= halfw;
    pry -= halfw;
    LKP_T(c_l0);
    const int ipx = (int)floorf(prx), ipy = (int)floorf(pry);
    if (ipx < -win || ipx >= Iw_ || ipy < -win || ipy >= Ih_) {
      if (level == 0) st = 0;
      if (level > 0) gather(level - 1);
      continue;
    }
    float a = prx - ipx, b = pry - ipy;
    int iw00 = (int)rintf((1.f - a) * (1.f - b) * WSCALE);
    int iw01 = (int)rintf(a * (1.f - b) * WSCALE);
    int iw10 = (int)rintf((1.f - a) * b * WSCALE);
    int iw11 = (1 << 14) - iw00 - iw01 - iw10;
    int sA11 = 0, sA12 = 0, sA22 = 0;
#pragma unroll
    for (int q = 0; q < kPer; q++) {
      const int ival = descale(dot4_i24(gi[q][0], gi[q][1], gi[q][2], gi[q][3], iw00, iw01, iw10, iw11), 14 - 5);
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (!(gm[q] >> k & 1)) gd[q][k] = 0;
      auto lo = [](int v) { return (int)(int16_t)(v & 0xffff); };
      auto hi = [](int v) { return v >> 16; };
      const int ixv = descale(dot4_i24(lo(gd[q][0]), lo(gd[q][1]), lo(gd[q][2]), lo(gd[q][3]), iw00, iw01, iw10, iw11), 14);
      const int iyv = descale(dot4_i24(hi(gd[q][0]), hi(gd[q][1]), hi(gd[q][2]), hi(gd[q][3]), iw00, iw01, iw10, iw11), 14);
      const bool in = lane + 64 * q < area;
      Iw[q] = in ? (int16_t)ival : 0;
      dIx[q] = in ? (int16_t)ixv : 0;
      dIy[q] = in ? (int16_t)iyv : 0;
      sA11 += dIx[q] * dIx[q];
      sA12 += dIx[q] * dIy[q];
      sA22 += dIy[q] * dIy[q];
    }
    if (level > 0) gather(level - 1);
    long long s3[3];
    wave_sum_rows_i32<3>({sA11, sA12, sA22}, s3);
    const float A11 = (float)s3[0] * FLT_SCALE, A12 = (float)s3[1] * FLT_SCALE, A22 = (float)s3[2] * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
    if (minEig < 1e-4f || D < 1.19209290e-07f) {
      if (level == 0) st = 0;
      continue;
    }
    D = 1.f / D;
    nlev++;
#ifdef UVHP_LK_PROF
    c_setup += clock64() - c_l0;
#endif
    float nx = qx - halfw, ny = qy - halfw;
    float pdx = 0.f, pdy = 0.f;
    int ox = -(1 << 28), oy = -(1 << 28);
    for (int j = 0; j < max_iters; j++) {
      LKP_T(c_i0);
      const int inx = (int)floorf(nx), iny = (int)floorf(ny);
      if (inx < -win || inx >= Jw_ || iny < -win || iny >= Jh_) {
        if (level == 0) st = 0;
        break;
      }
      if (inx - ox < 0 || inx - ox > 2 * kLkMargin || iny - oy < 0 || iny - oy > 2 * kLkMargin) {
        __syncthreads();
        ox = inx - kLkMargin;
        oy = iny - kLkMargin;
        uint8_t v[kStageN];
        if (ox >= 0 && ox + S <= Jw_ && oy >= 0 && oy + S <= Jh_) {
#pragma unroll
          for (int k = 0; k < kStageN; k++) v[k] = J[(size_t)(oy + sy[k]) * Jw_ + ox + sx[k]];
        } else {
#pragma unroll
          for (int k = 0; k < kStageN; k++) v[k] = J[(size_t)reflect101(oy + sy[k], Jh_) * Jw_ + reflect101(ox + sx[k], Jw_)];
        }
#pragma unroll
        for (int k = 0; k < kStageN; k++)
          if (lane + 64 * k < S * S) Jt[lane + 64 * k] = v[k];
        __syncthreads();
#ifdef UVHP_LK_PROF
        c_stage += clock64() - c_i0;
        n_stage++;
#endif
      }
      a = nx - inx;
      b = ny - iny;
      iw00 = (int)rintf((1.f - a) * (1.f - b) * WSCALE);
      iw01 = (int)rintf(a * (1.f - b) * WSCALE);
      iw10 = (int)rintf((1.f - a) * b * WSCALE);
      iw11 = (1 << 14) - iw00 - iw01 - iw10;
      int ib1 = 0, ib2 = 0;
      nit++;
      const uint8_t *t0 = Jt + (iny - oy) * S + (inx - ox);
      int tp[kPer][4];
#pragma unroll
      for (int q = 0; q < kPer; q++) {
        const uint8_t *t = t0 + jo[q];
        tp[q][0] = t[0];
        tp[q][1] = t[1];
        tp[q][2] = t[S];
        tp[q][3] = t[S + 1];
      }
#pragma unroll
      for (int q = 0; q < kPer; q++) {  // pixels past the window have dIx = dIy = 0
        const int diff = descale(dot4_i24(tp[q][0], tp[q][1], tp[q][2], tp[q][3], iw00, iw01, iw10, iw11), 14 - 5) - Iw[q];
        ib1 += diff * dIx[q];
        ib2 += diff * dIy[q];
      }
      long long s2[2];
      wave_sum_rows_i32<2>({ib1, ib2}, s2);
      const float b1 = (float)s2[0] * FLT_SCALE, b2 = (float)s2[1] * FLT_SCALE;
      const float dx = (A12 * b2 - A22 * b1) * D;
      const float dy = (A12 * b1 - A11 * b2) * D;
      nx += dx;
      ny += dy;
      qx = nx + halfw;
      qy = ny + halfw;
#ifdef UVHP_LK_PROF
      c_iter += clock64() - c_i0;
#endif
      // the reference's test is in double; a float estimate (relative error < 2^-21) decides it unless it
      // lies within 1e-4 of the threshold, where the double test runs
      const float e2 = dx * dx + dy * dy;
      bool conv = e2 < crit_eps * 0.9999f;
      if (!conv && !(e2 > crit_eps * 1.0001f)) conv = (double)dx * dx + (double)dy * dy <= (double)crit_eps;
      if (conv) break;
      if (j > 0 && fabsf(dx + pdx) < 0.01f && fabsf(dy + pdy) < 0.01f) {
        qx -= dx * 0.5f;
        qy -= dy * 0.5f;
        break;
      }
      pdx = dx;
      pdy = dy;
    }
  }
  if (lane == 0) {
    p1[2 * pi] = qx;
    p1[2 * pi + 1] = qy;
    status[pi] = st;
    if (bytes) atomicAdd(bytes, (unsigned long long)(256 * (5 * nlev + nit)));
#ifdef UVHP_LK_PROF
    if (pi < 4096) g_lk_prof[pi] = LkProf{c_setup, c_stage, c_iter - c_stage, clock64() - c_begin, nit, n_stage, nlev, 0};
#endif
  }
  return make_float2(qx, qy);  // the result every lane holds (wave-uniform)
}

// one point of one slot per workgroup (both cameras' temporal tracks in one launch).  Consecutive points (the
// tracker's order: grid cells, so image neighbours) go to one XCD, whose L2 then serves their overlapping
// windows and pyramid rows once instead of once per XCD
__global__ void __launch_bounds__(64) k_lk(LkSlots job, int win, int max_level, int max_iters, float crit_eps,
                                           int init_from_p0) {
  const int idx = xcd_contiguous(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int slot = idx / gridDim.x, p = idx - slot * gridDim.x;
  if (p >= job.n[slot]) return;
  const float2 q = lk_point(job.prev[slot], job.next[slot], job.p0[slot], job.p1[slot], job.st[slot], p, win,
                            max_level, max_iters, crit_eps, init_from_p0, job.bytes);
  if (job.undistort && threadIdx.x < 2) {  // RANSAC's undistortion of this point, the k_undistort formula
    const int w = threadIdx.x;
    const float px = w ? q.x : job.p0[slot][2 * p], py = w ? q.y : job.p0[slot][2 * p + 1];
    float x, y;
    const bool amb = cam_undistort_f(w ? job.c1[slot] : job.c0[slot], px, py, x, y);
    float *out = w ? job.p1n[slot] : job.p0n[slot];
    out[2 * p] = x;
    out[2 * p + 1] = y;
    if (w && job.p1amb[slot]) job.p1amb[slot][p] = amb ? 1 : 0;
  }
}

__global__ void __launch_bounds__(256) k_undistort_points(CamParams cam, int n, const float *__restrict__ uv,
                                                          float *__restrict__ uvn, uint8_t *__restrict__ amb) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  float x, y;
  const bool a = cam_undistort_f(cam, uv[2 * p], uv[2 * p + 1], x, y);
  uvn[2 * p] = x;
  uvn[2 * p + 1] = y;
  if (amb) amb[p] = a ? 1 : 0;
}

void launch_undistort_points(hipStream_t s, const CamParams &cam, int n, const float *uv, float *uvn, uint8_t *amb) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_undistort_points, dim3((n + 255) / 256), dim3(256), 0, s, cam, n, uv, uvn, amb);
}

// ---------------------------------------------------------------- undistort + RANSAC
// set blockIdx.y = 2 slot + (0: p0 with c0, 1: p1 with c1)
__global__ void k_undistort(RansacSlots job) {
  const int slot = blockIdx.y >> 1, which = blockIdx.y & 1;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= job.n[slot]) return;
  const float *pts = which ? job.p1[slot] : job.p0[slot];
  float *out = which ? job.p1n[slot] : job.p0n[slot];
  float x, y;
  cam_undistort_f(which ? job.c1[slot] : job.c0[slot], pts[2 * p], pts[2 * p + 1], x, y);
  out[2 * p] = x;
  out[2 * p + 1] = y;
}

__device__ int solve_cubic_d(const double *co, double *x) {
  double a = co[0], b = co[1], c = co[2], d = co[3];
  if (a == 0) {
    if (b == 0) {
      if (c == 0) return d == 0 ? -1 : 0;
      x[0] = -d / c;
      return 1;
    }
    double D = c * c - 4 * b * d;
    if (D >= 0) {
      D = sqrt(D);
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
    double theta = acos(R / sqrt(Qcubed));
    double sqrtQ = sqrt(Q);
    double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = b * (1. / 3);
    x[0] = t0 * cos(t1) - t2;
    x[1] = t0 * cos(t1 + (2. * M_PI / 3)) - t2;
    x[2] = t0 * cos(t1 + (4. * M_PI / 3)) - t2;
    return 3;
  } else if (dd == 0) {
    if (R >= 0) {
      x[0] = -2 * pow(R, 1. / 3) - a / 3;
      x[1] = pow(R, 1. / 3) - a / 3;
    } else {
      x[0] = 2 * pow(-R, 1. / 3) - a / 3;
      x[1] = -pow(-R, 1. / 3) - a / 3;
    }
    return x[0] == x[1] ? 1 : 2;
  }
  dd = sqrt(-dd);
  double e = pow(dd + fabs(R), 1. / 3);
  if (R > 0) e = -e;
  x[0] = (e + Q / e) - b * (1. / 3);
  return 1;
}

// 7-point fundamental matrices (oracle fundamental_7pt: Householder QR null space + run7Point cubic)
__device__ int fundamental_7pt_d(const double *x0, const double *y0, const double *x1, const double *y1, double *F) {
  double At[9][7];
  for (int i = 0; i < 7; i++) {
    double a[9] = {x1[i] * x0[i], x1[i] * y0[i], x1[i], y1[i] * x0[i], y1[i] * y0[i], y1[i], x0[i], y0[i], 1.0};
    for (int k = 0; k < 9; k++) At[k][i] = a[k];
  }
  double Vh[7][9], beta[7];
  for (int c = 0; c < 7; c++) {
    double ss = 0;
    for (int r = c; r < 9; r++) ss += At[r][c] * At[r][c];
    double x0v = At[c][c], alpha = (x0v > 0) ? -sqrt(ss) : sqrt(ss);
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
    double e[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    e[7 + q] = 1.0;
    for (int c = 6; c >= 0; c--) {
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
  int nr = solve_cubic_d(c, r);
  if (nr < 1 || nr > 3) return 0;
#pragma unroll
  for (int k = 0; k < 3; k++) {  // compile-time model index: F and r stay in registers
    if (k >= nr) continue;
    double lambda = r[k], mu = 1.;
    double s = f1[8] * r[k] + f2[8];
    double *Fm = F + 9 * k;
    if (fabs(s) > 2.220446049250313e-16) {
      mu = 1. / s;
      lambda *= mu;
      Fm[8] = 1.;
    } else {
      Fm[8] = 0.;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) Fm[i] = f1[i] * lambda + f2[i] * mu;
  }
  return nr;
}

__device__ __forceinline__ bool epipolar_inlier(const double *f, float x0, float y0, float x1, float y1, float t) {
  double a = f[0] * x0 + f[1] * y0 + f[2];
  double b = f[3] * x0 + f[4] * y0 + f[5];
  double c = f[6] * x0 + f[7] * y0 + f[8];
  double s2 = 1. / (a * a + b * b);
  double d2 = x1 * a + y1 * b + c;
  a = f[0] * x1 + f[3] * y1 + f[6];
  b = f[1] * x1 + f[4] * y1 + f[7];
  c = f[2] * x1 + f[5] * y1 + f[8];
  double s1 = 1. / (a * a + b * b);
  double d1 = x0 * a + y0 * b + c;
  float err = (float)fmax(d1 * d1 * s1, d2 * d2 * s2);
  return err <= t;
}

// one wavefront per hypothesis: every lane solves the (tiny) 7-point system redundantly, so the
// model is wave-uniform, then the lanes split the inlier count over the points
__global__ void __launch_bounds__(256) k_ransac_hyp(RansacSlots job, int max_iters) {
  const int slot = blockIdx.y;
  const float *__restrict__ p0n = job.p0n[slot], *__restrict__ p1n = job.p1n[slot];
  const int n = job.n[slot];
  const int *__restrict__ subsets = job.sub[slot];
  const float t = job.t[slot];
  double *__restrict__ Fout = job.F[slot];
  int *__restrict__ nmodels = job.nm[slot], *__restrict__ good = job.good[slot];
  const int it = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (it >= max_iters || n < 7) return;
  double x0[7], y0[7], x1[7], y1[7];
  for (int i = 0; i < 7; i++) {
    int k = subsets[it * 7 + i];
    x0[i] = p0n[2 * k];
    y0[i] = p0n[2 * k + 1];
    x1[i] = p1n[2 * k];
    y1[i] = p1n[2 * k + 1];
  }
  double F[27];
  const int nm = fundamental_7pt_d(x0, y0, x1, y1, F);
  if (lane == 0) nmodels[it] = nm;
  // the inlier counts of all of the hypothesis' models in one pass over the points (the models' division
  // chains interleave and each point is loaded once), two points per lane in flight
  int g[3] = {0, 0, 0};
  for (int i0 = lane; i0 < n; i0 += 128) {
    const int i1 = min(i0 + 64, n - 1);
    const float2 a0 = reinterpret_cast<const float2 *>(p0n)[i0], b0 = reinterpret_cast<const float2 *>(p1n)[i0];
    const float2 a1 = reinterpret_cast<const float2 *>(p0n)[i1], b1 = reinterpret_cast<const float2 *>(p1n)[i1];
    const bool second = i0 + 64 < n;
#pragma unroll
    for (int m = 0; m < 3; m++)
      if (m < nm) {
        g[m] += epipolar_inlier(F + 9 * m, a0.x, a0.y, b0.x, b0.y, t);
        if (second) g[m] += epipolar_inlier(F + 9 * m, a1.x, a1.y, b1.x, b1.y, t);
      }
  }
#pragma unroll
  for (int m = 0; m < 3; m++)
    if (m < nm) {
      int gm = g[m];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) gm += __shfl_xor(gm, o, 64);
      if (lane == 0) {
        good[it * 3 + m] = gm;
        for (int k = 0; k < 9; k++) Fout[(size_t)it * 27 + 9 * m + k] = F[9 * m + k];
      }
    }
}

__device__ int ransac_update_iters_d(double p, double ep, int model_points, int max_iters) {
  p = fmin(fmax(p, 0.), 1.);
  ep = fmin(fmax(ep, 0.), 1.);
  double num = fmax(1. - p, 2.2250738585072014e-308);
  double denom = 1. - pow(1. - ep, model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

// sequential adaptive scan (RANSACPointSetRegistrator::run) on thread 0, then the winner's mask
__global__ void __launch_bounds__(256) k_ransac_select(RansacSlots job, int max_iters, double conf) {
  const int slot = blockIdx.y;
  const float *__restrict__ p0n = job.p0n[slot], *__restrict__ p1n = job.p1n[slot];
  const int n = job.n[slot];
  const float t = job.t[slot];
  const double *__restrict__ Fs = job.F[slot];
  const int *__restrict__ nmodels = job.nm[slot], *__restrict__ good = job.good[slot];
  uint8_t *__restrict__ mask = job.mask[slot];
  if (n <= 0) return;
  if (n < 7) {  // findFundamentalMat needs 7 points: no inliers
    for (int i = threadIdx.x; i < n; i += blockDim.x) mask[i] = 0;
    return;
  }
  __shared__ int best_it, best_m;
  if (threadIdx.x == 0) {
    int niters = max_iters, best = 0, bi = -1, bm = -1;
    for (int it = 0; it < niters && it < max_iters; it++)
      for (int m = 0; m < nmodels[it]; m++) {
        int g = good[it * 3 + m];
        if (g > max(best, 6)) {
          best = g;
          bi = it;
          bm = m;
          niters = ransac_update_iters_d(conf, (double)(n - g) / n, 7, niters);
        }
      }
    best_it = bi;
    best_m = bm;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint8_t v = 0;
    if (best_it >= 0) v = epipolar_inlier(Fs + (size_t)best_it * 27 + 9 * best_m, p0n[2 * i], p0n[2 * i + 1], p1n[2 * i],
                                          p1n[2 * i + 1], t);
    mask[i] = v;
  }
}

// ---------------------------------------------------------------- launch wrappers
void launch_fast_multi(hipStream_t s, const FastJob &job, const int *cells, int thr, int kmax, float *out, int *out_n,
                       int *sort_stats) {
  if (job.ncam <= 0 || job.ncam > kMaxCams) return;
  const int ncell = job.cell_end[job.ncam - 1];
  if (ncell <= 0) return;
  size_t lds = 0;
  int shmax = 0;
  for (int k = 0; k < job.ncam; k++) {
    if (kmax > kFastMaxK || job.sw[k] * job.sh[k] > 65536)
      throw std::runtime_error("FAST cell / per-cell count beyond the kernel's limits");
    lds = max(lds, fast_lds_bytes(job.sw[k], job.sh[k]));
    shmax = max(shmax, job.sh[k]);
  }
  if (lds > 64 * 1024 && set_dyn_lds((const void *)k_fast_select, (int)lds) < (int)lds)
    throw std::runtime_error("FAST cell too large for LDS");
  hipLaunchKernelGGL(k_fast_score, dim3(ncell, (shmax + kFastBand - 1) / kFastBand), dim3(256), 0, s, job, cells, thr);
  hipLaunchKernelGGL(k_fast_select, dim3(ncell), dim3(kFastThreads), lds, s, job, cells, kmax, out, out_n, sort_stats);
}

void launch_grid_order_probe(hipStream_t s, const uint8_t *resp, const int *off, int ncell, int nmax, int kmax,
                             int depth, int *arrangement, int *top) {
  if (ncell <= 0) return;
  if (kmax > kFastMaxK || nmax > 65536) throw std::runtime_error("grid order probe: cell beyond the kernel's limits");
  const size_t lds = (size_t)nmax * 8;
  if (lds > 64 * 1024 && set_dyn_lds((const void *)k_grid_order_probe, (int)lds) < (int)lds)
    throw std::runtime_error("grid order probe: cell too large for LDS");
  hipLaunchKernelGGL(k_grid_order_probe, dim3(ncell), dim3(kFastThreads), lds, s, resp, off, kmax, depth, arrangement,
                     top);
}

void launch_fast_cells(hipStream_t s, const uint8_t *img, int w, int h, const int *cells, int ncell, int sw, int sh, int thr,
                       int kmax, float *out, int *out_n, uint8_t *score_map) {
  (void)h;
  FastJob job{};
  job.img[0] = img;
  job.score[0] = score_map;
  job.w[0] = w;
  job.sw[0] = sw;
  job.sh[0] = sh;
  job.cell_end[0] = ncell;
  job.ncam = 1;
  launch_fast_multi(s, job, cells, thr, kmax, out, out_n, nullptr);
}

void launch_subpix_multi(hipStream_t s, const SubpixJob &job, float *pts, const float *mask, int win, int max_iters,
                         double eps2) {
  if (job.ncam <= 0 || job.ncam > kMaxCams) return;
  const int n = job.end[job.ncam - 1];
  if (n <= 0) return;
  switch (win) {
#define UVHP_SUBPIX(W)                                                                            \
  case W:                                                                                         \
    hipLaunchKernelGGL(k_subpix<W>, dim3(n), dim3(64), 0, s, job, pts, mask, max_iters, eps2); \
    break;
    UVHP_SUBPIX(1)
    UVHP_SUBPIX(2)
    UVHP_SUBPIX(3)
    UVHP_SUBPIX(4)
    UVHP_SUBPIX(5)
#undef UVHP_SUBPIX
    default:
      throw std::runtime_error("cornerSubPix window outside the kernel's 1..5 instantiations");
  }
}

void launch_subpix(hipStream_t s, const uint8_t *img, int w, int h, float *pts, int n, const float *mask, int win,
                   int max_iters, double eps2) {
  SubpixJob job{};
  job.img[0] = img;
  job.w[0] = w;
  job.h[0] = h;
  job.end[0] = n;
  job.ncam = 1;
  launch_subpix_multi(s, job, pts, mask, win, max_iters, eps2);
}

void launch_lk(hipStream_t s, const LkSlots &job, int nslot, int win, int max_level, int max_iters, float eps,
               bool init_from_p0) {
  int nmax = 0;
  for (int k = 0; k < nslot; k++) nmax = max(nmax, job.n[k]);
  if (nmax <= 0) return;
  if (win > kLkMaxWin) throw std::runtime_error("LK window larger than the kernel supports");
  hipLaunchKernelGGL(k_lk, dim3(nmax, nslot), dim3(64), 0, s, job, win, max_level, max_iters, eps * eps,
                     init_from_p0 ? 1 : 0);
}

void launch_ransac(hipStream_t s, const RansacSlots &job, int nslot, int max_iters, double conf, bool undistorted) {
  int nmax = 0;
  for (int k = 0; k < nslot; k++) nmax = max(nmax, job.n[k]);
  if (nmax <= 0) return;
  if (!undistorted) hipLaunchKernelGGL(k_undistort, dim3((nmax + 127) / 128, 2 * nslot), dim3(128), 0, s, job);
  hipLaunchKernelGGL(k_ransac_hyp, dim3((max_iters + 3) / 4, nslot), dim3(256), 0, s, job, max_iters);
  hipLaunchKernelGGL(k_ransac_select, dim3(1, nslot), dim3(256), 0, s, job, max_iters, conf);
}

}  // namespace uvhp
