// KLT front-end host orchestration — see tracker.h.  Reference: ov_core TrackKLT.cpp:34-886,
// Grider_GRID.h:74-180 (restated for the checker in oracle/src/tracker_klt.cpp).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <unordered_map>
#include <unordered_set>

#include "tracker.h"

namespace uvhp {

// Open-addressing id -> value table for the per-frame track bookkeeping (a few hundred ids): one allocation per
// frame instead of one node per id (std::unordered_map / set cost tens of microseconds per frame here).
// emplace keeps the first value of an id, as std::unordered_map::emplace does.
class IdTable {
 public:
  explicit IdTable(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 1) cap <<= 1;
    keys_.assign(cap, kEmpty);
    vals_.resize(cap);
    mask_ = cap - 1;
  }
  void emplace(size_t id, size_t v) {
    size_t h = slot(id);
    while (keys_[h] != kEmpty && keys_[h] != id) h = (h + 1) & mask_;
    if (keys_[h] == kEmpty) {
      keys_[h] = id;
      vals_[h] = v;
    }
  }
  const size_t *find(size_t id) const {
    for (size_t h = slot(id);; h = (h + 1) & mask_) {
      if (keys_[h] == id) return &vals_[h];
      if (keys_[h] == kEmpty) return nullptr;
    }
  }
  bool contains(size_t id) const { return find(id) != nullptr; }

 private:
  static constexpr size_t kEmpty = ~(size_t)0;
  size_t slot(size_t id) const { return (size_t)((id * 0x9E3779B97F4A7C15ull) >> 20) & mask_; }
  std::vector<size_t> keys_, vals_;
  size_t mask_ = 0;
};

namespace {
constexpr int kRansacIters = 1000;      // findFundamentalMat(FM_RANSAC, thr, 0.999) default maxIters
constexpr double kRansacConf = 0.999;   // TrackKLT.cpp:878
constexpr int kLkIters = 30;            // TermCriteria(COUNT + EPS, 30, 0.01), TrackKLT.cpp:641 / 852
constexpr float kLkEps = 0.01f;
constexpr int kSubpixWin = 5, kSubpixIters = 20;  // Grider_GRID.h:170-175: Size(5,5), (20, 0.001)
constexpr double kSubpixEps = 0.001;
constexpr double kMinFeatPercent = 0.50;        // TrackKLT.cpp:466 / 590

// cv::RNG((uint64)-1): multiply-with-carry, coefficient 4164903690 (CV_RNG_COEFF)
struct MwcRng {
  uint64_t s;
  unsigned next() {
    s = (uint64_t)(unsigned)s * 4164903690U + (unsigned)(s >> 32);
    return (unsigned)s;
  }
};

uint8_t mask_px(const std::vector<uint8_t> &m, int w, int x, int y) { return m.empty() ? 0 : m[(size_t)y * w + x]; }
// cv::resize(mask, Size(GX, GY), INTER_NEAREST) sampled at grid cell (gx, gy)
uint8_t mask_cell(const std::vector<uint8_t> &m, int w, int h, int gx, int gy, int GX, int GY) {
  if (m.empty()) return 0;
  int sx = std::min((int)std::floor(gx * ((double)w / GX)), w - 1);
  int sy = std::min((int)std::floor(gy * ((double)h / GY)), h - 1);
  return m[(size_t)sy * w + sx];
}
// the min-distance boxes TrackKLT draws into mask0_updated (cv::rectangle FILLED, inclusive corners)
bool in_boxes(const std::vector<int> &boxes, int d, int x, int y) {
  for (size_t k = 0; k + 1 < boxes.size(); k += 2)
    if (std::abs(x - boxes[k]) <= d && std::abs(y - boxes[k + 1]) <= d) return true;
  return false;
}
struct Occupancy {  // cv::Mat grid_2d_close / grid_2d_grid (CV_8UC1)
  int w, h;
  std::vector<uint8_t> d;
  Occupancy(int w_, int h_) : w(w_), h(h_), d((size_t)std::max(w_, 0) * std::max(h_, 0), 0) {}
  uint8_t &at(int x, int y) { return d[(size_t)y * w + x]; }
};
}  // namespace

struct Tracker::Bufs {
  int cap = 0, maxcells = 0, kmax = 0;
  char *dmem = nullptr, *hmem = nullptr;
  size_t mirror = 0;  // bytes [0, mirror) of the device block are mirrored in pinned host memory
  // device (host mirror: hp(x)); the matching inputs [p0 | sub] x kMaxCams slots and outputs
  // [p1 | st | mask | amb | p1n] x kMaxCams are contiguous so each direction is one copy per frame
  float *p0[kMaxCams], *p1[kMaxCams], *p0n[kMaxCams], *p1n[kMaxCams];
  uint8_t *st[kMaxCams], *mask[kMaxCams], *amb[kMaxCams];
  int *sub[kMaxCams], *nm[kMaxCams], *good[kMaxCams];
  double *F[kMaxCams];
  int *cells, *fastn;
  float *fast, *det, *det1, *spmask;
  uint8_t *detst;
  template <class T>
  T *hp(T *dev) const {
    return (T *)(hmem + ((char *)dev - dmem));
  }
};

namespace {
struct Arena {
  size_t off = 0;
  char *base = nullptr;
  template <class T>
  T *take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T *p = (T *)(base ? base + off : nullptr);
    off += n * sizeof(T);
    return p;
  }
};
size_t span(const void *a, const void *b_end) { return (size_t)((const char *)b_end - (const char *)a); }
}  // namespace

Tracker::Tracker(const uvio_hp_options_t &o, const CamParams *cams, hipStream_t s, KProf *kp)
    : cams_(cams), s_(s), kp_(kp), cur_(s) {
  downsample_ = o.downsample_cameras != 0;
  // TrackKLT construction in VioManager.cpp:98-107: num_pts per camera = init_max_features / ncam
  num_features_ = (int)std::floor((double)o.init_max_features / (double)o.num_cameras);
  threshold_ = o.fast_threshold;
  grid_x_ = o.grid_x;
  grid_y_ = o.grid_y;
  min_px_dist_ = o.min_px_dist;
  histogram_method_ = o.histogram_method;
  use_stereo_ = o.use_stereo != 0;
  currid = 4 * (size_t)o.max_aruco_features + 1;
  if (num_features_ <= 0 || grid_x_ <= 0 || grid_y_ <= 0 || min_px_dist_ <= 0)
    throw HpError(UVIO_HP_E_CONFIG, "tracker: num features / grid / min_px_dist must be positive");
  // cornerSubPix window weights (cornersubpix.cpp: exp(-x^2) exp(-y^2), x, y in [-1, 1])
  const int ww = 2 * kSubpixWin + 1;
  spmask_host_.resize((size_t)ww * ww);
  for (int i = 0; i < ww; i++) {
    float y = (float)(i - kSubpixWin) / kSubpixWin;
    float vy = std::exp(-y * y);
    for (int j = 0; j < ww; j++) {
      float x = (float)(j - kSubpixWin) / kSubpixWin;
      spmask_host_[(size_t)i * ww + j] = (float)(vy * std::exp(-x * x));
    }
  }
  b_ = new Bufs();
  b_->maxcells = grid_x_ * grid_y_;
  int gx = grid_x_, gy = grid_y_;
  if (num_features_ < gx * gy) {
    double ratio = (double)gx / (double)gy;
    gy = (int)std::ceil(std::sqrt(num_features_ / ratio));
    gx = (int)std::ceil(gy * ratio);
  }
  b_->kmax = (int)((double)num_features_ / (double)(gx * gy)) + 1;
  ensure_cap(std::max(1024, 8 * num_features_));
  HP_HIP(hipMalloc(&d_lk_bytes_, sizeof(unsigned long long)));
  HP_HIP(hipMemsetAsync(d_lk_bytes_, 0, sizeof(unsigned long long), s_));
  HP_HIP(hipMalloc(&d_sort_stats_, sizeof(int)));
  HP_HIP(hipMemsetAsync(d_sort_stats_, 0, sizeof(int), s_));
}

void Tracker::set_num_features(int n) {
  if (n <= 0) throw HpError(UVIO_HP_E_CONFIG, "tracker: num features must be positive");
  predetect_join();
  discard_predetect();  // made with the previous count
  num_features_ = n;
  int gx = grid_x_, gy = grid_y_;
  if (num_features_ < gx * gy) {
    double ratio = (double)gx / (double)gy;
    gy = (int)std::ceil(std::sqrt(num_features_ / ratio));
    gx = (int)std::ceil(gy * ratio);
  }
  const int kmax = (int)((double)num_features_ / (double)(gx * gy)) + 1;
  const int cap = std::max(b_->cap, 8 * num_features_);
  if (kmax != b_->kmax || cap > b_->cap) {  // the per-cell FAST top-k table is sized by kmax: reallocate
    b_->kmax = kmax;
    b_->cap = 0;
    ensure_cap(cap);
  }
}

unsigned long long Tracker::lk_bytes() {
  predetect_join();
  unsigned long long v = 0;
  HP_HIP(hipMemcpyAsync(&v, d_lk_bytes_, sizeof(v), hipMemcpyDeviceToHost, s_));
  HP_HIP(hipStreamSynchronize(s_));
  return v;
}

void Tracker::grid_stats(unsigned long long *cells, unsigned long long *introsort_cells) {
  predetect_join();
  if (sd_) HP_HIP(hipStreamSynchronize(sd_));
  int v = 0;
  HP_HIP(hipMemcpyAsync(&v, d_sort_stats_, sizeof(v), hipMemcpyDeviceToHost, s_));
  HP_HIP(hipStreamSynchronize(s_));
  if (cells) *cells = grid_cells_;
  if (introsort_cells) *introsort_cells = (unsigned long long)v;
}

Tracker::~Tracker() {
  if (worker_.joinable()) {
    {
      std::unique_lock<std::mutex> lk(wm_);
      wcv_.wait(lk, [&] { return !w_task_ && !w_busy_; });
      w_quit_ = true;
    }
    wcv_.notify_all();
    worker_.join();
  }
  for (auto &kv : cs_) {
    for (int k = 0; k < 2; k++)
      if (kv.second.pyr_mem[k]) (void)hipFree(kv.second.pyr_mem[k]);
    if (kv.second.d_raw) (void)hipFree(kv.second.d_raw);
    if (kv.second.d_half) (void)hipFree(kv.second.d_half);
    if (kv.second.d_hist) (void)hipFree(kv.second.d_hist);
    if (kv.second.d_score) (void)hipFree(kv.second.d_score);
  }
  if (d_lk_bytes_) (void)hipFree(d_lk_bytes_);
  if (d_sort_stats_) (void)hipFree(d_sort_stats_);
  if (ev_match_) (void)hipEventDestroy(ev_match_);
  if (ev_up_) (void)hipEventDestroy(ev_up_);
  if (up_) (void)hipStreamDestroy(up_);
  if (ev_pyr_) (void)hipEventDestroy(ev_pyr_);
  if (sd_) {
    (void)hipStreamSynchronize(sd_);
    (void)hipStreamDestroy(sd_);
  }
  if (b_) {
    if (b_->dmem) (void)hipFree(b_->dmem);
    if (b_->hmem) (void)hipHostFree(b_->hmem);
    delete b_;
  }
}

// The tracker's device buffers an upload writes are read only by this frame's later launches: the previous
// frame's users of them finished before its results were read back.
void Tracker::upload(void *dst, const void *src, size_t bytes) {
  if (cur_ != s_) {  // predetect: its own stream, nothing queued on it to overlap
    HP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, cur_));
    return;
  }
  if (!up_) {
    HP_HIP(hipStreamCreateWithFlags(&up_, hipStreamNonBlocking));
    HP_HIP(hipEventCreateWithFlags(&ev_up_, hipEventDisableTiming));
  }
  if (hipStreamQuery(s_) == hipSuccess) {  // nothing to overlap: the cross-stream wait would only add latency
    HP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s_));
    return;
  }
  HP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, up_));
  HP_HIP(hipEventRecord(ev_up_, up_));
  HP_HIP(hipStreamWaitEvent(s_, ev_up_, 0));
}

void Tracker::sync() {
  auto t0 = std::chrono::steady_clock::now();
  spin_sync(cur_);
  const double w = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (pre_mode_) {
    pre_wait += w;
    pre_syncs++;
  } else {
    sync_wait += w;
    device_syncs++;
  }
}

void Tracker::ensure_cap(int n) {
  Bufs &b = *b_;
  if (n <= b.cap) return;
  if (b.dmem) {
    if (sd_) spin_sync(sd_);
    if (cur_ != s_) spin_sync(s_);  // predetect: the frame's updates hold no tracker buffer, but wait anyway
    sync();
    HP_HIP(hipFree(b.dmem));
    HP_HIP(hipHostFree(b.hmem));
    b.dmem = b.hmem = nullptr;
  }
  int cap = std::max(n, 2 * b.cap);
  size_t ncell = (size_t)b.maxcells * kMaxCams;  // the grid cells of every camera of one feed
  for (int pass = 0; pass < 2; pass++) {
    Arena d;
    if (pass == 1) d.base = b.dmem;
    for (int k = 0; k < kMaxCams; k++) {  // matching inputs of every slot: one upload
      b.p0[k] = d.take<float>(2 * cap);
      b.sub[k] = d.take<int>(7 * kRansacIters);
    }
    for (int k = 0; k < kMaxCams; k++) {  // matching outputs of every slot: one readback
      b.p1[k] = d.take<float>(2 * cap);
      b.st[k] = d.take<uint8_t>(cap);
      b.mask[k] = d.take<uint8_t>(cap);
      b.amb[k] = d.take<uint8_t>(cap);    // p1n's ambiguity flags (cam_undistort_f)
      b.p1n[k] = d.take<float>(2 * cap);  // the tracked points undistorted (RANSAC's input), for the database
    }
    b.cells = d.take<int>(2 * ncell);
    b.fastn = d.take<int>(ncell);
    b.fast = d.take<float>(3 * ncell * b.kmax);
    b.det = d.take<float>(2 * cap);
    b.det1 = d.take<float>(2 * cap);
    b.detst = d.take<uint8_t>(cap);
    const size_t mirror = d.off;
    for (int k = 0; k < kMaxCams; k++) {
      b.p0n[k] = d.take<float>(2 * cap);
      b.nm[k] = d.take<int>(kRansacIters);
      b.good[k] = d.take<int>(3 * kRansacIters);
      b.F[k] = d.take<double>(27 * kRansacIters);
    }
    b.spmask = d.take<float>(spmask_host_.size());
    if (pass == 0) {
      b.mirror = mirror;
      HP_HIP(hipMalloc(&b.dmem, d.off + 256));
      HP_HIP(hipHostMalloc(&b.hmem, mirror + 256, hipHostMallocDefault));
    }
  }
  b.cap = cap;
  HP_HIP(hipMemcpy(b.spmask, spmask_host_.data(), spmask_host_.size() * sizeof(float), hipMemcpyHostToDevice));
}

Tracker::CamState &Tracker::cam_state(int cid) {
  auto it = cs_.find(cid);
  if (it != cs_.end()) return it->second;
  CamState &c = cs_[cid];
  alloc_pyr(c, cams_[cid].w, cams_[cid].h);
  return c;
}

// buildOpticalFlowPyramid level sizes (stops once the next side would be <= win) for both slots
void Tracker::alloc_pyr(CamState &c, int w, int h) {
  DPyr p{};
  int lw = w, lh = h;
  size_t bytes = 0;
  std::vector<size_t> img_off, der_off;
  for (int level = 0; level <= pyr_levels_ && level < kMaxPyrLevels; level++) {
    p.w[level] = lw;
    p.h[level] = lh;
    p.levels = level + 1;
    img_off.push_back(bytes);
    bytes += ((size_t)lw * lh + 255) & ~(size_t)255;
    der_off.push_back(bytes);
    bytes += ((size_t)lw * lh * 4 + 255) & ~(size_t)255;
    lw = (lw + 1) / 2;
    lh = (lh + 1) / 2;
    if (lw <= win_ || lh <= win_) break;
  }
  for (int k = 0; k < 2; k++) {
    HP_HIP(hipMalloc(&c.pyr_mem[k], bytes));
    c.pyr[k] = p;
    for (int l = 0; l < p.levels; l++) {
      c.pyr[k].img[l] = (const uint8_t *)((char *)c.pyr_mem[k] + img_off[l]);
      c.pyr[k].der[l] = (const int16_t *)((char *)c.pyr_mem[k] + der_off[l]);
    }
  }
  HP_HIP(hipMalloc(&c.d_raw, (size_t)w * h * (downsample_ ? 4 : 1)));
  if (downsample_) HP_HIP(hipMalloc(&c.d_half, (size_t)w * h));
  HP_HIP(hipMalloc(&c.d_hist, 256 * sizeof(unsigned)));
  HP_HIP(hipMemset(c.d_hist, 0, 256 * sizeof(unsigned)));  // cleared after use by each frame's pyramid
  HP_HIP(hipMalloc(&c.d_score, (size_t)w * h));
}

// RANSACPointSetRegistrator::getSubset draws (ptsetreg.cpp), one rng per findFundamentalMat call
const std::vector<int> &Tracker::subsets(int count) {
  auto it = subset_cache_.find(count);
  if (it != subset_cache_.end()) return it->second;
  std::vector<int> &idx = subset_cache_[count];
  idx.assign((size_t)kRansacIters * 7, 0);
  MwcRng rng{~(uint64_t)0};
  for (int it2 = 0; it2 < kRansacIters; it2++) {
    int *s = &idx[(size_t)it2 * 7];
    for (int i = 0; i < 7; i++) {
      for (;;) {
        int v = (int)(rng.next() % (unsigned)count);
        bool dup = false;
        for (int j = 0; j < i; j++) dup |= (s[j] == v);
        if (!dup) {
          s[i] = v;
          break;
        }
      }
    }
  }
  return idx;
}

void Tracker::feed(double t, int ncam, const int *cam_ids, const uint8_t *const *imgs, const int *strides,
                   const uint8_t *const *masks, bool device_imgs, const DbSink &db,
                   std::function<void()> in_flight) {
  if (histogram_method_ == 2)
    throw HpError(UVIO_HP_E_CONFIG, "histogram_method 2 (CLAHE) is not implemented by the KLT front-end");
  if (ncam > kMaxCams) throw HpError(UVIO_HP_E_ARG, "too many cameras in one feed");
  // The predetection (worker thread, detection stream) reads only the last frame's pyramids, points, ids and masks.
  // When every camera of this feed already has its state (no insertion into cs_ while the worker reads it), this
  // frame's pyramids -- the other slot -- are launched first and built while the host joins the worker.
  bool early_pyr = true;
  for (int k = 0; k < ncam; k++)
    if (cs_.find(cam_ids[k]) == cs_.end()) early_pyr = false;
  if (!early_pyr) {
    HostProfScope hs(*hp_, "trk.join");
    predetect_join();
  }
  in_flight_ = std::move(in_flight);
  device_syncs = 0;
  sync_wait = 0.0;
  PyrJob job{};
  job.ncam = ncam;
  job.equalize = histogram_method_ == 1;
  DecimateJob dec{};
  dec.ncam = downsample_ ? ncam : 0;
  for (int k = 0; k < ncam; k++) {
    const int cid = cam_ids[k];
    // with downsample_cameras the configured size is the halved one (VioManagerOptions.h:251-260) and the
    // inputs are the raw 2w x 2h camera images
    const int w = cams_[cid].w, h = cams_[cid].h, f = downsample_ ? 2 : 1, rw = f * w, rh = f * h;
    if (strides[k] < rw) throw HpError(UVIO_HP_E_ARG, "image stride smaller than the configured width");
    CamState &c = cam_state(cid);
    const int nw = 1 - c.last;
    const uint8_t *src = imgs[k];
    int stride = strides[k];
    if (!device_imgs) {
      HP_HIP(hipMemcpy2DAsync(c.d_raw, rw, imgs[k], strides[k], rw, rh, hipMemcpyHostToDevice, s_));
      src = c.d_raw;
      stride = rw;
    }
    if (downsample_) {
      dec.src[k] = src;
      dec.stride[k] = stride;
      dec.dst[k] = c.d_half;
      dec.w[k] = w;
      dec.h[k] = h;
      src = c.d_half;
      stride = w;
    }
    job.p[k] = c.pyr[nw];
    job.src[k] = src;
    job.stride[k] = stride;
    job.hist[k] = c.d_hist;
    c.mask_new.clear();
    if (masks && masks[k]) {
      c.mask_new.resize((size_t)w * h);
      if (downsample_) {  // cv::pyrDown of the mask too (VioManager.cpp:276)
        for (int y = 0; y < h; y++)
          for (int x = 0; x < w; x++) {
            static const int k5[5] = {1, 4, 6, 4, 1};
            auto refl = [](int p, int n) {
              while (p < 0 || p >= n) p = (p < 0) ? -p : 2 * n - 2 - p;
              return p;
            };
            int acc = 0;
            for (int i = 0; i < 5; i++) {
              const uint8_t *row = masks[k] + (size_t)refl(2 * y + i - 2, rh) * strides[k];
              int r = 0;
              for (int j = 0; j < 5; j++) r += k5[j] * row[refl(2 * x + j - 2, rw)];
              acc += k5[i] * r;
            }
            c.mask_new[(size_t)y * w + x] = (uint8_t)((acc + 128) >> 8);
          }
      } else {
        for (int y = 0; y < h; y++) std::memcpy(&c.mask_new[(size_t)y * w], masks[k] + (size_t)y * strides[k], w);
      }
    }
  }
  pyr_launch_ = [this, dec, job]() {
    launch_decimate(s_, dec);
    {
      KScope ks(kp_, KC_PYR);
      launch_pyramids(s_, job);
    }
    if (!ev_pyr_) HP_HIP(hipEventCreateWithFlags(&ev_pyr_, hipEventDisableTiming));
    HP_HIP(hipEventRecord(ev_pyr_, s_));
    if (kp_) kp_->credit(KC_PYR, 0.0, pyramid_bytes(job));
  };
  if (early_pyr) {
    ensure_pyr();
    HostProfScope hs(*hp_, "trk.join");
    predetect_join();
  }
  if (pre_.valid && pre_.cams != std::vector<int>(cam_ids, cam_ids + ncam)) discard_predetect();
  if (ncam == 2 && use_stereo_) {
    feed_stereo(t, cam_ids[0], cam_ids[1], db);
  } else if (ncam > 2 && use_stereo_) {
    // TrackKLT.cpp:90-93: more than two images with use_stereo is an error (std::exit in the reference)
    throw HpError(UVIO_HP_E_ARG, "more than 2 images in one feed with use_stereo");
  } else {
    feed_multi(t, cam_ids, ncam, db);  // mono, or binocular tracking of each camera on its own
  }
  in_flight_ = nullptr;  // not reached (no matching this frame): the caller does that work afterwards
  ensure_pyr();          // a frame without matching still builds its pyramid for the next one
  // pyr_last / mask_last <- this frame's (every TrackKLT path ends this way)
  for (int k = 0; k < ncam; k++) {
    CamState &c = cs_[cam_ids[k]];
    c.last = 1 - c.last;
    c.have_last = true;
    c.mask_last.swap(c.mask_new);
  }
  last_cams_.assign(cam_ids, cam_ids + ncam);
  pre_.valid = false;  // consumed by this feed (or not made for it)
}


// ---------------------------------------------------------------- detection
// Grider_GRID::perform_griding + cornerSubPix for the requests of several cameras at once: the FAST
// scores / top-k of every camera's valid cells in one launch pair and one readback, the sub-pixel
// refinement of every camera's kept corners in one launch and one readback.  With lk_to (one request
// only) the refined points are also tracked into that pyramid (TrackKLT.cpp:640-655).
void Tracker::griding_multi(GridReq *reqs, int nr, const DPyr *lk_to, std::vector<KeyPt> *lk_pts,
                            std::vector<uint8_t> *lk_st) {
  Bufs &b = *b_;
  int gx = grid_x_, gy = grid_y_;
  if (num_features_ < gx * gy) {
    double ratio = (double)gx / (double)gy;
    gy = (int)std::ceil(std::sqrt(num_features_ / ratio));
    gx = (int)std::ceil(gy * ratio);
  }
  const int nfg = b.kmax;
  FastJob fj{};
  int nc = 0, nf = 0;
  std::vector<int> req_cam(nr, -1), cell0(nr, 0);
  for (int r = 0; r < nr; r++) {
    GridReq &q = reqs[r];
    q.out.clear();
    const int W = q.p->w[0], H = q.p->h[0];
    const int size_x = W / gx, size_y = H / gy;
    cell0[r] = nc;
    for (auto &g : q.valid) {
      int x = g.first * size_x, y = g.second * size_y;
      if (x + size_x > W || y + size_y > H) continue;
      b.hp(b.cells)[2 * nc] = x;
      b.hp(b.cells)[2 * nc + 1] = y;
      nc++;
    }
    if (nc == cell0[r]) continue;
    req_cam[r] = nf;
    fj.img[nf] = q.p->img[0];
    fj.score[nf] = cs_.at(q.cam).d_score;  // at(): may run on the worker (predetect)
    fj.w[nf] = W;
    fj.sw[nf] = size_x;
    fj.sh[nf] = size_y;
    fj.cell_end[nf] = nc;
    nf++;
  }
  if (nc == 0) return;
  fj.ncam = nf;
  upload(b.cells, b.hp(b.cells), 2 * nc * sizeof(int));
  {
    KScope ks(kcur(), KC_FAST);
    launch_fast_multi(cur_, fj, b.cells, threshold_, nfg, b.fast, b.fastn, d_sort_stats_);
    grid_cells_ += (unsigned long long)nc;
  }
  // algorithmic bytes: each cell's pixels read by the score pass, its score map written and read by the selection
  if (kcur()) {
    double px = 0.0;
    for (int k = 0; k < nf; k++) px += (double)fj.sw[k] * fj.sh[k] * (fj.cell_end[k] - (k ? fj.cell_end[k - 1] : 0));
    kcur()->credit(KC_FAST, 0.0, 3.0 * px);
  }
  HP_HIP(hipMemcpyAsync(b.hp(b.fastn), b.fastn, span(b.fastn, b.fast + (size_t)3 * nc * nfg), hipMemcpyDeviceToHost, cur_));
  sync();
  const int *h_fastn = b.hp(b.fastn);
  const float *h_fast = b.hp(b.fast);
  const int d = min_px_dist_;
  int total = 0;
  for (int r = 0; r < nr; r++) {
    GridReq &q = reqs[r];
    if (req_cam[r] < 0) continue;
    const int W = q.p->w[0], H = q.p->h[0];
    for (int c = cell0[r]; c < fj.cell_end[req_cam[r]]; c++)
      for (int i = 0; i < h_fastn[c]; i++) {
        const float *f = h_fast + ((size_t)c * nfg + i) * 3;
        KeyPt k{f[0], f[1], f[2]};
        if ((int)k.x < 0 || (int)k.x > W || (int)k.y < 0 || (int)k.y > H) continue;
        if (mask_px(*q.user_mask, W, (int)k.x, (int)k.y) > 127 || in_boxes(*q.boxes, d, (int)k.x, (int)k.y)) continue;
        q.out.push_back(k);
      }
    total += (int)q.out.size();
  }
  if (total == 0) return;
  ensure_cap(total);
  float *h_det = b.hp(b.det), *h_det1 = b.hp(b.det1);
  const uint8_t *h_detst = b.hp(b.detst);
  SubpixJob sj{};
  int np = 0;
  for (int r = 0; r < nr; r++) {
    GridReq &q = reqs[r];
    if (q.out.empty()) continue;
    for (auto &k : q.out) {
      h_det[2 * np] = k.x;
      h_det[2 * np + 1] = k.y;
      np++;
    }
    sj.img[sj.ncam] = q.p->img[0];
    sj.w[sj.ncam] = q.p->w[0];
    sj.h[sj.ncam] = q.p->h[0];
    sj.end[sj.ncam] = np;
    sj.ncam++;
  }
  upload(b.det, h_det, 2 * np * sizeof(float));
  {
    KScope ks(kcur(), KC_SUBPIX);
    launch_subpix_multi(cur_, sj, b.det, b.spmask, kSubpixWin, kSubpixIters, kSubpixEps * kSubpixEps);
  }
  // algorithmic bytes: per corner the (2 win + 3)^2 image patch its iterations sample, the point read and written
  if (kcur()) kcur()->credit(KC_SUBPIX, 0.0, (double)np * ((2 * kSubpixWin + 3) * (2 * kSubpixWin + 3) + 16));
  const bool do_lk = lk_to && nr == 1;
  if (do_lk) {
    LkSlots lk{};
    lk.prev[0] = *reqs[0].p;
    lk.next[0] = *lk_to;
    lk.p0[0] = b.det;
    lk.p1[0] = b.det1;
    lk.st[0] = b.detst;
    lk.n[0] = np;
    // timed on the stream it runs on (the library's, or the detection stream's pairs while predetecting)
    lk.bytes = (kcur() && kcur()->on) ? d_lk_bytes_ : nullptr;
    {
      KScope ks(kcur(), KC_LK);
      launch_lk(cur_, lk, 1, win_, pyr_levels_, kLkIters, kLkEps, true);
    }
    HP_HIP(hipMemcpyAsync(h_det, b.det, span(b.det, b.detst + np), hipMemcpyDeviceToHost, cur_));
  } else {
    HP_HIP(hipMemcpyAsync(h_det, b.det, 2 * np * sizeof(float), hipMemcpyDeviceToHost, cur_));
  }
  sync();
  int at = 0;
  for (int r = 0; r < nr; r++)
    for (auto &k : reqs[r].out) {
      k.x = h_det[2 * at];
      k.y = h_det[2 * at + 1];
      at++;
    }
  if (do_lk) {
    lk_pts->resize(np);
    lk_st->resize(np);
    for (int i = 0; i < np; i++) {
      (*lk_pts)[i] = KeyPt{h_det1[2 * i], h_det1[2 * i + 1], reqs[0].out[i].response};
      (*lk_st)[i] = h_detst[i];
    }
  }
}

void Tracker::griding(int cam, const DPyr &p, const std::vector<uint8_t> &user_mask, const std::vector<int> &boxes,
                      const std::vector<std::pair<int, int>> &valid, std::vector<KeyPt> &out, const DPyr *lk_to,
                      std::vector<KeyPt> *lk_pts, std::vector<uint8_t> *lk_st) {
  out.clear();
  if (valid.empty()) return;
  GridReq q{cam, &p, &user_mask, &boxes, valid, {}};
  griding_multi(&q, 1, lk_to, lk_pts, lk_st);
  out.swap(q.out);
}

// TrackKLT::perform_detection_monocular (TrackKLT.cpp:395-528) of one camera, split around the device
// griding so that the cameras of one feed share its launches: pre keeps the tracked points that pass the
// edge / occupancy / mask tests and lists the cells that need corners, post adds the new corners that
// keep the minimum distance and numbers them (++currid, in camera order: the serial schedule's ids).
struct Tracker::MonoDet {
  int cam;
  const DPyr *p;
  const std::vector<uint8_t> *mask;
  std::vector<KeyPt> pts;
  std::vector<size_t> ids;
  int scw = 0, sch = 0;
  std::vector<uint8_t> close;
  bool run = false;
  std::vector<int> boxes;
  GridReq g;
};

void Tracker::detect_mono_pre(MonoDet &m) {
  const DPyr &p = *m.p;
  const std::vector<uint8_t> &mask0 = *m.mask;
  const int W = p.w[0], H = p.h[0], d = min_px_dist_;
  const int scw = (int)((float)W / (float)d), sch = (int)((float)H / (float)d);
  Occupancy close(scw, sch), grid(grid_x_, grid_y_);
  const float size_x = (float)W / (float)grid_x_, size_y = (float)H / (float)grid_y_;
  std::vector<KeyPt> kp;
  std::vector<size_t> kid;
  m.boxes.clear();
  for (size_t i = 0; i < m.pts.size(); i++) {
    const KeyPt &k = m.pts[i];
    const int x = (int)k.x, y = (int)k.y, edge = 10;
    if (x < edge || x >= W - edge || y < edge || y >= H - edge) continue;
    const int xc = (int)(k.x / (float)d), yc = (int)(k.y / (float)d);
    if (xc < 0 || xc >= scw || yc < 0 || yc >= sch) continue;
    const int xg = (int)std::floor(k.x / size_x), yg = (int)std::floor(k.y / size_y);
    if (xg < 0 || xg >= grid_x_ || yg < 0 || yg >= grid_y_) continue;
    if (close.at(xc, yc) > 127) continue;
    if (mask_px(mask0, W, x, y) > 127) continue;
    close.at(xc, yc) = 255;
    if (grid.at(xg, yg) < 255) grid.at(xg, yg) += 1;
    if (x - d >= 0 && x + d < W && y - d >= 0 && y + d < H) {
      m.boxes.push_back(x);
      m.boxes.push_back(y);
    }
    kp.push_back(k);
    kid.push_back(m.ids[i]);
  }
  m.pts.swap(kp);
  m.ids.swap(kid);
  m.scw = scw;
  m.sch = sch;
  m.close.swap(close.d);
  m.g = GridReq{m.cam, m.p, m.mask, &m.boxes, {}, {}};
  const int needed = num_features_ - (int)m.pts.size();
  m.run = false;
  if (needed < std::min(20, (int)(kMinFeatPercent * num_features_))) return;
  const int nfg = (int)((double)num_features_ / (double)(grid_x_ * grid_y_)) + 1;
  const int nfg_req = std::max(1, (int)(kMinFeatPercent * nfg));
  for (int x = 0; x < grid_x_; x++)
    for (int y = 0; y < grid_y_; y++)
      if ((int)grid.at(x, y) < nfg_req && (int)mask_cell(mask0, W, H, x, y, grid_x_, grid_y_) != 255)
        m.g.valid.emplace_back(x, y);
  m.run = !m.g.valid.empty();
}

void Tracker::detect_mono_post(MonoDet &m) {
  if (!m.run) return;
  const int d = min_px_dist_;
  for (auto &k : m.g.out) {
    const int xg = (int)(k.x / (float)d), yg = (int)(k.y / (float)d);
    if (xg < 0 || xg >= m.scw || yg < 0 || yg >= m.sch) continue;
    uint8_t &cl = m.close[(size_t)yg * m.scw + xg];
    if (cl > 127) continue;
    cl = 255;
    m.pts.push_back(k);
    m.ids.push_back(++currid);
  }
}

// perform_detection_monocular of several cameras: host passes per camera, one shared device griding
void Tracker::detect_mono_multi(MonoDet *m, int n) {
  std::vector<GridReq> reqs;
  std::vector<int> who;
  for (int k = 0; k < n; k++) {
    detect_mono_pre(m[k]);
    if (m[k].run) {
      reqs.push_back(m[k].g);
      who.push_back(k);
    }
  }
  if (!reqs.empty()) {
    griding_multi(reqs.data(), (int)reqs.size(), nullptr, nullptr, nullptr);
    for (size_t r = 0; r < reqs.size(); r++) m[who[r]].g.out.swap(reqs[r].out);
  }
  for (int k = 0; k < n; k++) detect_mono_post(m[k]);
}

// TrackKLT::perform_detection_stereo (TrackKLT.cpp:530-827)
void Tracker::detect_stereo(int cl, int cr, const DPyr &p0, const DPyr &p1, const std::vector<uint8_t> &mask0,
                            const std::vector<uint8_t> &mask1, std::vector<KeyPt> &pts0, std::vector<KeyPt> &pts1,
                            std::vector<size_t> &ids0, std::vector<size_t> &ids1) {
  const int d = min_px_dist_;
  // ---- left: keep, then detect and track the new points into the right image
  {
    const int W = p0.w[0], H = p0.h[0];
    const int scw = (int)((float)W / (float)d), sch = (int)((float)H / (float)d);
    Occupancy close(scw, sch), grid(grid_x_, grid_y_);
    const float size_x = (float)W / (float)grid_x_, size_y = (float)H / (float)grid_y_;
    std::vector<int> boxes;
    std::vector<KeyPt> kp;
    std::vector<size_t> kid;
    for (size_t i = 0; i < pts0.size(); i++) {
      const KeyPt &k = pts0[i];
      const int x = (int)k.x, y = (int)k.y, edge = 10;
      if (x < edge || x >= W - edge || y < edge || y >= H - edge) continue;
      const int xc = (int)(k.x / (float)d), yc = (int)(k.y / (float)d);
      if (xc < 0 || xc >= scw || yc < 0 || yc >= sch) continue;
      const int xg = (int)std::floor(k.x / size_x), yg = (int)std::floor(k.y / size_y);
      if (xg < 0 || xg >= grid_x_ || yg < 0 || yg >= grid_y_) continue;
      if (close.at(xc, yc) > 127) continue;
      if (mask_px(mask0, W, x, y) > 127) continue;
      close.at(xc, yc) = 255;
      if (grid.at(xg, yg) < 255) grid.at(xg, yg) += 1;
      if (x - d >= 0 && x + d < W && y - d >= 0 && y + d < H) {
        boxes.push_back(x);
        boxes.push_back(y);
      }
      kp.push_back(k);
      kid.push_back(ids0[i]);
    }
    pts0.swap(kp);
    ids0.swap(kid);
    const int needed = num_features_ - (int)pts0.size();
    if (needed > std::min(20, (int)(kMinFeatPercent * num_features_))) {
      const int nfg = (int)((double)num_features_ / (double)(grid_x_ * grid_y_)) + 1;
      const int nfg_req = std::max(1, (int)(kMinFeatPercent * nfg));
      std::vector<std::pair<int, int>> valid;
      for (int x = 0; x < grid_x_; x++)
        for (int y = 0; y < grid_y_; y++)
          if ((int)grid.at(x, y) < nfg_req && (int)mask_cell(mask0, W, H, x, y, grid_x_, grid_y_) != 255)
            valid.emplace_back(x, y);
      // LK into the right image runs on every detected point in the same device pass; the
      // min-distance filter below then selects the subset the reference tracks (per-point
      // independent, so the results are the same)
      std::vector<KeyPt> ext, lk_pts;
      std::vector<uint8_t> lk_st;
      griding(cl, p0, mask0, boxes, valid, ext, &p1, &lk_pts, &lk_st);
      const int W1 = p1.w[0], H1 = p1.h[0];
      for (size_t e = 0; e < ext.size(); e++) {
        const KeyPt &k = ext[e];
        const int xg = (int)(k.x / (float)d), yg = (int)(k.y / (float)d);
        if (xg < 0 || xg >= scw || yg < 0 || yg >= sch) continue;
        if (close.at(xg, yg) > 127) continue;
        close.at(xg, yg) = 255;
        const KeyPt &k1 = lk_pts[e];
        const bool oobl = ((int)k.x < 0 || (int)k.x >= W || (int)k.y < 0 || (int)k.y >= H);
        const bool oobr = ((int)k1.x < 0 || (int)k1.x >= W1 || (int)k1.y < 0 || (int)k1.y >= H1);
        if (!oobl && !oobr && lk_st[e] == 1) {
          pts0.push_back(k);
          pts1.push_back(k1);
          const size_t id = ++currid;
          ids0.push_back(id);
          ids1.push_back(id);
        } else if (!oobl) {
          pts0.push_back(k);
          ids0.push_back(++currid);
        }
      }
    }
  }
  // ---- right
  {
    const int W = p1.w[0], H = p1.h[0];
    const int scw = (int)((float)W / (float)d), sch = (int)((float)H / (float)d);
    Occupancy close(scw, sch), grid(grid_x_, grid_y_);
    const float size_x = (float)W / (float)grid_x_, size_y = (float)H / (float)grid_y_;
    std::vector<int> boxes;  // drawn into a clone of the LEFT mask (TrackKLT.cpp:713)
    std::vector<KeyPt> kp;
    std::vector<size_t> kid;
    IdTable left_ids(ids0.size());
    for (size_t id : ids0) left_ids.emplace(id, 0);
    for (size_t i = 0; i < pts1.size(); i++) {
      const KeyPt &k = pts1[i];
      const int x = (int)k.x, y = (int)k.y, edge = 10;
      if (x < edge || x >= W - edge || y < edge || y >= H - edge) continue;
      const int xc = (int)(k.x / (float)d), yc = (int)(k.y / (float)d);
      if (xc < 0 || xc >= scw || yc < 0 || yc >= sch) continue;
      const int xg = (int)std::floor(k.x / size_x), yg = (int)std::floor(k.y / size_y);
      if (xg < 0 || xg >= grid_x_ || yg < 0 || yg >= grid_y_) continue;
      const bool is_stereo = left_ids.contains(ids1[i]);
      if (close.at(xc, yc) > 127 && !is_stereo) continue;
      if (mask_px(mask1, W, x, y) > 127) continue;
      close.at(xc, yc) = 255;
      if (grid.at(xg, yg) < 255) grid.at(xg, yg) += 1;
      if (x - d >= 0 && x + d < W && y - d >= 0 && y + d < H) {
        boxes.push_back(x);
        boxes.push_back(y);
      }
      kp.push_back(k);
      kid.push_back(ids1[i]);
    }
    pts1.swap(kp);
    ids1.swap(kid);
    const int needed = num_features_ - (int)pts1.size();
    if (needed > std::min(20, (int)(kMinFeatPercent * num_features_))) {
      const int nfg = (int)((double)num_features_ / (double)(grid_x_ * grid_y_)) + 1;
      const int nfg_req = std::max(1, (int)(kMinFeatPercent * nfg));
      std::vector<std::pair<int, int>> valid;
      for (int x = 0; x < grid_x_; x++)
        for (int y = 0; y < grid_y_; y++)
          if ((int)grid.at(x, y) < nfg_req && (int)mask_cell(mask1, W, H, x, y, grid_x_, grid_y_) != 255)
            valid.emplace_back(x, y);
      std::vector<KeyPt> ext;
      griding(cr, p1, mask0, boxes, valid, ext, nullptr, nullptr, nullptr);
      for (auto &k : ext) {
        const int xg = (int)(k.x / (float)d), yg = (int)(k.y / (float)d);
        if (xg < 0 || xg >= scw || yg < 0 || yg >= sch) continue;
        if (close.at(xg, yg) > 127) continue;
        pts1.push_back(k);
        ids1.push_back(++currid);
        close.at(xg, yg) = 255;
      }
    }
  }
}

// ---------------------------------------------------------------- temporal matching
// TrackKLT::perform_matching (TrackKLT.cpp:829-886): LK from the last pyramid, then
// findFundamentalMat(FM_RANSAC, 2 / max focal, 0.999) on undistorted points, all on the device.
// match_prepare stages one slot; match_run sends both slots' inputs in one copy, runs LK and RANSAC for
// both in one launch per stage and reads both results back in one copy.
void Tracker::match_prepare(int slot, const DPyr &p0, const DPyr &p1, int cam0, int cam1, const std::vector<KeyPt> &k0,
                            MatchJob &j) {
  j.n = (int)k0.size();
  j.run = j.n >= 10;
  j.slot = slot;
  if (!j.run) return;
  const int n = j.n;
  Bufs &b = *b_;
  float *h_p0 = b.hp(b.p0[slot]);
  for (int i = 0; i < n; i++) {
    h_p0[2 * i] = k0[i].x;
    h_p0[2 * i + 1] = k0[i].y;
  }
  const std::vector<int> &sub = subsets(n);
  std::memcpy(b.hp(b.sub[slot]), sub.data(), sub.size() * sizeof(int));
  j.prev = p0;
  j.next = p1;
  j.cam0 = cam0;
  j.cam1 = cam1;
}

void Tracker::match_run(MatchJob *jobs, int nj) {
  Bufs &b = *b_;
  LkSlots lk{};
  RansacSlots rs{};
  int ns = 0, lo = kMaxCams, hi = -1;
  for (int k = 0; k < nj; k++) {
    const MatchJob &j = jobs[k];
    if (!j.run) continue;
    const int sl = j.slot;
    lo = std::min(lo, sl);
    hi = std::max(hi, sl);
    lk.prev[ns] = j.prev;
    lk.next[ns] = j.next;
    lk.p0[ns] = b.p0[sl];
    lk.p1[ns] = b.p1[sl];
    lk.st[ns] = b.st[sl];
    lk.n[ns] = j.n;
    const CamParams &c0 = cams_[j.cam0], &c1 = cams_[j.cam1];
    const double fmax = std::max(std::max(c0.v[0], c0.v[1]), std::max(c1.v[0], c1.v[1]));
    const double thr = 2.0 / fmax;
    rs.c0[ns] = c0;
    rs.c1[ns] = c1;
    lk.c0[ns] = c0;
    lk.c1[ns] = c1;
    lk.p0n[ns] = b.p0n[sl];
    lk.p1n[ns] = b.p1n[sl];
    lk.p1amb[ns] = b.amb[sl];
    rs.p0[ns] = b.p0[sl];
    rs.p1[ns] = b.p1[sl];
    rs.p0n[ns] = b.p0n[sl];
    rs.p1n[ns] = b.p1n[sl];
    rs.sub[ns] = b.sub[sl];
    rs.F[ns] = b.F[sl];
    rs.nm[ns] = b.nm[sl];
    rs.good[ns] = b.good[sl];
    rs.mask[ns] = b.mask[sl];
    rs.t[ns] = (float)(thr * thr);
    rs.n[ns] = j.n;
    ns++;
  }
  if (ns == 0) return;
  {
    HostProfScope hs(*hp_, "trk.upload");
    upload(b.p0[lo], b.hp(b.p0[lo]), span(b.p0[lo], b.sub[hi] + 7 * kRansacIters));
  }
  {
    HostProfScope hs(*hp_, "trk.pyr");
    ensure_pyr();
  }
  lk.undistort = 1;  // RANSAC's undistortion in the LK epilogue (one launch less on the frame's critical path)
  lk.bytes = (kp_ && kp_->on) ? d_lk_bytes_ : nullptr;
  {
    KScope ks(kp_, KC_LK);
    launch_lk(s_, lk, ns, win_, pyr_levels_, kLkIters, kLkEps, true);
  }
  launch_ransac(s_, rs, ns, kRansacIters, kRansacConf, lk.undistort != 0);
  HP_HIP(hipMemcpyAsync(b.hp(b.p1[lo]), b.p1[lo], span(b.p1[lo], b.p1n[hi] + 2 * b.cap), hipMemcpyDeviceToHost, s_));
  if (in_flight_) {
    // wait for the matching results only, not for the work the callback enqueues behind them
    if (!ev_match_) HP_HIP(hipEventCreateWithFlags(&ev_match_, hipEventDisableTiming));
    HP_HIP(hipEventRecord(ev_match_, s_));
    std::function<void()> f = std::move(in_flight_);
    in_flight_ = nullptr;
    f();
    auto t0 = std::chrono::steady_clock::now();
    for (hipError_t e; (e = hipEventQuery(ev_match_)) != hipSuccess;) {  // spin (see spin_sync)
      if (e != hipErrorNotReady) throw HpError(UVIO_HP_E_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e));
      __builtin_ia32_pause();
    }
    sync_wait += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    device_syncs++;
    return;
  }
  sync();
}

// The database's normalized coordinates of tracked point i of a matching slot: RANSAC's undistortion of the same
// float LK result (LK's epilogue runs cam_undistort_f, read back with the results).  The radial-tangential
// model's arithmetic is the same on both sides; the equidistant model's tan may differ by an ulp on the device,
// which changes the float result only near a float rounding boundary: those points (flagged by the device,
// a few in 10^5) are undistorted here with the host's libm, so the database holds the host's floats.
void Tracker::tracked_undistort(int slot, int i, int cam, const KeyPt &k, float &un, float &vn) const {
  if (cams_[cam].model == 0 || !b_->hp(b_->amb[slot])[i]) {
    const float *h = b_->hp(b_->p1n[slot]);
    un = h[2 * i];
    vn = h[2 * i + 1];
  } else {
    cam_undistort_f(cams_[cam], k.x, k.y, un, vn);
  }
}

void Tracker::match_collect(int slot, const MatchJob &j, std::vector<KeyPt> &k1, std::vector<uint8_t> &mask_out) {
  mask_out.clear();
  if (j.n == 0) return;
  if (!j.run) {
    mask_out.assign(j.n, 0);
    return;
  }
  Bufs &b = *b_;
  mask_out.resize(j.n);
  const float *h_p1 = b.hp(b.p1[slot]);
  const uint8_t *h_st = b.hp(b.st[slot]), *h_mask = b.hp(b.mask[slot]);
  for (int i = 0; i < j.n; i++) {
    k1[i].x = h_p1[2 * i];
    k1[i].y = h_p1[2 * i + 1];
    mask_out[i] = (h_st[i] && h_mask[i]) ? 1 : 0;
  }
}

// ---------------------------------------------------------------- per-frame logic
// TrackKLT::feed_monocular (TrackKLT.cpp:96-200) of the n cameras of one feed.  The reference runs the
// cameras' feed_monocular side by side (TrackKLT.cpp:85-89, parallel_for_ over the images, one atomic
// currid); here their detections share one device griding, their temporal matchings one LK + RANSAC launch
// pair and one readback, and the ids and database inserts follow the camera order -- the schedule in
// which the cameras run one after the other (the reference's threads may interleave the ids of
// different cameras; any interleaving is a valid run of it).
void Tracker::feed_multi(double t, const int *cams, int n, const DbSink &db) {
  std::vector<MonoDet> det(n);
  std::vector<bool> first(n);
  for (int k = 0; k < n; k++) {
    CamState &c = cs_[cams[k]];
    first[k] = c.pts_last.empty();
    det[k].cam = cams[k];
    if (first[k]) {  // no tracks yet: detect on this frame and keep them
      det[k].p = &c.pyr[1 - c.last];
      det[k].mask = &c.mask_new;
    } else {
      det[k].p = &c.pyr[c.last];
      det[k].mask = &c.mask_last;
      det[k].pts = c.pts_last;
      det[k].ids = c.ids_last;
    }
  }
  for (int k = 0; k < n; k++)
    if (first[k]) ensure_pyr();  // detection on this frame's images
  if (pre_.valid) {  // run ahead by predetect (every camera had tracks, so none is first)
    for (int k = 0; k < n; k++) {
      det[k].pts.swap(pre_.pts[k]);
      det[k].ids.swap(pre_.ids[k]);
    }
    pre_.valid = false;
  } else {
    detect_mono_multi(det.data(), n);
  }
  std::vector<MatchJob> jobs;
  std::vector<int> who;
  size_t most = 0;
  for (int k = 0; k < n; k++) {
    CamState &c = cs_[cams[k]];
    if (first[k]) {
      c.pts_last = det[k].pts;
      c.ids_last = det[k].ids;
      continue;
    }
    most = std::max(most, det[k].pts.size());
    who.push_back(k);
  }
  if (who.empty()) return;
  ensure_cap((int)most);  // no reallocation between the slots
  jobs.resize(who.size());
  for (size_t j = 0; j < who.size(); j++) {
    CamState &c = cs_[cams[who[j]]];
    match_prepare((int)j, c.pyr[c.last], c.pyr[1 - c.last], cams[who[j]], cams[who[j]], det[who[j]].pts, jobs[j]);
  }
  match_run(jobs.data(), (int)jobs.size());
  for (size_t j = 0; j < who.size(); j++) {
    const int k = who[j], cam = cams[k];
    CamState &c = cs_[cam];
    const DPyr &pn = c.pyr[1 - c.last];
    std::vector<KeyPt> pts_new = det[k].pts;
    std::vector<uint8_t> mask_ll;
    match_collect((int)j, jobs[j], pts_new, mask_ll);
    if (mask_ll.empty()) {
      c.pts_last.clear();
      c.ids_last.clear();
      continue;
    }
    const int W = pn.w[0], H = pn.h[0];
    std::vector<KeyPt> good;
    std::vector<size_t> gid;
    std::vector<int> gsrc;
    for (size_t i = 0; i < pts_new.size(); i++) {
      if (pts_new[i].x < 0 || pts_new[i].y < 0 || (int)pts_new[i].x >= W || (int)pts_new[i].y >= H) continue;
      if (mask_px(c.mask_new, W, (int)pts_new[i].x, (int)pts_new[i].y) > 127) continue;
      if (mask_ll[i]) {
        good.push_back(pts_new[i]);
        gid.push_back(det[k].ids[i]);
        gsrc.push_back((int)i);
      }
    }
    std::vector<float> nu(2 * good.size());
    auto undist = [&](size_t b, size_t e) {
      for (size_t i = b; i < e; i++) tracked_undistort((int)j, gsrc[i], cam, good[i], nu[2 * i], nu[2 * i + 1]);
    };
    undist(0, good.size());  // reads of the device's results (a host undistortion is rare, see tracked_undistort)
    for (size_t i = 0; i < good.size(); i++) db(gid[i], t, cam, good[i].x, good[i].y, nu[2 * i], nu[2 * i + 1]);
    c.pts_last.swap(good);
    c.ids_last.swap(gid);
  }
}

// TrackKLT::feed_stereo (TrackKLT.cpp:202-393)
void Tracker::feed_stereo(double t, int cl, int cr, const DbSink &db) {
  CamState &A = cs_[cl], &B = cs_[cr];
  const DPyr &nl = A.pyr[1 - A.last], &nr = B.pyr[1 - B.last];
  const DPyr &ll = A.pyr[A.last], &lr = B.pyr[B.last];
  if (A.pts_last.empty() && B.pts_last.empty()) {
    ensure_pyr();  // detection on this frame's images
    std::vector<KeyPt> gl, gr;
    std::vector<size_t> il, ir;
    detect_stereo(cl, cr, nl, nr, A.mask_new, B.mask_new, gl, gr, il, ir);
    A.pts_last = gl;
    B.pts_last = gr;
    A.ids_last = il;
    B.ids_last = ir;
    return;
  }
  std::vector<KeyPt> pl_old, pr_old;
  std::vector<size_t> il_old, ir_old;
  if (pre_.valid) {  // run ahead by predetect
    pl_old.swap(pre_.pts[0]);
    pr_old.swap(pre_.pts[1]);
    il_old.swap(pre_.ids[0]);
    ir_old.swap(pre_.ids[1]);
    pre_.valid = false;
  } else {
    pl_old = A.pts_last;
    pr_old = B.pts_last;
    il_old = A.ids_last;
    ir_old = B.ids_last;
    HostProfScope hs(*hp_, "trk.detect");
    detect_stereo(cl, cr, ll, lr, A.mask_last, B.mask_last, pl_old, pr_old, il_old, ir_old);
  }
  MatchJob jm[2];
  {
    HostProfScope hs(*hp_, "trk.prep");
    ensure_cap((int)std::max(pl_old.size(), pr_old.size()));  // no reallocation between the two slots
    match_prepare(0, ll, nl, cl, cl, pl_old, jm[0]);
    match_prepare(1, lr, nr, cr, cr, pr_old, jm[1]);
  }
  {
    HostProfScope hs(*hp_, "trk.match");
    match_run(jm, 2);
  }
  HostProfScope hs_post(*hp_, "trk.post");
  const MatchJob &jl = jm[0], &jr = jm[1];
  std::vector<KeyPt> pl_new = pl_old, pr_new = pr_old;
  std::vector<uint8_t> mask_ll, mask_rr;
  match_collect(0, jl, pl_new, mask_ll);
  match_collect(1, jr, pr_new, mask_rr);
  if (mask_ll.empty() && mask_rr.empty()) {
    A.pts_last.clear();
    B.pts_last.clear();
    A.ids_last.clear();
    B.ids_last.clear();
    return;
  }
  const int Wl = nl.w[0], Hl = nl.h[0], Wr = nr.w[0], Hr = nr.h[0];
  std::vector<KeyPt> gl, gr;
  std::vector<size_t> gil, gir;
  std::vector<int> sl, sr;  // each kept point's index in its matching slot
  // first index of each id among the right points (the reference's linear search returns the first)
  IdTable first_r(ir_old.size());
  for (size_t n = 0; n < ir_old.size(); n++) first_r.emplace(ir_old[n], n);
  for (size_t i = 0; i < pl_new.size(); i++) {
    if (pl_new[i].x < 0 || pl_new[i].y < 0 || (int)pl_new[i].x > Wl || (int)pl_new[i].y > Hl) continue;
    const size_t *fr = first_r.find(il_old[i]);
    const bool found = fr != nullptr;
    const size_t ir = found ? *fr : 0;
    if (mask_ll[i] && found && mask_rr[ir]) {
      if (pr_new[ir].x < 0 || pr_new[ir].y < 0 || (int)pr_new[ir].x >= Wr || (int)pr_new[ir].y >= Hr) continue;
      gl.push_back(pl_new[i]);
      gr.push_back(pr_new[ir]);
      gil.push_back(il_old[i]);
      gir.push_back(ir_old[ir]);
      sl.push_back((int)i);
      sr.push_back((int)ir);
    } else if (mask_ll[i]) {
      gl.push_back(pl_new[i]);
      gil.push_back(il_old[i]);
      sl.push_back((int)i);
    }
  }
  IdTable in_gir(gir.size() + pr_new.size());  // membership in gir, kept in step with it
  for (size_t id : gir) in_gir.emplace(id, 0);
  for (size_t i = 0; i < pr_new.size(); i++) {
    if (pr_new[i].x < 0 || pr_new[i].y < 0 || (int)pr_new[i].x >= Wr || (int)pr_new[i].y >= Hr) continue;
    const bool added = in_gir.contains(ir_old[i]);
    if (mask_rr[i] && !added) {
      gr.push_back(pr_new[i]);
      gir.push_back(ir_old[i]);
      sr.push_back((int)i);
      in_gir.emplace(ir_old[i], 0);
    }
  }
  // the device's undistortions (a host one is rare, see tracked_undistort); the database inserts keep their order
  std::vector<float> uvl(2 * gl.size()), uvr(2 * gr.size());
  auto undist = [&](size_t b, size_t e) {
    for (size_t i = b; i < e; i++) {
      if (i < gl.size())
        tracked_undistort(0, sl[i], cl, gl[i], uvl[2 * i], uvl[2 * i + 1]);
      else
        tracked_undistort(1, sr[i - gl.size()], cr, gr[i - gl.size()], uvr[2 * (i - gl.size())], uvr[2 * (i - gl.size()) + 1]);
    }
  };
  {
    HostProfScope hs(*hp_, "trk.post.undist");
    undist(0, gl.size() + gr.size());
  }
  HostProfScope hs_db(*hp_, "trk.post.db");
  for (size_t i = 0; i < gl.size(); i++) db(gil[i], t, cl, gl[i].x, gl[i].y, uvl[2 * i], uvl[2 * i + 1]);
  for (size_t i = 0; i < gr.size(); i++) db(gir[i], t, cr, gr[i].x, gr[i].y, uvr[2 * i], uvr[2 * i + 1]);
  A.pts_last.swap(gl);
  B.pts_last.swap(gr);
  A.ids_last.swap(gil);
  B.ids_last.swap(gir);
}

// The next feed's perform_detection_* on the last pyramids / points / masks (see tracker.h), on the detection
// stream.  Only when every camera of the last feed has tracks: a camera without tracks detects on the NEW
// frame's pyramid (TrackKLT.cpp:104-110, 215-222), which does not exist yet.
void Tracker::predetect() {
  const bool pyr_waited = pre_pyr_waited_;
  pre_pyr_waited_ = false;
  pre_syncs = 0;
  pre_wait = 0.0;
  if (pre_.valid || last_cams_.empty()) return;
  const int n = (int)last_cams_.size();
  const bool stereo = n == 2 && use_stereo_;
  // cs_.at: the engine's thread may read the map (last_tracks) while this runs on the worker
  if (stereo) {
    if (cs_.at(last_cams_[0]).pts_last.empty() && cs_.at(last_cams_[1]).pts_last.empty()) return;
  } else {
    for (int c : last_cams_)
      if (cs_.at(c).pts_last.empty()) return;
  }
  make_detect_stream();
  // the wait on the last pyramid launch: enqueued by predetect_async on the caller's thread (before the worker
  // starts, so the next feed's re-record of ev_pyr_ cannot come first); here when called synchronously
  if (!pyr_waited && ev_pyr_) HP_HIP(hipStreamWaitEvent(sd_, ev_pyr_, 0));
  kp_pre_.stream = sd_;
  kp_pre_.on = kp_ && kp_->on;
  kp_pre_.harvest(false);
  pre_.currid0 = currid;
  pre_.cams = last_cams_;
  pre_.pts.assign(n, {});
  pre_.ids.assign(n, {});
  cur_ = sd_;
  pre_mode_ = true;
  try {
    if (stereo) {
      CamState &A = cs_.at(last_cams_[0]), &B = cs_.at(last_cams_[1]);
      pre_.pts[0] = A.pts_last;
      pre_.pts[1] = B.pts_last;
      pre_.ids[0] = A.ids_last;
      pre_.ids[1] = B.ids_last;
      detect_stereo(last_cams_[0], last_cams_[1], A.pyr[A.last], B.pyr[B.last], A.mask_last, B.mask_last, pre_.pts[0],
                    pre_.pts[1], pre_.ids[0], pre_.ids[1]);
    } else {
      std::vector<MonoDet> det(n);
      for (int k = 0; k < n; k++) {
        CamState &c = cs_.at(last_cams_[k]);
        det[k].cam = last_cams_[k];
        det[k].p = &c.pyr[c.last];
        det[k].mask = &c.mask_last;
        det[k].pts = c.pts_last;
        det[k].ids = c.ids_last;
      }
      detect_mono_multi(det.data(), n);
      for (int k = 0; k < n; k++) {
        pre_.pts[k].swap(det[k].pts);
        pre_.ids[k].swap(det[k].ids);
      }
    }
  } catch (...) {
    cur_ = s_;
    pre_mode_ = false;
    currid = pre_.currid0;
    throw;
  }
  cur_ = s_;
  pre_mode_ = false;
  pre_.valid = true;
}

void Tracker::worker_loop() {
  std::unique_lock<std::mutex> lk(wm_);
  for (;;) {
    wcv_.wait(lk, [&] { return w_task_ || w_quit_; });
    if (w_quit_) return;
    w_task_ = false;
    w_busy_ = true;
    lk.unlock();
    try {
      // HIP's current device is per thread: bind the engine's before any HIP call of this task
      HP_HIP(hipSetDevice(dev_));
      predetect();
    } catch (...) {
      w_err_ = std::current_exception();
    }
    lk.lock();
    w_busy_ = false;
    wcv_.notify_all();
  }
}

// The detection stream (created on first use).  Measured and dropped (gpurun_out/cum): restricting it to a CU subset
// (hipExtStreamCreateWithCUMask, half / 7 of 8 / every other CU) left cfg3 within the run-to-run spread.
void Tracker::make_detect_stream() {
  if (!sd_) HP_HIP(hipStreamCreateWithFlags(&sd_, hipStreamNonBlocking));
}

void Tracker::predetect_async() {
  predetect_join();
  HP_HIP(hipGetDevice(&dev_));  // the engine's device (bound by the calling C-ABI entry)
  make_detect_stream();
  if (ev_pyr_) HP_HIP(hipStreamWaitEvent(sd_, ev_pyr_, 0));
  pre_pyr_waited_ = true;
  if (!worker_.joinable()) worker_ = std::thread([this] { worker_loop(); });
  {
    std::lock_guard<std::mutex> lk(wm_);
    w_task_ = true;
  }
  wcv_.notify_all();
}

const KProf &Tracker::pre_prof() {
  predetect_join();
  if (sd_) {
    HP_HIP(hipStreamSynchronize(sd_));
    kp_pre_.harvest(true);
  }
  return kp_pre_;
}

void Tracker::predetect_join() {
  if (!worker_.joinable()) return;
  std::exception_ptr e;
  {
    std::unique_lock<std::mutex> lk(wm_);
    wcv_.wait(lk, [&] { return !w_task_ && !w_busy_; });
    e = w_err_;
    w_err_ = nullptr;
  }
  if (e) std::rethrow_exception(e);
}

// ---------------------------------------------------------------- inspection
void Tracker::last_tracks(int cam, std::vector<KeyPt> &pts, std::vector<size_t> &ids) const {
  pts.clear();
  ids.clear();
  auto it = cs_.find(cam);
  if (it == cs_.end()) return;
  pts = it->second.pts_last;
  ids = it->second.ids_last;
}

bool Tracker::last_pyramid(int cam, int level, int *w, int *h, std::vector<uint8_t> *img, std::vector<int16_t> *der) {
  predetect_join();  // its sync() must see the tracker's own stream selection
  auto it = cs_.find(cam);
  if (it == cs_.end() || !it->second.have_last) return false;
  const DPyr &p = it->second.pyr[it->second.last];
  if (level < 0 || level >= p.levels) return false;
  *w = p.w[level];
  *h = p.h[level];
  sync();
  if (img) {
    img->resize((size_t)*w * *h);
    HP_HIP(hipMemcpy(img->data(), p.img[level], img->size(), hipMemcpyDeviceToHost));
  }
  if (der) {
    der->resize((size_t)*w * *h * 2);
    HP_HIP(hipMemcpy(der->data(), p.der[level], der->size() * sizeof(int16_t), hipMemcpyDeviceToHost));
  }
  return true;
}

}  // namespace uvhp
