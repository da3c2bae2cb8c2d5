// KLT front-end host orchestration (ov_core::TrackKLT, TrackKLT.cpp:34-886; Grider_GRID.h:74-180).
//
// The per-pixel and per-point work runs on the device (kernels_track.hip); the host keeps what the
// reference keeps in TrackKLT's maps — the last points / ids / mask per camera — and makes the
// same decisions in the same order (grid occupancy, min-distance grid, id assignment, stereo
// bookkeeping), so the feature ids and their order in the database are the reference's.
// Pyramids stay in HBM: two slots per camera (last, new), swapped every frame.
#pragma once
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "hp_common.h"
#include "hprof.h"
#include "kernels.h"

namespace uvhp {

struct KeyPt {
  float x, y, response;
};

using DbSink = std::function<void(size_t id, double t, int cam, float u, float v, float un, float vn)>;

class Tracker {
 public:
  Tracker(const uvio_hp_options_t &o, const CamParams *cams, hipStream_t s, KProf *kp = nullptr);
  ~Tracker();
  Tracker(const Tracker &) = delete;
  Tracker &operator=(const Tracker &) = delete;

  // TrackKLT::feed_new_camera.  imgs: host (device_imgs false) or device u8 images of the
  // configured size with row stride strides[k]; masks: host u8, same stride, may be null.
  // in_flight (optional) runs once on the host while the frame's LK + RANSAC are on the device, before
  // the tracker waits for them: work behind it on the same stream overlaps nothing of the tracker's
  // results, only the host's wait
  void feed(double t, int ncam, const int *cam_ids, const uint8_t *const *imgs, const int *strides,
            const uint8_t *const *masks, bool device_imgs, const DbSink &db,
            std::function<void()> in_flight = nullptr);

  // TrackBase::get_last_obs / get_last_ids for one camera
  void last_tracks(int cam, std::vector<KeyPt> &pts, std::vector<size_t> &ids) const;
  // last pyramid level of one camera (img: w*h, der: w*h*2); returns false if absent
  bool last_pyramid(int cam, int level, int *w, int *h, std::vector<uint8_t> *img, std::vector<int16_t> *der);

  size_t currid;
  // TrackBase::set_num_features (TrackBase.h:152): after an initializer succeeds (VioManagerHelper.cpp:124)
  void set_num_features(int n);
  void set_host_prof(HostProf *p) { hp_ = p; }
  int device_syncs = 0;     // host waits in the last feed
  double sync_wait = 0.0;   // seconds blocked in them
  // LK algorithmic bytes accumulated on the device since creation (LkSlots::bytes), read on demand
  unsigned long long lk_bytes();
  // Grider_GRID cells FAST'ed since creation and how many of them had more than 16 candidates (std::sort's
  // introsort path, where its tie order differs from a stable one); joins the predetect, reads the device count
  void grid_stats(unsigned long long *cells, unsigned long long *introsort_cells);
  // The next feed's detection, run ahead.  TrackKLT::perform_detection_{monocular,stereo} reads only the
  // previous frame's pyramid, points, ids and mask (TrackKLT.cpp:130, 249: img_pyramid_last, pts_last,
  // ids_last, img_mask_last), so it can run as soon as a feed has ended -- on its own stream, while the device
  // works on that frame's updates (Engine::update_frame calls it before its wait).  The next feed uses the
  // result when it has the same cameras; otherwise, or after set_num_features, the result is discarded and
  // currid restored, so ids and points are always those of the serial order.
  void predetect();
  // predetect on the tracker's worker thread: returns at once; the next feed (or anything that needs the
  // tracker's detection state) joins it first, rethrowing its error
  void predetect_async();
  void predetect_join();
  int pre_syncs = 0;        // host waits / seconds of the last predetect (on its own thread: off the frame)
  double pre_wait = 0.0;
  // the kernel-class timing of the detection stream (the predetect's FAST / sub-pixel / stereo LK launches on
  // sd_, recorded from the worker thread): joins the predetect, waits for its stream, harvests every pair
  const KProf &pre_prof();

 private:
  struct CamState {
    DPyr pyr[2]{};
    void *pyr_mem[2] = {nullptr, nullptr};
    int last = 0;            // slot of pyr_last
    bool have_last = false;
    uint8_t *d_raw = nullptr;  // staging of a host image (the raw 2w x 2h one with downsample_cameras)
    uint8_t *d_half = nullptr;  // downsample_cameras: the pyrDown'ed input (w x h)
    unsigned *d_hist = nullptr;
    uint8_t *d_score = nullptr;  // FAST score map (w x h)
    std::vector<uint8_t> mask_last, mask_new;  // host masks (empty = none)
    std::vector<KeyPt> pts_last;
    std::vector<size_t> ids_last;
  };
  // one perform_matching in flight (slot 0 / 1)
  struct MatchJob {
    int n = 0, slot = 0, cam0 = 0, cam1 = 0;
    bool run = false;   // LK + RANSAC launched
    DPyr prev{}, next{};
  };
  struct Bufs;

  const CamParams *cams_;
  hipStream_t s_;
  KProf *kp_ = nullptr;
  KProf kp_pre_;  // the detection stream's event pairs (used by the worker thread while pre_mode_)
  KProf *kcur() { return pre_mode_ ? &kp_pre_ : kp_; }
  unsigned long long *d_lk_bytes_ = nullptr;
  int *d_sort_stats_ = nullptr;              // k_fast_select's count of introsort cells
  unsigned long long grid_cells_ = 0;        // cells launched (host count, the feeding or the worker thread)
  bool downsample_ = false;  // VioManager.cpp:270-278: the inputs are 2w x 2h and pyrDown'ed first
  int num_features_, threshold_, grid_x_, grid_y_, min_px_dist_, histogram_method_;
  bool use_stereo_;
  const int pyr_levels_ = 5, win_ = 15;
  std::unordered_map<int, CamState> cs_;
  std::vector<float> spmask_host_;
  Bufs *b_ = nullptr;
  std::unordered_map<int, std::vector<int>> subset_cache_;
  std::function<void()> in_flight_;
  hipEvent_t ev_match_ = nullptr;
  HostProf own_hp_;                // used when the engine does not share its own
  HostProf *hp_ = &own_hp_;        // the engine's section timer (UVIO_HP_HOST_PROF)
  // host-to-device uploads on their own stream: the DMA transfer overlaps the kernels queued before it (the
  // pyramid) instead of starting after them; s_ waits on ev_up_ before its next launch
  hipStream_t up_ = nullptr;
  hipEvent_t ev_up_ = nullptr;
  void upload(void *dst, const void *src, size_t bytes);
  // the frame's decimation + pyramid launches, deferred until the new pyramid is first needed: the detection on
  // the previous frame's pyramid and the upload of the matching inputs go out before it, so the upload's DMA
  // overlaps the pyramid kernels
  std::function<void()> pyr_launch_;
  void ensure_pyr() {
    if (!pyr_launch_) return;
    std::function<void()> f = std::move(pyr_launch_);
    pyr_launch_ = nullptr;
    f();
  }

  CamState &cam_state(int cid);
  void alloc_pyr(CamState &c, int w, int h);
  void ensure_cap(int n);
  void sync();
  void make_detect_stream();
  // detection stream state: the detection functions launch on cur_ (s_, or sd_ while predetect runs)
  hipStream_t sd_ = nullptr, cur_ = nullptr;
  bool pre_pyr_waited_ = false;  // predetect_async enqueued sd_'s wait on ev_pyr_ (the worker must not read it)
  hipEvent_t ev_pyr_ = nullptr;  // after the last pyramid launch on s_ (predetect reads that pyramid)
  bool pre_mode_ = false;
  struct PreDet {
    bool valid = false;
    std::vector<int> cams;
    size_t currid0 = 0;
    std::vector<std::vector<KeyPt>> pts;
    std::vector<std::vector<size_t>> ids;
  };
  PreDet pre_;
  std::vector<int> last_cams_;
  // the predetect worker: one persistent thread, one task at a time
  std::thread worker_;
  std::mutex wm_;
  std::condition_variable wcv_;
  bool w_task_ = false, w_busy_ = false, w_quit_ = false;
  int dev_ = 0;  // the engine's HIP device, bound on the worker before each task
  std::exception_ptr w_err_;
  void worker_loop();
  void discard_predetect() {
    if (pre_.valid) currid = pre_.currid0;
    pre_.valid = false;
  }
  const std::vector<int> &subsets(int count);

  // one Grider_GRID request: camera, pyramid, user mask, min-distance boxes, cells to fill -> corners
  struct GridReq {
    int cam;
    const DPyr *p;
    const std::vector<uint8_t> *user_mask;
    const std::vector<int> *boxes;
    std::vector<std::pair<int, int>> valid;
    std::vector<KeyPt> out;
  };
  struct MonoDet;

  void feed_multi(double t, const int *cams, int n, const DbSink &db);
  void feed_stereo(double t, int cl, int cr, const DbSink &db);
  void detect_mono_pre(MonoDet &m);
  void detect_mono_post(MonoDet &m);
  void detect_mono_multi(MonoDet *m, int n);
  void griding_multi(GridReq *reqs, int nr, const DPyr *lk_to, std::vector<KeyPt> *lk_pts, std::vector<uint8_t> *lk_st);
  void detect_stereo(int cl, int cr, const DPyr &p0, const DPyr &p1, const std::vector<uint8_t> &m0,
                     const std::vector<uint8_t> &m1, std::vector<KeyPt> &pts0, std::vector<KeyPt> &pts1,
                     std::vector<size_t> &ids0, std::vector<size_t> &ids1);
  // Grider_GRID::perform_griding + cornerSubPix; when lk_to is set also tracks the new points into
  // that pyramid (TrackKLT.cpp:640-655) and returns the results in lk_pts / lk_st.
  void griding(int cam, const DPyr &p, const std::vector<uint8_t> &user_mask, const std::vector<int> &rects,
               const std::vector<std::pair<int, int>> &valid, std::vector<KeyPt> &out, const DPyr *lk_to,
               std::vector<KeyPt> *lk_pts, std::vector<uint8_t> *lk_st);
  void match_prepare(int slot, const DPyr &p0, const DPyr &p1, int cam0, int cam1, const std::vector<KeyPt> &k0,
                     MatchJob &j);
  void match_run(MatchJob *jobs, int nj);
  void match_collect(int slot, const MatchJob &j, std::vector<KeyPt> &k1, std::vector<uint8_t> &mask_out);
  void tracked_undistort(int slot, int i, int cam, const KeyPt &k, float &un, float &vn) const;
};

}  // namespace uvhp
