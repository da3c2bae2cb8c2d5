// ORACLE — test infrastructure only (see la.h header).
// CPU restatement of the KLT front-end:
//   ov_core/src/track/TrackKLT.cpp:34-886 (feed_new_camera, feed_monocular, feed_stereo,
//   perform_detection_monocular/stereo, perform_matching) and Grider_GRID.h:74-180, over the OpenCV
//   4.2 primitives it calls (not in /root/reference; restated from SURVEY.md Appendix A and the
//   published OpenCV algorithms):
//     equalizeHist, buildOpticalFlowPyramid (pyrDown + Scharr), FAST-9 (+NMS), cornerSubPix,
//     calcOpticalFlowPyrLK, findFundamentalMat(FM_RANSAC) with cv::RNG((uint64)-1).
// Parity of this front-end against OpenCV itself is unpinned (no OpenCV here); the product's GPU
// kernels are checked against this restatement.
//   * Equal FAST responses: Grider_GRID.h:128 sorts each cell's cv::FAST output (raster order, fast.cpp
//     pushes row by row, x ascending) with std::sort and the response-only Grider_FAST::compare_response.
//     std::sort is not stable, and its tie order IS observable (it decides which corners a cell keeps and
//     so every ++currid of TrackKLT.cpp:483-520): grid_sort calls libstdc++'s std::sort itself on the same
//     sequence (introsort, _S_threshold 16, median-of-three, unguarded partition, heap-sort fallback at
//     depth 2 lg n; the same algorithm in the GCC 7-13 libstdc++ the reference's ROS distributions ship).
//     Rounds 1-5 used the stable order here and on the device; that was not the reference's.
//   * LK window sums: OpenCV's calcOpticalFlowPyrLK (lkpyramid.cpp) accumulates the iteration's b-vector
//     (ib1, ib2) in float and the products come from CV_DESCALE'd integers.  This restatement takes the
//     sums as exact integers; the two agree whenever every partial float sum is exactly representable
//     (|sum| < 2^24), which a 15x15 window of 8-bit/Scharr products can exceed.  Not checkable here
//     (OpenCV is absent): this choice is unpinned, and the device follows it.
#pragma once
#include <functional>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "cam.h"

namespace orc {

struct GrayImg {
  int w = 0, h = 0;
  std::vector<uint8_t> d;
  uint8_t at(int x, int y) const { return d[(size_t)y * w + x]; }
};

struct Pyramid {
  std::vector<GrayImg> img;                 // levels 0..L
  std::vector<std::vector<int16_t>> deriv;  // per level, interleaved (dx, dy), w*h*2
  int levels() const { return (int)img.size(); }
};

struct KeyPt {
  float x, y, response;
};

// cv::equalizeHist
GrayImg equalize_hist(const GrayImg &src);
// cv::pyrDown (5x5 Gaussian, BORDER_REFLECT_101, dst ((w+1)/2, (h+1)/2))
GrayImg pyr_down(const GrayImg &src);
// calcSharrDeriv: interleaved (dx, dy) int16 per pixel, BORDER_REFLECT_101
std::vector<int16_t> scharr_deriv(const GrayImg &s);
// buildOpticalFlowPyramid(win, maxLevel, withDerivatives): stops when the next level side <= win
Pyramid build_pyramid(const GrayImg &img, int win, int max_level);
// cv::FAST(img(roi), thr, nonmax) — keypoints in ROI coordinates, raster order
std::vector<KeyPt> fast_roi(const GrayImg &img, int x0, int y0, int w, int h, int thr);
// std::sort(kp, Grider_FAST::compare_response) (Grider_GRID.h:128, Grider_FAST.h compare_response)
void grid_sort(std::vector<KeyPt> &kp);
// cv::cornerSubPix(win 5x5, zeroZone -1, 20 iterations, eps 1e-3)
void corner_subpix(const GrayImg &img, std::vector<KeyPt> &pts, int win, int max_iters, double eps);
// cv::calcOpticalFlowPyrLK(win, maxLevel, COUNT|EPS 30 / 0.01, OPTFLOW_USE_INITIAL_FLOW, minEig 1e-4)
// cv::parallel_for_ stand-in (tracker.cpp): thread count of the OpenCV calls, a parallel loop over [0, n)
void set_cv_threads(int k);
int cv_threads();
void cv_parallel_for(size_t n, const std::function<void(size_t, size_t)> &f);
void lk_track(const Pyramid &prev, const Pyramid &next, const std::vector<KeyPt> &p0, std::vector<KeyPt> &p1,
              std::vector<uint8_t> &status, int win, int max_level, int max_iters, float eps);
// cv::findFundamentalMat(FM_RANSAC, thr, 0.999) mask (7-point RANSAC, cv::RNG((uint64)-1))
void ransac_fundamental_mask(const std::vector<float> &x0, const std::vector<float> &y0, const std::vector<float> &x1,
                             const std::vector<float> &y1, double thr, double conf, int max_iters,
                             std::vector<uint8_t> &mask);
// RANSAC subsets exactly as RANSACPointSetRegistrator::getSubset draws them (used by the device too)
void ransac_subsets(int count, int max_iters, std::vector<int> &idx);
// 7-point fundamental matrices of one subset (<= 3, F(2,2) normalized to 1 when possible)
int fundamental_7pt(const double *x0, const double *y0, const double *x1, const double *y1, double *F);

struct FeatureDatabase;

// TrackKLT (TrackKLT.h:50): state per camera and the per-frame logic.
struct TrackKLT {
  int num_features = 25, threshold = 20, grid_x = 5, grid_y = 5, min_px_dist = 10;
  int histogram_method = 1;
  bool use_stereo = true;
  int pyr_levels = 5, win = 15;
  size_t currid = 1;
  std::unordered_map<size_t, Camera> *cams = nullptr;
  std::unordered_map<size_t, Pyramid> pyr_last;
  std::unordered_map<size_t, GrayImg> mask_last;
  std::unordered_map<size_t, std::vector<KeyPt>> pts_last;
  std::unordered_map<size_t, std::vector<size_t>> ids_last;

  // feed_new_camera: images[k] for cam_ids[k]; masks may be empty images (no mask)
  void feed(double t, const std::vector<int> &cam_ids, const std::vector<GrayImg> &images, const std::vector<GrayImg> &masks,
            FeatureDatabase &db);

  void feed_monocular(double t, int cam, const Pyramid &pyr, const GrayImg &mask, FeatureDatabase &db);
  void feed_stereo(double t, int cl, int cr, const Pyramid &pl, const Pyramid &pr, const GrayImg &ml, const GrayImg &mr,
                   FeatureDatabase &db);
  void perform_detection_monocular(const Pyramid &pyr, const GrayImg &mask, std::vector<KeyPt> &pts, std::vector<size_t> &ids);
  void perform_detection_stereo(const Pyramid &p0, const Pyramid &p1, const GrayImg &m0, const GrayImg &m1, int cl, int cr,
                                std::vector<KeyPt> &pts0, std::vector<KeyPt> &pts1, std::vector<size_t> &ids0,
                                std::vector<size_t> &ids1);
  void perform_griding(const GrayImg &img, const GrayImg &mask, const std::vector<std::pair<int, int>> &valid_locs,
                       std::vector<KeyPt> &pts);
  void perform_matching(const Pyramid &p0, const Pyramid &p1, std::vector<KeyPt> &k0, std::vector<KeyPt> &k1, int id0, int id1,
                        std::vector<uint8_t> &mask_out);
};

}  // namespace orc
