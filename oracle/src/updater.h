// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_msckf/src/update/UpdaterHelper.cpp:32-487, UpdaterMSCKF.cpp:58-295,
// UpdaterSLAM.cpp:61-647 and uvio/src/update/{UpdaterUWB.cpp:13-90, UVioUpdaterHelper.cpp:147-241}.
#pragma once
#include <map>

#include "feat.h"

namespace orc {

struct HelperFeature {
  size_t featid;
  const Feature *f;  // uvs / uvs_norm / timestamps (copies in the reference; same iteration order)
  int rep;
  int anchor_cam_id = -1;
  double anchor_clone_timestamp = -1;
  Mat p_FinA = Mat(3, 1), p_FinA_fej = Mat(3, 1), p_FinG = Mat(3, 1), p_FinG_fej = Mat(3, 1);
};

namespace UpdaterHelper {
void get_feature_jacobian_representation(State &s, HelperFeature &f, Mat &H_f, std::vector<Mat> &H_x,
                                         std::vector<Ref> &x_order);
void get_feature_jacobian_full(State &s, HelperFeature &f, Mat &H_f, Mat &H_x, Mat &res, std::vector<Ref> &x_order);
void nullspace_project_inplace(Mat &H_f, Mat &H_x, Mat &res);
void measurement_compress_inplace(Mat &H_x, Mat &res);
}  // namespace UpdaterHelper

struct FeatDebug {
  size_t id;
  double p_FinG[3];
  int status;  // 0 accepted, 1 triangulation / refine failed, 3 chi2 rejected
  double chi2;
};
struct UpdateStats {
  int rows_stacked = 0, cols = 0, accepted = 0, rows_compressed = 0;
  std::vector<FeatDebug> feats;
};

// Lock-step steering (flip.h).  The tests hand the oracle the device's per-feature results of the frame it
// is about to process (targets, keyed by updater kind and feature id).  Where the oracle's triangulation /
// refinement (stage 0) or its chi2 (stage 1) disagree with the target beyond the strict parity bounds, the
// stage is re-run with one near-tie float cast rounded the other way, smallest margin first, until it
// agrees; the event (cast index, its margin, the disagreement before / after) is logged.  A disagreement
// that no single cast explains is logged with found = 0 and the oracle's own result is kept.
struct SteerTarget {
  int status;
  double p_FinG[3];
  double chi2;
};
struct SteerEvent {
  int kind;       // 0 MSCKF update, 1 SLAM update, 2 delayed initialization
  size_t featid;
  int stage;      // 0 triangulation + refinement, 1 Jacobian / chi2
  long index;     // the cast rounded the other way (-1: none found)
  double margin;  // its relative distance to the float rounding midpoint
  double before;  // disagreement with the device before / after
  double after;
  int found;
  int candidates; // near-tie casts tried
};
struct FrameDebug {
  std::vector<std::pair<int, FeatDebug>> feats;  // this frame's per-feature results (kind, result)
  bool steer = false;
  std::map<std::pair<int, size_t>, SteerTarget> targets;
  std::vector<SteerEvent> log;
  void record(int kind, const FeatDebug &d) { feats.push_back({kind, d}); }
  const SteerTarget *target(int kind, size_t id) const {
    if (!steer) return nullptr;
    auto it = targets.find({kind, id});
    return it == targets.end() ? nullptr : &it->second;
  }
};

struct UpdaterMSCKF {
  double sigma_pix_sq, chi2_mult;
  std::map<int, double> chi_squared_table;
  FeatureInitializer init;
  FrameDebug *dbg = nullptr;
  UpdaterMSCKF(const uvio_hp_options_t &o);
  // returns <0 on fatal numeric error
  int update(State &s, std::vector<FeatP> &feature_vec, UpdateStats *st = nullptr);
};

struct UpdaterSLAM {
  double sigma_pix_sq, chi2_mult;
  std::map<int, double> chi_squared_table;
  FeatureInitializer init;
  FrameDebug *dbg = nullptr;
  UpdaterSLAM(const uvio_hp_options_t &o);
  int delayed_init(State &s, std::vector<FeatP> &feature_vec);
  int update(State &s, std::vector<FeatP> &feature_vec);
  int change_anchors(State &s);  // landmarks re-anchored (>= 0), < 0 on a numeric error
  int perform_anchor_change(State &s, VarP landmark, double new_anchor_timestamp, size_t new_cam_id);
};

void uwb_jacobian_single(State &s, const VarP &anchor, double range, Mat &res, Mat &H_x, std::vector<Ref> &x_order);

struct UpdaterUWB {
  double sigma_range, chi2_mult;
  std::map<int, double> chi_squared_table;
  UpdaterUWB(const uvio_hp_options_t &o);
  // returns 1 if applied, 0 if gated, <0 on fatal error
  int update_single(State &s, double timestamp, size_t anchor_id, double range);
};

}  // namespace orc
