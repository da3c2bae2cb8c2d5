// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_core/src/feat/Feature.{h,cpp} (:26-111), FeatureDatabase.cpp (:59-263) and
// FeatureInitializer.cpp (:30-423). libstdc++ unordered_map is used on purpose so that the
// per-camera iteration order (anchor choice, Jacobian column order) matches the reference.
#pragma once
#include <unordered_map>
#include <vector>

#include "state.h"

namespace orc {

struct Feature {
  size_t featid = 0;
  bool to_delete = false;
  std::unordered_map<size_t, std::vector<std::pair<float, float>>> uvs;
  std::unordered_map<size_t, std::vector<std::pair<float, float>>> uvs_norm;
  std::unordered_map<size_t, std::vector<double>> timestamps;
  int anchor_cam_id = -1;
  double anchor_clone_timestamp = -1;
  Mat p_FinA = Mat(3, 1), p_FinG = Mat(3, 1);

  void clean_old_measurements(const std::vector<double> &valid_times);
  void clean_older_measurements(double timestamp);
};
using FeatP = std::shared_ptr<Feature>;

struct FeatureDatabase {
  std::unordered_map<size_t, FeatP> features_idlookup;
  FeatP get_feature(size_t id) {
    auto it = features_idlookup.find(id);
    return it == features_idlookup.end() ? nullptr : it->second;
  }
  void update_feature(size_t id, double t, size_t cam, float u, float v, float un, float vn);
  std::vector<FeatP> features_not_containing_newer(double t, bool remove, bool skip_deleted);
  std::vector<FeatP> features_containing(double t, bool remove, bool skip_deleted);
  void cleanup();
  void cleanup_measurements(double t);
};

struct ClonePose {
  Mat R, p;  // R_GtoCi, p_CiinG
};
using ClonesCam = std::unordered_map<size_t, std::unordered_map<double, ClonePose>>;

struct FeatureInitializer {
  uvio_hp_options_t o;
  explicit FeatureInitializer(const uvio_hp_options_t &opt) : o(opt) {}
  bool single_triangulation(Feature &f, ClonesCam &c);
  bool single_triangulation_1d(Feature &f, ClonesCam &c);
  bool single_gaussnewton(Feature &f, ClonesCam &c);
  double compute_error(ClonesCam &c, Feature &f, double alpha, double beta, double rho);
};

}  // namespace orc
