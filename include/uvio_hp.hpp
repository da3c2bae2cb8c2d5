/*
 * uvio_hp.hpp — header-only C++ facade over the C ABI (uvio_hp.h) with the reference's method names, for
 * a maintainer who swaps ov_msckf::VioManager / uvio::UVioManager and the Updater classes for the MI355X
 * path.  Plain standard-library types only (no Eigen / OpenCV / ROS): the ROS adapter converts its
 * cv::Mat / Eigen values at the call site.  Errors become uvio_amd::Error exceptions
 * carrying the status code and the library's message; the library itself never exits the process.
 *
 *   Manager                        <- VioManager (VioManager.h:75-114) + UVioManager (UVioManager.h:48-73)
 *   Manager::msckf_update          <- UpdaterMSCKF::update (UpdaterMSCKF.h:68)
 *   Manager::slam_update           <- UpdaterSLAM::update (UpdaterSLAM.h:70)
 *   Manager::slam_delayed_init     <- UpdaterSLAM::delayed_init (UpdaterSLAM.h:77)
 *   Manager::slam_change_anchors   <- UpdaterSLAM::change_anchors (UpdaterSLAM.h:87)
 *   Manager::uwb_update_single     <- UpdaterUWB::update_single (UpdaterUWB.h:55)
 *   Manager::propagate_and_clone   <- Propagator::propagate_and_clone (Propagator.h:110)
 */
#ifndef UVIO_HP_HPP
#define UVIO_HP_HPP

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "uvio_hp.h"

namespace uvio_amd {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// One 8-bit camera image (CV_8UC1 data pointer and row stride); mask optional (nullptr)
struct Image {
  const uint8_t *data = nullptr;
  int stride = 0;
  const uint8_t *mask = nullptr;
};

// ov_core::Feature as plain data: measurements in observation order
struct Feature {
  uint64_t featid = 0;
  std::vector<uvio_hp_feat_meas_t> meas;
};

class Manager {
 public:
  explicit Manager(const std::string &estimator_config_yaml, int device = 0) {
    uvio_hp_options_t o;
    check_static(uvio_hp_options_default(&o), "options_default");  // the load overlays the YAML's keys on these
    check_static(uvio_hp_options_load(estimator_config_yaml.c_str(), &o), "options_load " + estimator_config_yaml);
    create(o, device);
  }
  Manager(const uvio_hp_options_t &o, int device) { create(o, device); }
  ~Manager() {
    if (h_) uvio_hp_destroy(h_);
  }
  Manager(const Manager &) = delete;
  Manager &operator=(const Manager &) = delete;

  // ---- VioManager / UVioManager feeds ----
  void initialize_with_gt(const std::array<double, 17> &x) { check(uvio_hp_initialize_with_gt(h_, x.data())); }
  void feed_measurement_imu(double t, const std::array<double, 3> &wm, const std::array<double, 3> &am) {
    check(uvio_hp_feed_imu(h_, t, wm.data(), am.data()));
  }
  // a burst of samples (t[i], wm[i], am[i]) in one call
  void feed_measurement_imu(const std::vector<double> &t, const std::vector<std::array<double, 3>> &wm,
                            const std::vector<std::array<double, 3>> &am) {
    if (wm.size() != t.size() || am.size() != t.size()) throw Error(UVIO_HP_E_ARG, "feed_measurement_imu: size mismatch");
    check(uvio_hp_feed_imu_batch(h_, (int)t.size(), t.data(), wm.empty() ? nullptr : wm[0].data(),
                                 am.empty() ? nullptr : am[0].data()));
  }
  // TrackSIM input: per camera (feature id, raw uv); false before initialization (the reference returns silently)
  bool feed_measurement_simulation(double t, const std::vector<int> &camids,
                                   const std::vector<std::vector<std::pair<uint64_t, std::array<float, 2>>>> &feats) {
    std::vector<int> counts;
    std::vector<uint64_t> ids;
    std::vector<float> uv;
    for (const auto &fc : feats) {
      counts.push_back((int)fc.size());
      for (const auto &f : fc) {
        ids.push_back(f.first);
        uv.push_back(f.second[0]);
        uv.push_back(f.second[1]);
      }
    }
    return soft(uvio_hp_feed_simulation(h_, t, (int)camids.size(), camids.data(), counts.data(), ids.data(), uv.data()));
  }
  // CameraData: images (host memory, or device memory with on_device) per sensor id
  bool feed_measurement_camera(double t, const std::vector<int> &camids, const std::vector<Image> &images,
                               bool on_device = false) {
    std::vector<const uint8_t *> imgs, masks;
    std::vector<int> strides;
    bool any_mask = false;
    for (const auto &im : images) {
      imgs.push_back(im.data);
      strides.push_back(im.stride);
      masks.push_back(im.mask);
      any_mask |= im.mask != nullptr;
    }
    const uint8_t *const *mp = any_mask ? masks.data() : nullptr;
    const int rc = on_device ? uvio_hp_feed_camera_device(h_, t, (int)camids.size(), camids.data(), imgs.data(),
                                                          strides.data(), mp)
                             : uvio_hp_feed_camera(h_, t, (int)camids.size(), camids.data(), imgs.data(),
                                                   strides.data(), mp);
    return soft(rc);
  }
  void feed_measurement_uwb(double t, const std::vector<uint64_t> &anchor_ids, const std::vector<double> &ranges) {
    if (anchor_ids.size() != ranges.size()) throw Error(UVIO_HP_E_ARG, "feed_measurement_uwb: size mismatch");
    check(uvio_hp_feed_uwb(h_, t, (int)anchor_ids.size(), anchor_ids.data(), ranges.data()));
  }
  void try_to_initialize_uwb_anchors(const std::vector<uvio_hp_anchor_t> &anchors) {
    check(uvio_hp_init_anchors(h_, (int)anchors.size(), anchors.data()));
  }

  // ---- getters ----
  bool initialized() const {
    int v = 0;
    check(uvio_hp_initialized(h_, &v));
    return v != 0;
  }
  // [q_GtoI(4) p_IinG(3) v_IinG(3) bg(3) ba(3)] and the state time
  std::array<double, 16> imu_value(double *t = nullptr) const {
    std::array<double, 16> x{};
    double tt = 0;
    check(uvio_hp_get_imu_state(h_, &tt, x.data()));
    if (t) *t = tt;
    return x;
  }
  int cov_dim() const {
    int n = 0;
    check(uvio_hp_get_cov_dim(h_, &n));
    return n;
  }
  std::vector<double> covariance() const {  // row-major N x N
    const int n = cov_dim();
    std::vector<double> P((size_t)n * n);
    check(uvio_hp_get_cov(h_, P.data(), n));
    return P;
  }
  std::vector<double> state_vector() const {
    std::vector<double> x(8192);
    int len = 0, nv = 0;
    check(uvio_hp_get_state_vector(h_, x.data(), (int)x.size(), &len, nullptr, 0, &nv));
    x.resize(len);
    return x;
  }
  uvio_hp_timing_t timing() const {
    uvio_hp_timing_t t{};
    check(uvio_hp_get_timing(h_, &t));
    return t;
  }

  // ---- updater-level calls (uvio_hp.h "Updater-level boundary") ----
  void set_state(const std::vector<double> &val, const std::vector<double> &fej, const std::vector<double> &P) {
    const int n = cov_dim();
    if (val.size() != fej.size() || P.size() != (size_t)n * n) throw Error(UVIO_HP_E_ARG, "set_state: size mismatch");
    check(uvio_hp_set_state(h_, val.data(), fej.data(), (int)val.size(), P.data(), n, n));
  }
  void propagate_and_clone(double t) { check(uvio_hp_propagate_and_clone(h_, t)); }
  std::vector<uvio_hp_feat_result_t> msckf_update(const std::vector<Feature> &fv) {
    return updater(uvio_hp_msckf_update, fv);
  }
  std::vector<uvio_hp_feat_result_t> slam_update(const std::vector<Feature> &fv) {
    return updater(uvio_hp_slam_update, fv);
  }
  std::vector<uvio_hp_feat_result_t> slam_delayed_init(const std::vector<Feature> &fv) {
    return updater(uvio_hp_slam_delayed_init, fv);
  }
  void slam_change_anchors() { check(uvio_hp_slam_change_anchors(h_)); }
  void marginalize_slam() { check(uvio_hp_marginalize_slam(h_)); }
  void marginalize_old_clone() { check(uvio_hp_marginalize_old_clone(h_)); }
  bool uwb_update_single(double t, uint64_t anchor_id, double range) {
    int applied = 0;
    check(uvio_hp_uwb_update_single(h_, t, anchor_id, range, &applied));
    return applied != 0;
  }

  uvio_hp_t *handle() { return h_; }

 private:
  uvio_hp_t *h_ = nullptr;

  void create(const uvio_hp_options_t &o, int device) {
    const int rc = uvio_hp_create(&o, device, &h_);
    if (rc) {
      const char *m = uvio_hp_last_error(nullptr);
      throw Error(rc, std::string("uvio_hp_create: ") + (m ? m : ""));
    }
  }
  static void check_static(int rc, const std::string &what) {
    if (rc) throw Error(rc, what);
  }
  void check(int rc) const {
    if (rc) {
      const char *m = uvio_hp_last_error(h_);
      throw Error(rc, m ? m : "uvio_hp");
    }
  }
  // E_STATE before initialization: the reference's feeds return without doing anything
  bool soft(int rc) const {
    if (rc == UVIO_HP_E_STATE) return false;
    check(rc);
    return true;
  }
  template <class Fn>
  std::vector<uvio_hp_feat_result_t> updater(Fn fn, const std::vector<Feature> &fv) {
    std::vector<uint64_t> ids;
    std::vector<int> off{0};
    std::vector<uvio_hp_feat_meas_t> meas;
    for (const auto &f : fv) {
      ids.push_back(f.featid);
      meas.insert(meas.end(), f.meas.begin(), f.meas.end());
      off.push_back((int)meas.size());
    }
    std::vector<uvio_hp_feat_result_t> out(fv.size());
    check(fn(h_, (int)fv.size(), ids.data(), off.data(), meas.data(), out.data()));
    return out;
  }
};

}  // namespace uvio_amd

#endif  // UVIO_HP_HPP
