// Options: defaults of the reference option structs and a loader for the reference YAML files.
//
// The reference parses with ov_core::YamlParser over cv::FileStorage (opencv_yaml_parse.h:65-163):
// parse_config reads keys of estimator_config.yaml, parse_external reads "relative_config_imu" /
// "relative_config_imucam" / "config_uwb" / "uwb_anchors" files relative to it.  The keys read
// here follow VioManagerOptions::print_and_load (VioManagerOptions.h:62-556), StateOptions
// (StateOptions.h:97-138) and UVioManagerOptions (UVioManagerOptions.h:44-112).  The YAML subset
// is the one those files use: "%YAML:1.0" header, "key: value", nested maps by indentation,
// inline lists "[a, b]" and block lists of inline rows ("- [a, b, c, d]").
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "hp_common.h"

namespace uvhp {

namespace {

struct YNode {
  std::string scalar;
  std::vector<std::string> list;               // inline list items
  std::vector<std::vector<std::string>> rows;  // block list of inline lists
  std::vector<std::pair<std::string, std::shared_ptr<YNode>>> map;
  YNode *get(const std::string &k) {
    for (auto &kv : map)
      if (kv.first == k) return kv.second.get();
    return nullptr;
  }
};

std::string trim(const std::string &s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

std::string strip_comment(const std::string &s) {
  bool in_q = false;
  char qc = 0;
  for (size_t i = 0; i < s.size(); i++) {
    char c = s[i];
    if ((c == '"' || c == '\'') && (!in_q || c == qc)) {
      in_q = !in_q;
      qc = c;
    }
    if (c == '#' && !in_q) return s.substr(0, i);
  }
  return s;
}

std::string unquote(std::string s) {
  s = trim(s);
  if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\'')))
    return s.substr(1, s.size() - 2);
  return s;
}

std::vector<std::string> parse_inline_list(const std::string &s) {
  std::vector<std::string> out;
  std::string body = trim(s);
  if (body.size() < 2) return out;
  body = body.substr(1, body.size() - 2);
  std::stringstream ss(body);
  std::string item;
  while (std::getline(ss, item, ',')) {
    item = unquote(item);
    if (!item.empty()) out.push_back(item);
  }
  return out;
}

struct YLine {
  int indent;
  std::string text;
};

// Parse lines[i..] at exactly `indent` into `node` (a map); returns the next unconsumed index.
size_t parse_block(const std::vector<YLine> &L, size_t i, int indent, YNode *node) {
  while (i < L.size() && L[i].indent >= indent) {
    if (L[i].indent > indent || L[i].text[0] == '-') {  // stray deeper line: skip
      i++;
      continue;
    }
    const std::string &t = L[i].text;
    size_t colon = t.find(':');
    if (colon == std::string::npos) {
      i++;
      continue;
    }
    auto child = std::make_shared<YNode>();
    node->map.push_back({trim(t.substr(0, colon)), child});
    std::string val = trim(t.substr(colon + 1));
    i++;
    if (!val.empty()) {
      if (val[0] == '[')
        child->list = parse_inline_list(val);
      else
        child->scalar = unquote(val);
      continue;
    }
    if (i < L.size() && L[i].text[0] == '-' && L[i].indent >= indent) {
      int li = L[i].indent;
      while (i < L.size() && L[i].indent == li && L[i].text[0] == '-') {
        std::string item = trim(L[i].text.substr(1));
        if (!item.empty() && item[0] == '[')
          child->rows.push_back(parse_inline_list(item));
        else
          child->list.push_back(unquote(item));
        i++;
      }
    } else if (i < L.size() && L[i].indent > indent) {
      i = parse_block(L, i, L[i].indent, child.get());
    }
  }
  return i;
}

std::shared_ptr<YNode> parse_yaml(const std::string &path, bool *ok) {
  *ok = false;
  std::ifstream f(path);
  if (!f) return nullptr;
  std::vector<YLine> lines;
  std::string raw;
  while (std::getline(f, raw)) {
    if (raw.rfind("%YAML", 0) == 0 || raw.rfind("---", 0) == 0) continue;
    std::string s = strip_comment(raw);
    if (trim(s).empty()) continue;
    int ind = 0;
    while (ind < (int)s.size() && (s[ind] == ' ' || s[ind] == '\t')) ind++;
    lines.push_back({ind, trim(s)});
  }
  auto root = std::make_shared<YNode>();
  size_t i = 0;
  while (i < lines.size()) {
    size_t j = parse_block(lines, i, lines[i].indent, root.get());
    i = (j == i) ? i + 1 : j;
  }
  *ok = true;
  return root;
}

bool to_bool(const std::string &s) {
  std::string t;
  for (char c : s) t += (char)std::tolower(c);
  return t == "true" || t == "1" || t == "yes" || t == "on";
}

struct Doc {
  std::shared_ptr<YNode> root;
  YNode *node(const std::vector<std::string> &path) {
    YNode *n = root.get();
    for (auto &k : path) {
      if (!n) return nullptr;
      n = n->get(k);
    }
    return n;
  }
  void get(const std::vector<std::string> &p, int &v) {
    YNode *n = node(p);
    if (n && !n->scalar.empty()) {
      const std::string &s = n->scalar;
      if (s == "true" || s == "false")
        v = to_bool(s);
      else
        v = (int)std::strtol(s.c_str(), nullptr, 10);
    }
  }
  void get(const std::vector<std::string> &p, double &v) {
    YNode *n = node(p);
    if (n && !n->scalar.empty()) v = std::strtod(n->scalar.c_str(), nullptr);
  }
  void getb(const std::vector<std::string> &p, int &v) {
    YNode *n = node(p);
    if (n && !n->scalar.empty()) v = to_bool(n->scalar) ? 1 : 0;
  }
  bool gets(const std::vector<std::string> &p, std::string &v) {
    YNode *n = node(p);
    if (n && !n->scalar.empty()) {
      v = n->scalar;
      return true;
    }
    return false;
  }
  bool getvec(const std::vector<std::string> &p, std::vector<double> &v) {
    YNode *n = node(p);
    if (!n || n->list.empty()) return false;
    v.clear();
    for (auto &s : n->list) v.push_back(std::strtod(s.c_str(), nullptr));
    return true;
  }
  bool getmat(const std::vector<std::string> &p, std::vector<std::vector<double>> &m) {
    YNode *n = node(p);
    if (!n || n->rows.empty()) return false;
    m.clear();
    for (auto &r : n->rows) {
      std::vector<double> row;
      for (auto &s : r) row.push_back(std::strtod(s.c_str(), nullptr));
      m.push_back(row);
    }
    return true;
  }
};

std::string dirname_of(const std::string &p) {
  size_t k = p.find_last_of('/');
  return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

int rep_from_string(const std::string &s) {
  static const char *names[] = {"GLOBAL_3D",
                                "GLOBAL_FULL_INVERSE_DEPTH",
                                "ANCHORED_3D",
                                "ANCHORED_FULL_INVERSE_DEPTH",
                                "ANCHORED_MSCKF_INVERSE_DEPTH",
                                "ANCHORED_INVERSE_DEPTH_SINGLE"};
  for (int i = 0; i < 6; i++)
    if (s == names[i]) return i;
  return -1;
}

// 3x3 inverse (Tw / Ta -> Dw / Da, VioManagerOptions.h:319-320)
bool inv3(const double A[9], double out[9]) {
  double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) + A[2] * (A[3] * A[7] - A[4] * A[6]);
  if (det == 0 || std::isnan(det)) return false;
  double id = 1.0 / det;
  out[0] = (A[4] * A[8] - A[5] * A[7]) * id;
  out[1] = (A[2] * A[7] - A[1] * A[8]) * id;
  out[2] = (A[1] * A[5] - A[2] * A[4]) * id;
  out[3] = (A[5] * A[6] - A[3] * A[8]) * id;
  out[4] = (A[0] * A[8] - A[2] * A[6]) * id;
  out[5] = (A[2] * A[3] - A[0] * A[5]) * id;
  out[6] = (A[3] * A[7] - A[4] * A[6]) * id;
  out[7] = (A[1] * A[6] - A[0] * A[7]) * id;
  out[8] = (A[0] * A[4] - A[1] * A[3]) * id;
  return true;
}

}  // namespace

void options_default(uvio_hp_options_t *o) {
  std::memset(o, 0, sizeof(*o));
  // StateOptions.h
  o->do_fej = 1;
  o->integration = 1;  // RK4
  o->num_cameras = 1;
  o->use_stereo = 1;
  o->imu_model = 0;
  o->max_clone_size = 11;
  o->max_slam_features = 25;
  o->max_slam_in_update = 1000;
  o->max_msckf_in_update = 1000;
  o->max_aruco_features = 1024;
  o->feat_rep_msckf = 0;  // GLOBAL_3D
  o->feat_rep_slam = 0;
  o->dt_slam_delay = 2.0;
  o->gravity_mag = 9.81;
  // UpdaterOptions.h
  o->msckf_sigma_pix = 1.0;
  o->msckf_chi2_multipler = 5.0;
  o->slam_sigma_pix = 1.0;
  o->slam_chi2_multipler = 5.0;
  // NoiseManager (Propagator.h)
  o->sigma_w = 1.6968e-04;
  o->sigma_wb = 1.9393e-05;
  o->sigma_a = 2.0000e-3;
  o->sigma_ab = 3.0000e-03;
  double d6[6] = {1, 0, 0, 1, 0, 1};
  std::memcpy(o->imu_dw, d6, sizeof(d6));
  std::memcpy(o->imu_da, d6, sizeof(d6));
  o->q_GYROtoIMU[3] = 1;
  o->q_ACCtoIMU[3] = 1;
  // FeatureInitializerOptions.h
  o->fi_triangulate_1d = 0;
  o->fi_refine_features = 1;
  o->fi_max_runs = 5;
  o->fi_init_lamda = 1e-3;
  o->fi_max_lamda = 1e10;
  o->fi_min_dx = 1e-6;
  o->fi_min_dcost = 1e-6;
  o->fi_lam_mult = 10;
  o->fi_min_dist = 0.10;
  o->fi_max_dist = 60;
  o->fi_max_baseline = 40;
  o->fi_max_cond_number = 10000;
  for (int i = 0; i < UVIO_HP_MAX_CAMS; i++) {
    o->cams[i].model = 0;
    o->cams[i].width = 752;
    o->cams[i].height = 480;
    double intr[8] = {458.654, 457.296, 367.215, 248.375, -0.28340811, 0.07395907, 0.00019359, 1.76187114e-05};
    std::memcpy(o->cams[i].intrinsics, intr, sizeof(intr));
    o->cams[i].q_ItoC[3] = 1;
  }
  // TrackKLT defaults (VioManagerOptions.h:440-452)
  o->num_pts = 150;
  o->fast_threshold = 20;
  o->grid_x = 5;
  o->grid_y = 5;
  o->min_px_dist = 10;
  o->histogram_method = 1;
  o->downsample_cameras = 0;
  o->track_frequency = 20.0;
  // uvio
  o->use_uwb = 0;
  o->do_calib_uwb_extrinsics = 0;
  o->prior_uwb_imu_cov = 0.1;
  o->uwb_sigma_range = 0.5;
  o->uwb_chi2_multipler = 1.0;
  o->min_dist_to_use_uwb = 0.5;
  o->record_timing = 1;
  o->init_max_features = 50;
  // UpdaterZeroVelocity (VioManagerOptions.h:83-95; UpdaterOptions chi2_multipler default 5)
  o->try_zupt = 0;
  o->zupt_chi2_multipler = 5;
  o->zupt_max_velocity = 1.0;
  o->zupt_noise_multiplier = 1.0;
  o->zupt_max_disparity = 1.0;
  o->zupt_only_at_beginning = 0;
  o->use_klt = 1;
  o->use_aruco = 0;
  o->record_timing_information = 0;
  std::snprintf(o->record_timing_filepath, sizeof(o->record_timing_filepath), "%s", "ov_msckf_timing.txt");
  // InertialInitializerOptions.h:64-76
  o->init_window_time = 1.0;
  o->init_imu_thresh = 1.0;
  o->init_max_disparity = 1.0;
  o->init_dyn_use = 0;
}

int options_load(const char *path, uvio_hp_options_t *o, std::string *err) {
  bool ok = false;
  Doc est{parse_yaml(path, &ok)};
  if (!ok) {
    if (err) *err = std::string("cannot read ") + path;
    return UVIO_HP_E_CONFIG;
  }
  std::string dir = dirname_of(path);
  // StateOptions
  est.getb({"use_fej"}, o->do_fej);
  std::string integ;
  if (est.gets({"integration"}, integ)) o->integration = integ == "discrete" ? 0 : (integ == "analytical" ? 2 : 1);
  est.getb({"calib_cam_extrinsics"}, o->do_calib_camera_pose);
  est.getb({"calib_cam_intrinsics"}, o->do_calib_camera_intrinsics);
  est.getb({"calib_cam_timeoffset"}, o->do_calib_camera_timeoffset);
  est.getb({"calib_imu_intrinsics"}, o->do_calib_imu_intrinsics);
  est.getb({"calib_imu_g_sensitivity"}, o->do_calib_imu_g_sensitivity);
  est.get({"max_clones"}, o->max_clone_size);
  est.get({"max_slam"}, o->max_slam_features);
  est.get({"max_slam_in_update"}, o->max_slam_in_update);
  est.get({"max_msckf_in_update"}, o->max_msckf_in_update);
  est.get({"num_aruco"}, o->max_aruco_features);
  est.get({"max_cameras"}, o->num_cameras);
  std::string rep;
  for (auto key : {"feat_rep_msckf", "feat_rep_slam"}) {
    if (!est.gets({key}, rep)) continue;
    const int r = rep_from_string(rep);
    if (r < 0) {  // LandmarkRepresentation::from_string (LandmarkRepresentation.h:80-101) knows no other name
      if (err) *err = std::string(key) + ": unknown landmark representation '" + rep + "'";
      return UVIO_HP_E_CONFIG;
    }
    (std::string(key) == "feat_rep_msckf" ? o->feat_rep_msckf : o->feat_rep_slam) = r;
  }
  est.getb({"try_zupt"}, o->try_zupt);
  est.get({"zupt_chi2_multipler"}, o->zupt_chi2_multipler);
  est.get({"zupt_max_velocity"}, o->zupt_max_velocity);
  est.get({"zupt_noise_multiplier"}, o->zupt_noise_multiplier);
  est.get({"zupt_max_disparity"}, o->zupt_max_disparity);
  est.getb({"zupt_only_at_beginning"}, o->zupt_only_at_beginning);
  est.getb({"use_klt"}, o->use_klt);
  est.getb({"use_aruco"}, o->use_aruco);
  est.getb({"use_stereo"}, o->use_stereo);
  est.get({"dt_slam_delay"}, o->dt_slam_delay);
  est.get({"gravity_mag"}, o->gravity_mag);
  est.get({"up_msckf_sigma_px"}, o->msckf_sigma_pix);
  est.get({"up_msckf_chi2_multipler"}, o->msckf_chi2_multipler);
  est.get({"up_slam_sigma_px"}, o->slam_sigma_pix);
  est.get({"up_slam_chi2_multipler"}, o->slam_chi2_multipler);
  // feature initializer (fi_* keys, FeatureInitializerOptions.h:74-85)
  est.getb({"fi_triangulate_1d"}, o->fi_triangulate_1d);
  est.getb({"fi_refine_features"}, o->fi_refine_features);
  est.get({"fi_max_runs"}, o->fi_max_runs);
  est.get({"fi_init_lamda"}, o->fi_init_lamda);
  est.get({"fi_max_lamda"}, o->fi_max_lamda);
  est.get({"fi_min_dx"}, o->fi_min_dx);
  est.get({"fi_min_dcost"}, o->fi_min_dcost);
  est.get({"fi_lam_mult"}, o->fi_lam_mult);
  est.get({"fi_min_dist"}, o->fi_min_dist);
  est.get({"fi_max_dist"}, o->fi_max_dist);
  est.get({"fi_max_baseline"}, o->fi_max_baseline);
  est.get({"fi_max_cond_number"}, o->fi_max_cond_number);
  // tracker
  est.get({"num_pts"}, o->num_pts);
  est.get({"fast_threshold"}, o->fast_threshold);
  est.get({"init_max_features"}, o->init_max_features);
  est.get({"init_window_time"}, o->init_window_time);
  est.get({"init_imu_thresh"}, o->init_imu_thresh);
  est.get({"init_max_disparity"}, o->init_max_disparity);
  est.getb({"init_dyn_use"}, o->init_dyn_use);
  est.get({"grid_x"}, o->grid_x);
  est.get({"grid_y"}, o->grid_y);
  est.get({"min_px_dist"}, o->min_px_dist);
  est.get({"track_frequency"}, o->track_frequency);
  est.getb({"downsample_cameras"}, o->downsample_cameras);
  std::string hm;
  if (est.gets({"histogram_method"}, hm)) o->histogram_method = hm == "NONE" ? 0 : (hm == "CLAHE" ? 2 : 1);
  est.getb({"record_timing_information"}, o->record_timing_information);
  std::string tpath;
  if (est.gets({"record_timing_filepath"}, tpath))
    std::snprintf(o->record_timing_filepath, sizeof(o->record_timing_filepath), "%s", tpath.c_str());
  o->record_timing = 1;  // the per-frame timing struct is always kept (cheap); the CSV file is the option above

  // IMU chain (relative_config_imu)
  std::string rel;
  if (est.gets({"relative_config_imu"}, rel)) {
    bool ok2 = false;
    Doc imu{parse_yaml(dir + "/" + rel, &ok2)};
    if (!ok2) {
      if (err) *err = "cannot read " + dir + "/" + rel;
      return UVIO_HP_E_CONFIG;
    }
    imu.get({"imu0", "gyroscope_noise_density"}, o->sigma_w);
    imu.get({"imu0", "gyroscope_random_walk"}, o->sigma_wb);
    imu.get({"imu0", "accelerometer_noise_density"}, o->sigma_a);
    imu.get({"imu0", "accelerometer_random_walk"}, o->sigma_ab);
    std::string model;
    if (imu.gets({"imu0", "model"}, model)) o->imu_model = (model == "rpng") ? 1 : 0;
    auto m3 = [&](const char *k, double out[9], bool ident) {
      std::vector<std::vector<double>> m;
      for (int i = 0; i < 9; i++) out[i] = ident ? ((i % 4 == 0) ? 1.0 : 0.0) : 0.0;
      if (imu.getmat({"imu0", k}, m) && m.size() == 3)
        for (int r = 0; r < 3; r++)
          for (int c = 0; c < 3 && c < (int)m[r].size(); c++) out[3 * r + c] = m[r][c];
    };
    double Tw[9], Ta[9], Racc[9], Rgyro[9], Tg[9], Dw[9], Da[9];
    m3("Tw", Tw, true);
    m3("Ta", Ta, true);
    m3("R_IMUtoACC", Racc, true);
    m3("R_IMUtoGYRO", Rgyro, true);
    m3("Tg", Tg, false);
    if (!inv3(Tw, Dw) || !inv3(Ta, Da)) {
      if (err) *err = "bad IMU intrinsics";
      return UVIO_HP_E_CONFIG;
    }
    auto D = [](const double *M, int r, int c) { return M[3 * r + c]; };
    if (o->imu_model == 0) {
      double vdw[6] = {D(Dw, 0, 0), D(Dw, 1, 0), D(Dw, 2, 0), D(Dw, 1, 1), D(Dw, 2, 1), D(Dw, 2, 2)};
      double vda[6] = {D(Da, 0, 0), D(Da, 1, 0), D(Da, 2, 0), D(Da, 1, 1), D(Da, 2, 1), D(Da, 2, 2)};
      std::memcpy(o->imu_dw, vdw, sizeof(vdw));
      std::memcpy(o->imu_da, vda, sizeof(vda));
    } else {
      double vdw[6] = {D(Dw, 0, 0), D(Dw, 0, 1), D(Dw, 1, 1), D(Dw, 0, 2), D(Dw, 1, 2), D(Dw, 2, 2)};
      double vda[6] = {D(Da, 0, 0), D(Da, 0, 1), D(Da, 1, 1), D(Da, 0, 2), D(Da, 1, 2), D(Da, 2, 2)};
      std::memcpy(o->imu_dw, vdw, sizeof(vdw));
      std::memcpy(o->imu_da, vda, sizeof(vda));
    }
    double vtg[9] = {D(Tg, 0, 0), D(Tg, 1, 0), D(Tg, 2, 0), D(Tg, 0, 1), D(Tg, 1, 1), D(Tg, 2, 1),
                     D(Tg, 0, 2), D(Tg, 1, 2), D(Tg, 2, 2)};
    std::memcpy(o->imu_tg, vtg, sizeof(vtg));
    // R_GYROtoIMU = R_IMUtoGYRO^T ; q = rot_2_quat(R)
    double Rg[9], Ra[9];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        Rg[3 * r + c] = Rgyro[3 * c + r];
        Ra[3 * r + c] = Racc[3 * c + r];
      }
    rot_2_quat(Rg, o->q_GYROtoIMU);
    rot_2_quat(Ra, o->q_ACCtoIMU);
  }
  // camera chain (relative_config_imucam)
  if (est.gets({"relative_config_imucam"}, rel)) {
    bool ok2 = false;
    Doc cam{parse_yaml(dir + "/" + rel, &ok2)};
    if (!ok2) {
      if (err) *err = "cannot read " + dir + "/" + rel;
      return UVIO_HP_E_CONFIG;
    }
    for (int i = 0; i < o->num_cameras && i < UVIO_HP_MAX_CAMS; i++) {
      std::string cn = "cam" + std::to_string(i);
      uvio_hp_camera_t &c = o->cams[i];
      if (i == 0) cam.get({cn, "timeshift_cam_imu"}, o->calib_camimu_dt);
      std::string dm;
      if (cam.gets({cn, "distortion_model"}, dm)) c.model = (dm == "equidistant") ? 1 : 0;
      std::vector<double> in, dc, res;
      if (cam.getvec({cn, "intrinsics"}, in) && in.size() == 4)
        for (int k = 0; k < 4; k++) c.intrinsics[k] = in[k];
      if (cam.getvec({cn, "distortion_coeffs"}, dc) && dc.size() == 4)
        for (int k = 0; k < 4; k++) c.intrinsics[4 + k] = dc[k];
      if (cam.getvec({cn, "resolution"}, res) && res.size() == 2) {
        c.width = (int)res[0];
        c.height = (int)res[1];
      }
      if (o->downsample_cameras) {
        // VioManagerOptions.h:251-260: fx fy cx cy and the resolution halved (the trackers run on the
        // pyrDown'ed images, VioManager.cpp:270-278).  An odd raw size has no exact 2:1 inverse in the
        // feed's contract (raw = 2 w x 2 h), so it is refused.
        if (c.width % 2 || c.height % 2) {
          if (err) *err = cn + ": downsample_cameras needs an even resolution";
          return UVIO_HP_E_CONFIG;
        }
        c.width /= 2;
        c.height /= 2;
        for (int k = 0; k < 4; k++) c.intrinsics[k] /= 2.0;
      }
      std::vector<std::vector<double>> T;
      bool have_T = cam.getmat({cn, "T_imu_cam"}, T) && T.size() >= 3;
      if (!have_T && cam.getmat({cn, "T_cam_imu"}, T) && T.size() >= 3) {
        // YamlParser::parse(Matrix4d) (opencv_yaml_parse.h:487-530): T_imu_cam missing -> read T_cam_imu
        // = [R_ItoC p_IinC] and return its inverse [R_ItoC^T, -R_ItoC^T p_IinC]
        std::vector<std::vector<double>> Ti(4, std::vector<double>(4, 0.0));
        for (int r = 0; r < 3; r++) {
          for (int cc = 0; cc < 3; cc++) Ti[r][cc] = T[cc][r];
          Ti[r][3] = -(T[0][r] * T[0][3] + T[1][r] * T[1][3] + T[2][r] * T[2][3]);
        }
        Ti[3][3] = 1.0;
        T = Ti;
        have_T = true;
      }
      if (have_T) {
        // T_imu_cam = [R_CtoI p_CinI]; q_ItoC = rot_2_quat(R_CtoI^T); p_IinC = -R_CtoI^T p_CinI
        double RT[9];
        for (int r = 0; r < 3; r++)
          for (int cc = 0; cc < 3; cc++) RT[3 * r + cc] = T[cc][r];
        rot_2_quat(RT, c.q_ItoC);
        for (int r = 0; r < 3; r++) c.p_IinC[r] = -(RT[3 * r] * T[0][3] + RT[3 * r + 1] * T[1][3] + RT[3 * r + 2] * T[2][3]);
      }
    }
  }
  // uvio: config_uwb / uwb_anchors (UVioManagerOptions.h:52-90)
  if (est.gets({"config_uwb"}, rel)) {
    bool ok2 = false;
    Doc uwb{parse_yaml(dir + "/" + rel, &ok2)};
    if (ok2) {
      o->use_uwb = 1;
      uwb.get({"init", "n_fixed_anchors"}, o->n_anchors_to_fix);
      uwb.get({"init", "n_known_anchors"}, o->n_anchors);
      uwb.get({"init", "min_dist_to_use_uwb"}, o->min_dist_to_use_uwb);
      uwb.getb({"tag0", "calib_uwb_extrinsics"}, o->do_calib_uwb_extrinsics);
      uwb.get({"tag0", "prior_uwb_imu_cov"}, o->prior_uwb_imu_cov);
      uwb.get({"tag0", "uwb_sigma_range"}, o->uwb_sigma_range);
      uwb.get({"tag0", "uwb_chi2_multipler"}, o->uwb_chi2_multipler);
      std::vector<double> p_UinI, p0;
      if (uwb.getvec({"tag0", "p_UinI"}, p_UinI) && p_UinI.size() == 3)
        for (int k = 0; k < 3; k++) o->p_IinU[k] = -p_UinI[k];
      double off[3] = {0, 0, 0};
      if (uwb.getvec({"tag0", "p_IinG0"}, p0) && p0.size() == 3)
        for (int k = 0; k < 3; k++) off[k] = p0[k];
      if (o->n_anchors > UVIO_HP_MAX_ANCHORS) o->n_anchors = UVIO_HP_MAX_ANCHORS;
      if (o->n_anchors > 0) {
        bool ok3 = false;
        Doc anc{parse_yaml(dir + "/uwb_anchors.yaml", &ok3)};
        for (int i = 0; ok3 && i < o->n_anchors; i++) {
          std::string an = "anchor" + std::to_string(i);
          uvio_hp_anchor_t &a = o->anchors[i];
          int id = 0, fix = 0;
          anc.get({an, "id"}, id);
          anc.getb({an, "fix"}, fix);
          a.id = (uint64_t)id;
          a.fix = fix;
          std::vector<double> pos;
          if (anc.getvec({an, "p_AinG"}, pos) && pos.size() == 3)
            for (int k = 0; k < 3; k++) a.p_AinG[k] = pos[k] - off[k];
          anc.get({an, "const_bias"}, a.const_bias);
          anc.get({an, "dist_bias"}, a.dist_bias);
          double p = 0, c = 0, d = 0;
          anc.get({an, "prior_p_AinG_cov"}, p);
          anc.get({an, "prior_const_bias_cov"}, c);
          anc.get({an, "prior_dist_bias_cov"}, d);
          double cd[5] = {p, p, p, c, d};
          std::memcpy(a.cov_diag, cd, sizeof(cd));
        }
      }
    }
  }
  return UVIO_HP_OK;
}

}  // namespace uvhp
