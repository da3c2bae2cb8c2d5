// uvio_run_asl: a ROS-free serial runner over an ASL (EuRoC-format) dataset folder, driving the library through
// its C ABI exactly as ov_msckf/src/ros1_serial_msckf.cpp:127-275 drives VioManager through ROS1Visualizer:
// every message in time order, IMU straight in, a camera message together with the other cameras' messages
// within 0.02 s after it (skipped if one is missing), ground-truth initialization at the first camera message
// that has a ground-truth state (DatasetReader::get_gt_state, dataset_reader.h:110-160), and per camera frame
// the estimate written in ov_eval's trajectory format.  The timing CSV is the library's own
// (record_timing_information in the config, VioManager.cpp:105-122, 631-644).
//
//   uvio_run_asl CONFIG.yaml DATASET [--gt FILE.csv] [--start S] [--duration D] [--out TRAJ.txt] [--dry-run]
//
// DATASET/mav0/imu0/data.csv        #timestamp [ns],w_x,w_y,w_z,a_x,a_y,a_z
// DATASET/mav0/camK/data.csv        #timestamp [ns],filename   (K < num_cameras; 8-bit grayscale PNGs in camK/data/)
// DATASET/mav0/uwb0/data.csv        optional (uvio): #timestamp [ns],anchor_id,range[m]   -> uvio_hp_feed_uwb
// --gt: ASL ground truth (#timestamp [ns],p(3),q_wxyz(4),v(3),bw(3),ba(3)); --start / --duration in seconds from
// the first message (ros1_serial_msckf's bag_start / bag_durr); --dry-run parses and decodes everything and prints
// a JSON summary without creating the estimator (no GPU needed).
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "uvio_hp.h"

namespace {

struct Img {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
};

[[noreturn]] void die(const std::string &m) {
  std::fprintf(stderr, "uvio_run_asl: %s\n", m.c_str());
  std::exit(2);
}

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// 8-bit grayscale, non-interlaced PNG (the EuRoC / TUM-VI / UZH-FPV images): chunks, zlib inflate, the five
// scanline filters of the PNG specification
Img read_png(const std::string &path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) die("cannot open " + path);
  std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) die("not a PNG: " + path);
  Img im;
  std::vector<uint8_t> z;
  size_t p = 8;
  int depth = 0, ctype = -1, interlace = 0;
  while (p + 8 <= d.size()) {
    const uint32_t len = be32(&d[p]);
    const std::string type((const char *)&d[p + 4], 4);
    if (p + 12 + len > d.size()) die("truncated PNG: " + path);
    const uint8_t *c = &d[p + 8];
    if (type == "IHDR") {
      im.w = (int)be32(c);
      im.h = (int)be32(c + 4);
      depth = c[8];
      ctype = c[9];
      interlace = c[12];
    } else if (type == "IDAT") {
      z.insert(z.end(), c, c + len);
    } else if (type == "IEND") {
      break;
    }
    p += 12 + len;
  }
  if (depth != 8 || ctype != 0 || interlace != 0) die("only 8-bit grayscale non-interlaced PNGs: " + path);
  const size_t stride = (size_t)im.w + 1;
  std::vector<uint8_t> raw(stride * im.h);
  uLongf n = (uLongf)raw.size();
  if (uncompress(raw.data(), &n, z.data(), (uLong)z.size()) != Z_OK || n != raw.size()) die("bad PNG data: " + path);
  im.px.resize((size_t)im.w * im.h);
  for (int y = 0; y < im.h; y++) {
    const uint8_t ft = raw[y * stride];
    const uint8_t *s = &raw[y * stride + 1];
    uint8_t *o = &im.px[(size_t)y * im.w];
    const uint8_t *up = y > 0 ? &im.px[(size_t)(y - 1) * im.w] : nullptr;
    for (int x = 0; x < im.w; x++) {
      const int a = x > 0 ? o[x - 1] : 0, b = up ? up[x] : 0, cc = (up && x > 0) ? up[x - 1] : 0;
      int v = s[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: {
          const int pp = a + b - cc, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - cc);
          v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
          break;
        }
        default: die("bad PNG filter: " + path);
      }
      o[x] = (uint8_t)v;
    }
  }
  return im;
}

std::vector<std::vector<std::string>> read_csv(const std::string &path, bool required) {
  std::vector<std::vector<std::string>> rows;
  std::ifstream f(path);
  if (!f) {
    if (required) die("cannot open " + path);
    return rows;
  }
  std::string line;
  while (std::getline(f, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty() || line[0] == '#') continue;
    std::vector<std::string> r;
    std::istringstream s(line);
    std::string field;
    while (std::getline(s, field, ',')) r.push_back(field);
    rows.push_back(r);
  }
  return rows;
}

double ns_to_s(const std::string &s) { return 1e-9 * std::atof(s.c_str()); }

// one message of the merged stream (ros1_serial_msckf.cpp:160-183)
struct Msg {
  double t;
  int kind;  // 0 imu, 1 camera, 2 uwb
  int cam;
  size_t idx;
};

}  // namespace

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: uvio_run_asl CONFIG.yaml DATASET [--gt FILE] [--start S] [--duration D] [--out FILE] "
                         "[--dry-run]\n");
    return 2;
  }
  const std::string config = argv[1], ds = std::string(argv[2]) + "/mav0";
  std::string gt_path, out_path;
  double start = 0.0, dur = -1.0;
  bool dry = false;
  for (int i = 3; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) die("missing value after " + a);
      return argv[++i];
    };
    if (a == "--gt") gt_path = next();
    else if (a == "--start") start = std::atof(next().c_str());
    else if (a == "--duration") dur = std::atof(next().c_str());
    else if (a == "--out") out_path = next();
    else if (a == "--dry-run") dry = true;
    else die("unknown argument " + a);
  }

  uvio_hp_options_t opts;
  uvio_hp_options_default(&opts);
  if (uvio_hp_options_load(config.c_str(), &opts) != UVIO_HP_OK) die("cannot load " + config);
  const int ncam = opts.num_cameras;

  // ---- the dataset
  auto imu = read_csv(ds + "/imu0/data.csv", true);
  std::vector<std::vector<std::vector<std::string>>> cam(ncam);
  for (int k = 0; k < ncam; k++) cam[k] = read_csv(ds + "/cam" + std::to_string(k) + "/data.csv", true);
  auto uwb = read_csv(ds + "/uwb0/data.csv", false);
  std::map<double, std::vector<double>> gt;  // load_gt_file: time (s) -> the 17 values of the line
  if (!gt_path.empty())
    for (auto &r : read_csv(gt_path, true)) {
      std::vector<double> v;
      for (auto &f : r) v.push_back(std::atof(f.c_str()));
      if (v.size() < 17) die("ground truth line too short in " + gt_path);
      gt[1e-9 * v[0]] = v;
    }
  std::vector<Msg> msgs;
  for (size_t i = 0; i < imu.size(); i++) msgs.push_back({ns_to_s(imu[i][0]), 0, -1, i});
  for (int k = 0; k < ncam; k++)
    for (size_t i = 0; i < cam[k].size(); i++) msgs.push_back({ns_to_s(cam[k][i][0]), 1, k, i});
  // UWB: consecutive rows with one timestamp form one message
  std::vector<std::pair<double, std::vector<std::pair<uint64_t, double>>>> uwbm;
  for (auto &r : uwb) {
    const double t = ns_to_s(r[0]);
    if (uwbm.empty() || uwbm.back().first != t) uwbm.push_back({t, {}});
    uwbm.back().second.push_back({(uint64_t)std::atoll(r[1].c_str()), std::atof(r[2].c_str())});
  }
  for (size_t i = 0; i < uwbm.size(); i++) msgs.push_back({uwbm[i].first, 2, -1, i});
  // bag order: by time; at equal times IMU, then UWB, then cameras in camera order
  std::stable_sort(msgs.begin(), msgs.end(), [](const Msg &a, const Msg &b) {
    if (a.t != b.t) return a.t < b.t;
    const int ra = a.kind == 1 ? 2 : (a.kind == 2 ? 1 : 0), rb = b.kind == 1 ? 2 : (b.kind == 2 ? 1 : 0);
    if (ra != rb) return ra < rb;
    return a.cam < b.cam;
  });
  if (msgs.empty()) die("no messages");
  const double t_init = msgs.front().t + start;
  const double t_fin = dur < 0 ? INFINITY : t_init + dur;
  double max_cam_t = -1;
  for (auto &m : msgs)
    if (m.kind == 1) max_cam_t = std::max(max_cam_t, m.t);

  uvio_hp_t *h = nullptr;
  if (!dry && uvio_hp_create(&opts, 0, &h) != UVIO_HP_OK) die(std::string("uvio_hp_create: ") + uvio_hp_last_error(nullptr));
  FILE *out = nullptr;
  if (!out_path.empty()) {
    out = std::fopen(out_path.c_str(), "w");
    if (!out) die("cannot write " + out_path);
    std::fprintf(out, "# timestamp(s) tx ty tz qx qy qz qw\n");  // ov_eval's estimate format
  }
  size_t n_imu = 0, n_frames = 0, n_skipped = 0, n_uwb = 0, n_img = 0;
  uint64_t pix_sum = 0;
  int rc_last = 0;
  std::vector<bool> used(msgs.size(), false);
  for (size_t m = 0; m < msgs.size(); m++) {
    const Msg &g = msgs[m];
    if (g.t > t_fin || g.t > max_cam_t) break;
    if (g.t < t_init) continue;
    if (used[m]) continue;
    if (g.kind == 0) {
      const auto &r = imu[g.idx];
      const double wm[3] = {std::atof(r[1].c_str()), std::atof(r[2].c_str()), std::atof(r[3].c_str())};
      const double am[3] = {std::atof(r[4].c_str()), std::atof(r[5].c_str()), std::atof(r[6].c_str())};
      if (h && uvio_hp_feed_imu(h, g.t, wm, am) != UVIO_HP_OK) die(std::string("feed_imu: ") + uvio_hp_last_error(h));
      n_imu++;
      continue;
    }
    if (g.kind == 2) {
      std::vector<uint64_t> ids;
      std::vector<double> rg;
      for (auto &a : uwbm[g.idx].second) ids.push_back(a.first), rg.push_back(a.second);
      if (h && uvio_hp_feed_uwb(h, g.t, (int)ids.size(), ids.data(), rg.data()) != UVIO_HP_OK)
        die(std::string("feed_uwb: ") + uvio_hp_last_error(h));
      n_uwb++;
      continue;
    }
    // a camera message: the other cameras' next messages within 0.02 s (ros1_serial_msckf.cpp:204-227)
    std::vector<size_t> pick(ncam, (size_t)-1);
    pick[g.cam] = m;
    for (int k = 0; k < ncam; k++) {
      if (k == g.cam) continue;
      for (size_t q = m; q < msgs.size(); q++) {
        if (msgs[q].kind != 1 || msgs[q].cam != k) continue;
        if (std::fabs(msgs[q].t - g.t) < 0.02) pick[k] = q;
        break;
      }
    }
    if (std::count(pick.begin(), pick.end(), (size_t)-1) > 0) {
      n_skipped++;
      continue;
    }
    if (ncam > 2) die("the serial runner takes 1 or 2 cameras (ros1_serial_msckf.cpp:254-267)");
    for (size_t q : pick) used[q] = true;
    used[m] = false;
    std::vector<Img> imgs(ncam);
    for (int k = 0; k < ncam; k++) {
      const Msg &mk = msgs[pick[k]];
      imgs[k] = read_png(ds + "/cam" + std::to_string(k) + "/data/" + cam[k][mk.idx][1]);
      n_img++;
      for (uint8_t v : imgs[k].px) pix_sum += v;
    }
    // ground-truth initialization (ros1_serial_msckf.cpp:237-243 + DatasetReader::get_gt_state)
    int initialized = 1;
    if (h) uvio_hp_initialized(h, &initialized);
    if (!gt.empty() && !initialized) {
      double best = INFINITY;
      for (auto &kv : gt)
        if (std::fabs(kv.first - g.t) < std::fabs(best - g.t)) best = kv.first;
      const double ts = std::fabs(best - g.t) < 0.10 ? best : g.t;
      auto it = gt.find(ts);
      if (it != gt.end()) {
        const std::vector<double> &v = it->second;
        const double x[17] = {ts, v[5], v[6], v[7], v[4], v[1], v[2], v[3], v[8], v[9], v[10], v[11], v[12], v[13],
                              v[14], v[15], v[16]};
        if (h && uvio_hp_initialize_with_gt(h, x) != UVIO_HP_OK) die(std::string("initialize_with_gt: ") + uvio_hp_last_error(h));
      }
    }
    std::vector<int> ids(ncam), strides(ncam);
    std::vector<const uint8_t *> ptrs(ncam);
    for (int k = 0; k < ncam; k++) ids[k] = k, strides[k] = imgs[k].w, ptrs[k] = imgs[k].px.data();
    n_frames++;
    if (!h) continue;
    rc_last = uvio_hp_feed_camera(h, g.t, ncam, ids.data(), ptrs.data(), strides.data(), nullptr);
    if (rc_last != UVIO_HP_OK && rc_last != UVIO_HP_E_STATE && rc_last != UVIO_HP_E_ORDER)
      die(std::string("feed_camera: ") + uvio_hp_last_error(h));
    int init = 0;
    uvio_hp_initialized(h, &init);
    if (out && init && rc_last == UVIO_HP_OK) {
      double ts, x[16];
      uvio_hp_get_imu_state(h, &ts, x);
      std::fprintf(out, "%.9f %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", ts, x[4], x[5], x[6], x[0], x[1], x[2], x[3]);
    }
  }
  if (out) std::fclose(out);
  if (h) uvio_hp_destroy(h);
  std::printf("{\"imu\": %zu, \"frames\": %zu, \"skipped_unsynced\": %zu, \"uwb\": %zu, \"images\": %zu, "
              "\"pixel_sum\": %llu, \"gt_states\": %zu, \"dry_run\": %s, \"options\": {\"init_max_features\": %d, "
              "\"max_msckf_in_update\": %d, \"max_slam_features\": %d, \"max_slam_in_update\": %d, "
              "\"dt_slam_delay\": %.17g}}\n",
              n_imu, n_frames, n_skipped, n_uwb, n_img, (unsigned long long)pix_sum, gt.size(), dry ? "true" : "false",
              opts.init_max_features, opts.max_msckf_in_update, opts.max_slam_features, opts.max_slam_in_update,
              opts.dt_slam_delay);
  return 0;
}
