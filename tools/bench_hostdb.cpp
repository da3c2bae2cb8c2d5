// Host-side cost model of the TrackSIM feed + feature database at cfg4 shapes (CPU only; no GPU):
// undistort per observation, FeatureDatabase::update_feature, the per-frame selection scans and the
// marginalization cleanup.  Build: hipcc -O3 -std=c++17 -I include tools/bench_hostdb.cpp -o /tmp/bhd
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../uvio_amd/csrc/hp_math.h"

using namespace uvhp;
using clk = std::chrono::steady_clock;

#ifdef OLD_LAYOUT
struct Feature {
  size_t featid = 0;
  bool to_delete = false;
  std::unordered_map<size_t, std::vector<std::pair<float, float>>> uvs, uvs_norm;
  std::unordered_map<size_t, std::vector<double>> timestamps;
};
#else
struct FeatMeas { float u, v, un, vn; double t; };
struct CamTrack { size_t cam; std::vector<FeatMeas> m; };
struct Feature {
  size_t featid = 0;
  bool to_delete = false;
  std::vector<CamTrack> tracks;
  CamTrack &track(size_t cam) {
    for (auto &c : tracks) if (c.cam == cam) return c;
    tracks.insert(tracks.begin(), CamTrack{cam, {}});
    return tracks.front();
  }
};
#endif
using FeatP = std::shared_ptr<Feature>;

int main() {
  CamParams c{};
  c.model = 1;
  double v[8] = {275.3, 275.1, 315.8, 233.7, -0.0178, 0.049, -0.0414, 0.0114};
  for (int k = 0; k < 8; k++) c.v[k] = v[k];
  c.w = 640, c.h = 480;
  const int F = 800, life = 26, K = 2, frames = 60;
  std::unordered_map<size_t, FeatP> db;
  double t_und = 0, t_db = 0, t_scan = 0, t_clean = 0;
  size_t nid = 0;
  std::vector<size_t> alive;
  for (int fr = 0; fr < frames; fr++) {
    double t = fr * 0.05;
    for (int i = 0; i < F; i++) alive.push_back(nid++);
    if ((int)alive.size() > F * life) alive.erase(alive.begin(), alive.begin() + F);
    std::vector<float> uv(2 * alive.size() * K), un(uv.size());
    for (size_t i = 0; i < uv.size(); i++) uv[i] = 20.f + (float)((i * 7919) % 600);
    auto a = clk::now();
    for (size_t i = 0; i < uv.size() / 2; i++) cam_undistort_f(c, uv[2 * i], uv[2 * i + 1], un[2 * i], un[2 * i + 1]);
    auto b = clk::now();
    size_t k = 0;
    for (int cam = 0; cam < K; cam++)
      for (size_t id : alive) {
        auto it = db.find(id);
        FeatP f;
        if (it != db.end())
          f = it->second;
        else {
          f = std::make_shared<Feature>();
          f->featid = id;
          db[id] = f;
        }
#ifdef OLD_LAYOUT
        f->uvs[cam].push_back({uv[2 * k], uv[2 * k + 1]});
        f->uvs_norm[cam].push_back({un[2 * k], un[2 * k + 1]});
        f->timestamps[cam].push_back(t);
#else
        f->track(cam).m.push_back({uv[2 * k], uv[2 * k + 1], un[2 * k], un[2 * k + 1], t});
#endif
        k++;
      }
    auto cc = clk::now();
    // selection scans: features_not_containing_newer + marg lookup
    size_t lost = 0, marg = 0;
    double mt = t - life * 0.05;
#ifdef OLD_LAYOUT
    for (auto &kv : db) {
      bool newer = false;
      for (auto &p : kv.second->timestamps) {
        newer = !p.second.empty() && p.second.back() >= t;
        if (newer) break;
      }
      if (!newer) lost++;
      for (auto &p : kv.second->timestamps)
        if (std::find(p.second.begin(), p.second.end(), mt) != p.second.end()) {
          marg++;
          break;
        }
    }
#else
    for (auto &kv : db) {
      bool newer = false;
      for (auto &p : kv.second->tracks) { newer = !p.m.empty() && p.m.back().t >= t; if (newer) break; }
      if (!newer) lost++;
      for (auto &p : kv.second->tracks)
        if (std::find_if(p.m.begin(), p.m.end(), [mt](const FeatMeas &x) { return x.t == mt; }) != p.m.end()) { marg++; break; }
    }
#endif
    volatile size_t sink = lost + marg; (void)sink;
    auto d = clk::now();
    // cleanup: drop measurements older than the marginalized clone
    for (auto it = db.begin(); it != db.end();) {
      auto &f = *it->second;
      size_t cnt = 0;
#ifndef OLD_LAYOUT
      for (auto &c : f.tracks) {
        size_t w = 0;
        for (size_t i = 0; i < c.m.size(); i++) if (!(c.m[i].t <= mt)) c.m[w++] = c.m[i];
        c.m.resize(w);
        cnt += w;
      }
#else
      for (auto &pair : f.timestamps) {
        auto &ts = pair.second;
        auto &u = f.uvs[pair.first];
        auto &n2 = f.uvs_norm[pair.first];
        size_t w = 0;
        for (size_t i = 0; i < ts.size(); i++)
          if (!(ts[i] <= mt)) ts[w] = ts[i], u[w] = u[i], n2[w] = n2[i], w++;
        ts.resize(w), u.resize(w), n2.resize(w);
        cnt += w;
      }
#endif
      if (cnt < 1)
        it = db.erase(it);
      else
        it++;
    }
    auto e = clk::now();
    if (fr >= frames - 20) {
      t_und += std::chrono::duration<double>(b - a).count();
      t_db += std::chrono::duration<double>(cc - b).count();
      t_scan += std::chrono::duration<double>(d - cc).count();
      t_clean += std::chrono::duration<double>(e - d).count();
    }
    (void)lost, (void)marg;
  }
  std::printf("per frame (ms): undistort %.3f  db_update %.3f  selection scans %.3f  cleanup %.3f  (db %zu features)\n",
              t_und / 20 * 1e3, t_db / 20 * 1e3, t_scan / 20 * 1e3, t_clean / 20 * 1e3, db.size());
  return 0;
}
