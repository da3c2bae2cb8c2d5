// ORACLE — test infrastructure only (see la.h header).
// TrackKLT per-frame logic: TrackKLT.cpp:34-886 and Grider_GRID.h:74-180 (see tracker.h).
#include <algorithm>
#include <cmath>

#include "feat.h"
#include "tracker.h"

namespace orc {

namespace {
struct U8Grid {
  int w, h;
  std::vector<uint8_t> d;
  U8Grid(int w_, int h_) : w(w_), h(h_), d((size_t)w_ * h_, 0) {}
  uint8_t &at(int x, int y) { return d[(size_t)y * w + x]; }
};
uint8_t mask_at(const GrayImg &m, int x, int y) { return m.d.empty() ? 0 : m.at(x, y); }
void fill_rect(GrayImg &m, int x1, int y1, int x2, int y2) {  // cv::rectangle(..., 255, FILLED), inclusive
  for (int y = std::max(0, y1); y <= std::min(m.h - 1, y2); y++)
    for (int x = std::max(0, x1); x <= std::min(m.w - 1, x2); x++) m.d[(size_t)y * m.w + x] = 255;
}
// cv::resize(mask, grid, INTER_NEAREST)
uint8_t mask_grid_at(const GrayImg &m, int gx, int gy, int GX, int GY) {
  if (m.d.empty()) return 0;
  int sx = std::min((int)std::floor(gx * ((double)m.w / GX)), m.w - 1);
  int sy = std::min((int)std::floor(gy * ((double)m.h / GY)), m.h - 1);
  return m.at(sx, sy);
}
}  // namespace

// Grider_GRID::perform_griding (Grider_GRID.h:74-180)
void TrackKLT::perform_griding(const GrayImg &img, const GrayImg &mask, const std::vector<std::pair<int, int>> &valid_locs,
                               std::vector<KeyPt> &pts) {
  if (valid_locs.empty()) return;
  int gx = grid_x, gy = grid_y;
  if (num_features < gx * gy) {
    double ratio = (double)gx / (double)gy;
    gy = (int)std::ceil(std::sqrt(num_features / ratio));
    gx = (int)std::ceil(gy * ratio);
  }
  int num_features_grid = (int)((double)num_features / (double)(gx * gy)) + 1;
  int size_x = img.w / gx, size_y = img.h / gy;
  std::vector<KeyPt> out;
  for (auto &g : valid_locs) {
    int x = g.first * size_x, y = g.second * size_y;
    if (x + size_x > img.w || y + size_y > img.h) continue;
    std::vector<KeyPt> kp = fast_roi(img, x, y, size_x, size_y, threshold);
    grid_sort(kp);
    for (size_t i = 0; i < (size_t)num_features_grid && i < kp.size(); i++) {
      KeyPt p = kp[i];
      p.x += (float)x;
      p.y += (float)y;
      if ((int)p.x < 0 || (int)p.x > img.w || (int)p.y < 0 || (int)p.y > img.h) continue;
      if (mask_at(mask, (int)p.x, (int)p.y) > 127) continue;
      out.push_back(p);
    }
  }
  if (out.empty()) return;
  corner_subpix(img, out, 5, 20, 0.001);
  pts.insert(pts.end(), out.begin(), out.end());
}

// TrackKLT::perform_detection_monocular (TrackKLT.cpp:395-528)
void TrackKLT::perform_detection_monocular(const Pyramid &pyr, const GrayImg &mask0, std::vector<KeyPt> &pts0,
                                           std::vector<size_t> &ids0) {
  const GrayImg &img = pyr.img[0];
  int scw = (int)((float)img.w / (float)min_px_dist), sch = (int)((float)img.h / (float)min_px_dist);
  U8Grid close(scw, sch), grid(grid_x, grid_y);
  float size_x = (float)img.w / (float)grid_x, size_y = (float)img.h / (float)grid_y;
  GrayImg mask_up = mask0;
  if (mask_up.d.empty()) {
    mask_up.w = img.w;
    mask_up.h = img.h;
    mask_up.d.assign((size_t)img.w * img.h, 0);
  }
  std::vector<KeyPt> kp;
  std::vector<size_t> kid;
  for (size_t i = 0; i < pts0.size(); i++) {
    const KeyPt &k = pts0[i];
    int x = (int)k.x, y = (int)k.y, edge = 10;
    if (x < edge || x >= img.w - edge || y < edge || y >= img.h - edge) continue;
    int xc = (int)(k.x / (float)min_px_dist), yc = (int)(k.y / (float)min_px_dist);
    if (xc < 0 || xc >= scw || yc < 0 || yc >= sch) continue;
    int xg = (int)std::floor(k.x / size_x), yg = (int)std::floor(k.y / size_y);
    if (xg < 0 || xg >= grid_x || yg < 0 || yg >= grid_y) continue;
    if (close.at(xc, yc) > 127) continue;
    if (mask_at(mask0, x, y) > 127) continue;
    close.at(xc, yc) = 255;
    if (grid.at(xg, yg) < 255) grid.at(xg, yg) += 1;
    if (x - min_px_dist >= 0 && x + min_px_dist < img.w && y - min_px_dist >= 0 && y + min_px_dist < img.h)
      fill_rect(mask_up, x - min_px_dist, y - min_px_dist, x + min_px_dist, y + min_px_dist);
    kp.push_back(k);
    kid.push_back(ids0[i]);
  }
  pts0 = kp;
  ids0 = kid;
  double min_feat_percent = 0.50;
  int needed = num_features - (int)pts0.size();
  if (needed < std::min(20, (int)(min_feat_percent * num_features))) return;
  int nfg = (int)((double)num_features / (double)(grid_x * grid_y)) + 1;
  int nfg_req = std::max(1, (int)(min_feat_percent * nfg));
  std::vector<std::pair<int, int>> valid;
  for (int x = 0; x < grid_x; x++)
    for (int y = 0; y < grid_y; y++)
      if ((int)grid.at(x, y) < nfg_req && (int)mask_grid_at(mask0, x, y, grid_x, grid_y) != 255) valid.emplace_back(x, y);
  std::vector<KeyPt> ext;
  perform_griding(img, mask_up, valid, ext);
  for (auto &k : ext) {
    int xg = (int)(k.x / (float)min_px_dist), yg = (int)(k.y / (float)min_px_dist);
    if (xg < 0 || xg >= scw || yg < 0 || yg >= sch) continue;
    if (close.at(xg, yg) > 127) continue;
    close.at(xg, yg) = 255;
    pts0.push_back(k);
    ids0.push_back(++currid);
  }
}

// TrackKLT::perform_detection_stereo (TrackKLT.cpp:530-827)
void TrackKLT::perform_detection_stereo(const Pyramid &p0, const Pyramid &p1, const GrayImg &mask0, const GrayImg &mask1, int cl,
                                        int cr, std::vector<KeyPt> &pts0, std::vector<KeyPt> &pts1, std::vector<size_t> &ids0,
                                        std::vector<size_t> &ids1) {
  (void)cl;
  (void)cr;
  const double min_feat_percent = 0.50;
  // ---- left ----
  {
    const GrayImg &img = p0.img[0];
    int scw = (int)((float)img.w / (float)min_px_dist), sch = (int)((float)img.h / (float)min_px_dist);
    U8Grid close(scw, sch), grid(grid_x, grid_y);
    float size_x = (float)img.w / (float)grid_x, size_y = (float)img.h / (float)grid_y;
    GrayImg mask_up = mask0;
    if (mask_up.d.empty()) {
      mask_up.w = img.w;
      mask_up.h = img.h;
      mask_up.d.assign((size_t)img.w * img.h, 0);
    }
    std::vector<KeyPt> kp;
    std::vector<size_t> kid;
    for (size_t i = 0; i < pts0.size(); i++) {
      const KeyPt &k = pts0[i];
      int x = (int)k.x, y = (int)k.y, edge = 10;
      if (x < edge || x >= img.w - edge || y < edge || y >= img.h - edge) continue;
      int xc = (int)(k.x / (float)min_px_dist), yc = (int)(k.y / (float)min_px_dist);
      if (xc < 0 || xc >= scw || yc < 0 || yc >= sch) continue;
      int xg = (int)std::floor(k.x / size_x), yg = (int)std::floor(k.y / size_y);
      if (xg < 0 || xg >= grid_x || yg < 0 || yg >= grid_y) continue;
      if (close.at(xc, yc) > 127) continue;
      if (mask_at(mask0, x, y) > 127) continue;
      close.at(xc, yc) = 255;
      if (grid.at(xg, yg) < 255) grid.at(xg, yg) += 1;
      if (x - min_px_dist >= 0 && x + min_px_dist < img.w && y - min_px_dist >= 0 && y + min_px_dist < img.h)
        fill_rect(mask_up, x - min_px_dist, y - min_px_dist, x + min_px_dist, y + min_px_dist);
      kp.push_back(k);
      kid.push_back(ids0[i]);
    }
    pts0 = kp;
    ids0 = kid;
    int needed = num_features - (int)pts0.size();
    if (needed > std::min(20, (int)(min_feat_percent * num_features))) {
      int nfg = (int)((double)num_features / (double)(grid_x * grid_y)) + 1;
      int nfg_req = std::max(1, (int)(min_feat_percent * nfg));
      std::vector<std::pair<int, int>> valid;
      for (int x = 0; x < grid_x; x++)
        for (int y = 0; y < grid_y; y++)
          if ((int)grid.at(x, y) < nfg_req && (int)mask_grid_at(mask0, x, y, grid_x, grid_y) != 255) valid.emplace_back(x, y);
      std::vector<KeyPt> ext;
      perform_griding(img, mask_up, valid, ext);
      std::vector<KeyPt> k0new;
      for (auto &k : ext) {
        int xg = (int)(k.x / (float)min_px_dist), yg = (int)(k.y / (float)min_px_dist);
        if (xg < 0 || xg >= scw || yg < 0 || yg >= sch) continue;
        if (close.at(xg, yg) > 127) continue;
        close.at(xg, yg) = 255;
        k0new.push_back(k);
      }
      if (!k0new.empty()) {
        std::vector<KeyPt> k1new = k0new;
        std::vector<uint8_t> st;
        lk_track(p0, p1, k0new, k1new, st, win, pyr_levels, 30, 0.01f);
        for (size_t i = 0; i < k0new.size(); i++) {
          const GrayImg &i1 = p1.img[0];
          bool oobl = ((int)k0new[i].x < 0 || (int)k0new[i].x >= img.w || (int)k0new[i].y < 0 || (int)k0new[i].y >= img.h);
          bool oobr = ((int)k1new[i].x < 0 || (int)k1new[i].x >= i1.w || (int)k1new[i].y < 0 || (int)k1new[i].y >= i1.h);
          if (!oobl && !oobr && st[i] == 1) {
            pts0.push_back(k0new[i]);
            pts1.push_back(k1new[i]);
            size_t id = ++currid;
            ids0.push_back(id);
            ids1.push_back(id);
          } else if (!oobl) {
            pts0.push_back(k0new[i]);
            ids0.push_back(++currid);
          }
        }
      }
    }
  }
  // ---- right ----
  {
    const GrayImg &img = p1.img[0];
    int scw = (int)((float)img.w / (float)min_px_dist), sch = (int)((float)img.h / (float)min_px_dist);
    U8Grid close(scw, sch), grid(grid_x, grid_y);
    float size_x = (float)img.w / (float)grid_x, size_y = (float)img.h / (float)grid_y;
    // the reference clones mask0 here (TrackKLT.cpp:713)
    GrayImg mask_up = mask0;
    if (mask_up.d.empty()) {
      mask_up.w = img.w;
      mask_up.h = img.h;
      mask_up.d.assign((size_t)img.w * img.h, 0);
    }
    std::vector<KeyPt> kp;
    std::vector<size_t> kid;
    for (size_t i = 0; i < pts1.size(); i++) {
      const KeyPt &k = pts1[i];
      int x = (int)k.x, y = (int)k.y, edge = 10;
      if (x < edge || x >= img.w - edge || y < edge || y >= img.h - edge) continue;
      int xc = (int)(k.x / (float)min_px_dist), yc = (int)(k.y / (float)min_px_dist);
      if (xc < 0 || xc >= scw || yc < 0 || yc >= sch) continue;
      int xg = (int)std::floor(k.x / size_x), yg = (int)std::floor(k.y / size_y);
      if (xg < 0 || xg >= grid_x || yg < 0 || yg >= grid_y) continue;
      bool is_stereo = std::find(ids0.begin(), ids0.end(), ids1[i]) != ids0.end();
      if (close.at(xc, yc) > 127 && !is_stereo) continue;
      if (mask_at(mask1, x, y) > 127) continue;
      close.at(xc, yc) = 255;
      if (grid.at(xg, yg) < 255) grid.at(xg, yg) += 1;
      if (x - min_px_dist >= 0 && x + min_px_dist < img.w && y - min_px_dist >= 0 && y + min_px_dist < img.h)
        fill_rect(mask_up, x - min_px_dist, y - min_px_dist, x + min_px_dist, y + min_px_dist);
      kp.push_back(k);
      kid.push_back(ids1[i]);
    }
    pts1 = kp;
    ids1 = kid;
    int needed = num_features - (int)pts1.size();
    if (needed > std::min(20, (int)(min_feat_percent * num_features))) {
      int nfg = (int)((double)num_features / (double)(grid_x * grid_y)) + 1;
      int nfg_req = std::max(1, (int)(min_feat_percent * nfg));
      std::vector<std::pair<int, int>> valid;
      for (int x = 0; x < grid_x; x++)
        for (int y = 0; y < grid_y; y++)
          if ((int)grid.at(x, y) < nfg_req && (int)mask_grid_at(mask1, x, y, grid_x, grid_y) != 255) valid.emplace_back(x, y);
      std::vector<KeyPt> ext;
      perform_griding(img, mask_up, valid, ext);
      for (auto &k : ext) {
        int xg = (int)(k.x / (float)min_px_dist), yg = (int)(k.y / (float)min_px_dist);
        if (xg < 0 || xg >= scw || yg < 0 || yg >= sch) continue;
        if (close.at(xg, yg) > 127) continue;
        pts1.push_back(k);
        ids1.push_back(++currid);
        close.at(xg, yg) = 255;
      }
    }
  }
}

// TrackKLT::perform_matching (TrackKLT.cpp:829-886)
void TrackKLT::perform_matching(const Pyramid &p0, const Pyramid &p1, std::vector<KeyPt> &k0, std::vector<KeyPt> &k1, int id0,
                                int id1, std::vector<uint8_t> &mask_out) {
  if (k0.empty() || k1.empty()) return;
  if (k0.size() < 10) {
    mask_out.assign(k0.size(), 0);
    return;
  }
  std::vector<uint8_t> st;
  lk_track(p0, p1, k0, k1, st, win, pyr_levels, 30, 0.01f);
  const Camera &c0 = cams->at(id0), &c1 = cams->at(id1);
  size_t n = k0.size();
  std::vector<float> x0(n), y0(n), x1(n), y1(n);
  for (size_t i = 0; i < n; i++) {
    c0.undistort_f(k0[i].x, k0[i].y, x0[i], y0[i]);
    c1.undistort_f(k1[i].x, k1[i].y, x1[i], y1[i]);
  }
  double f0 = std::max(c0.v[0], c0.v[1]), f1 = std::max(c1.v[0], c1.v[1]);
  double fmax = std::max(f0, f1);
  std::vector<uint8_t> rsc;
  ransac_fundamental_mask(x0, y0, x1, y1, 2.0 / fmax, 0.999, 1000, rsc);
  mask_out.resize(n);
  for (size_t i = 0; i < n; i++) mask_out[i] = (st[i] && i < rsc.size() && rsc[i]) ? 1 : 0;
}

void TrackKLT::feed_monocular(double t, int cam, const Pyramid &pyr, const GrayImg &mask, FeatureDatabase &db) {
  if (pts_last[cam].empty()) {
    std::vector<KeyPt> good;
    std::vector<size_t> gid;
    perform_detection_monocular(pyr, mask, good, gid);
    pyr_last[cam] = pyr;
    mask_last[cam] = mask;
    pts_last[cam] = good;
    ids_last[cam] = gid;
    return;
  }
  auto pts_old = pts_last[cam];
  auto ids_old = ids_last[cam];
  perform_detection_monocular(pyr_last[cam], mask_last[cam], pts_old, ids_old);
  std::vector<uint8_t> mask_ll;
  std::vector<KeyPt> pts_new = pts_old;
  perform_matching(pyr_last[cam], pyr, pts_old, pts_new, cam, cam, mask_ll);
  if (mask_ll.empty()) {
    pyr_last[cam] = pyr;
    mask_last[cam] = mask;
    pts_last[cam].clear();
    ids_last[cam].clear();
    return;
  }
  const GrayImg &img = pyr.img[0];
  std::vector<KeyPt> good;
  std::vector<size_t> gid;
  for (size_t i = 0; i < pts_new.size(); i++) {
    if (pts_new[i].x < 0 || pts_new[i].y < 0 || (int)pts_new[i].x >= img.w || (int)pts_new[i].y >= img.h) continue;
    if (mask_at(mask, (int)pts_new[i].x, (int)pts_new[i].y) > 127) continue;
    if (mask_ll[i]) {
      good.push_back(pts_new[i]);
      gid.push_back(ids_old[i]);
    }
  }
  const Camera &c = cams->at(cam);
  for (size_t i = 0; i < good.size(); i++) {
    float un, vn;
    c.undistort_f(good[i].x, good[i].y, un, vn);
    db.update_feature(gid[i], t, cam, good[i].x, good[i].y, un, vn);
  }
  pyr_last[cam] = pyr;
  mask_last[cam] = mask;
  pts_last[cam] = good;
  ids_last[cam] = gid;
}

void TrackKLT::feed_stereo(double t, int cl, int cr, const Pyramid &pl, const Pyramid &pr, const GrayImg &ml, const GrayImg &mr,
                           FeatureDatabase &db) {
  if (pts_last[cl].empty() && pts_last[cr].empty()) {
    std::vector<KeyPt> gl, gr;
    std::vector<size_t> il, ir;
    perform_detection_stereo(pl, pr, ml, mr, cl, cr, gl, gr, il, ir);
    pyr_last[cl] = pl;
    pyr_last[cr] = pr;
    mask_last[cl] = ml;
    mask_last[cr] = mr;
    pts_last[cl] = gl;
    pts_last[cr] = gr;
    ids_last[cl] = il;
    ids_last[cr] = ir;
    return;
  }
  auto pl_old = pts_last[cl], pr_old = pts_last[cr];
  auto il_old = ids_last[cl], ir_old = ids_last[cr];
  perform_detection_stereo(pyr_last[cl], pyr_last[cr], mask_last[cl], mask_last[cr], cl, cr, pl_old, pr_old, il_old, ir_old);
  std::vector<uint8_t> mask_ll, mask_rr;
  std::vector<KeyPt> pl_new = pl_old, pr_new = pr_old;
  perform_matching(pyr_last[cl], pl, pl_old, pl_new, cl, cl, mask_ll);
  perform_matching(pyr_last[cr], pr, pr_old, pr_new, cr, cr, mask_rr);
  if (mask_ll.empty() && mask_rr.empty()) {
    pyr_last[cl] = pl;
    pyr_last[cr] = pr;
    mask_last[cl] = ml;
    mask_last[cr] = mr;
    pts_last[cl].clear();
    pts_last[cr].clear();
    ids_last[cl].clear();
    ids_last[cr].clear();
    return;
  }
  const GrayImg &imgl = pl.img[0], &imgr = pr.img[0];
  std::vector<KeyPt> gl, gr;
  std::vector<size_t> gil, gir;
  for (size_t i = 0; i < pl_new.size(); i++) {
    if (pl_new[i].x < 0 || pl_new[i].y < 0 || (int)pl_new[i].x > imgl.w || (int)pl_new[i].y > imgl.h) continue;
    bool found = false;
    size_t ir = 0;
    for (size_t n = 0; n < ir_old.size(); n++)
      if (il_old[i] == ir_old[n]) {
        found = true;
        ir = n;
        break;
      }
    if (mask_ll[i] && found && mask_rr[ir]) {
      if (pr_new[ir].x < 0 || pr_new[ir].y < 0 || (int)pr_new[ir].x >= imgr.w || (int)pr_new[ir].y >= imgr.h) continue;
      gl.push_back(pl_new[i]);
      gr.push_back(pr_new[ir]);
      gil.push_back(il_old[i]);
      gir.push_back(ir_old[ir]);
    } else if (mask_ll[i]) {
      gl.push_back(pl_new[i]);
      gil.push_back(il_old[i]);
    }
  }
  for (size_t i = 0; i < pr_new.size(); i++) {
    if (pr_new[i].x < 0 || pr_new[i].y < 0 || (int)pr_new[i].x >= imgr.w || (int)pr_new[i].y >= imgr.h) continue;
    bool added = std::find(gir.begin(), gir.end(), ir_old[i]) != gir.end();
    if (mask_rr[i] && !added) {
      gr.push_back(pr_new[i]);
      gir.push_back(ir_old[i]);
    }
  }
  const Camera &c0 = cams->at(cl), &c1 = cams->at(cr);
  for (size_t i = 0; i < gl.size(); i++) {
    float un, vn;
    c0.undistort_f(gl[i].x, gl[i].y, un, vn);
    db.update_feature(gil[i], t, cl, gl[i].x, gl[i].y, un, vn);
  }
  for (size_t i = 0; i < gr.size(); i++) {
    float un, vn;
    c1.undistort_f(gr[i].x, gr[i].y, un, vn);
    db.update_feature(gir[i], t, cr, gr[i].x, gr[i].y, un, vn);
  }
  pyr_last[cl] = pl;
  pyr_last[cr] = pr;
  mask_last[cl] = ml;
  mask_last[cr] = mr;
  pts_last[cl] = gl;
  pts_last[cr] = gr;
  ids_last[cl] = gil;
  ids_last[cr] = gir;
}

// TrackKLT::feed_new_camera (TrackKLT.cpp:34-94)
void TrackKLT::feed(double t, const std::vector<int> &cam_ids, const std::vector<GrayImg> &images, const std::vector<GrayImg> &masks,
                    FeatureDatabase &db) {
  std::vector<Pyramid> pyrs;
  for (size_t k = 0; k < images.size(); k++) {
    GrayImg img = (histogram_method == 1) ? equalize_hist(images[k]) : images[k];
    pyrs.push_back(build_pyramid(img, win, pyr_levels));
  }
  if (images.size() == 1) {
    feed_monocular(t, cam_ids[0], pyrs[0], masks[0], db);
  } else if (images.size() == 2 && use_stereo) {
    feed_stereo(t, cam_ids[0], cam_ids[1], pyrs[0], pyrs[1], masks[0], masks[1], db);
  } else {
    for (size_t k = 0; k < images.size(); k++) feed_monocular(t, cam_ids[k], pyrs[k], masks[k], db);
  }
}

}  // namespace orc
