// ORACLE — test infrastructure only (see la.h header).
#include "feat.h"

#include <algorithm>

#include "flip.h"

namespace orc {

thread_local FlipCtl *g_flip = nullptr;

// Feature.cpp:26-49
void Feature::clean_old_measurements(const std::vector<double> &valid_times) {
  for (auto const &pair : timestamps) {
    auto &ts = timestamps[pair.first];
    auto &u = uvs[pair.first];
    auto &un = uvs_norm[pair.first];
    size_t w = 0;
    for (size_t i = 0; i < ts.size(); i++) {
      if (std::find(valid_times.begin(), valid_times.end(), ts[i]) != valid_times.end()) {
        ts[w] = ts[i];
        u[w] = u[i];
        un[w] = un[i];
        w++;
      }
    }
    ts.resize(w);
    u.resize(w);
    un.resize(w);
  }
}

// Feature.cpp:85-111
void Feature::clean_older_measurements(double timestamp) {
  for (auto const &pair : timestamps) {
    auto &ts = timestamps[pair.first];
    auto &u = uvs[pair.first];
    auto &un = uvs_norm[pair.first];
    size_t w = 0;
    for (size_t i = 0; i < ts.size(); i++) {
      if (!(ts[i] <= timestamp)) {
        ts[w] = ts[i];
        u[w] = u[i];
        un[w] = un[i];
        w++;
      }
    }
    ts.resize(w);
    u.resize(w);
    un.resize(w);
  }
}

// FeatureDatabase.cpp:59-85
void FeatureDatabase::update_feature(size_t id, double t, size_t cam, float u, float v, float un, float vn) {
  auto it = features_idlookup.find(id);
  if (it != features_idlookup.end()) {
    auto &f = it->second;
    f->uvs[cam].push_back({u, v});
    f->uvs_norm[cam].push_back({un, vn});
    f->timestamps[cam].push_back(t);
    return;
  }
  auto f = std::make_shared<Feature>();
  f->featid = id;
  f->uvs[cam].push_back({u, v});
  f->uvs_norm[cam].push_back({un, vn});
  f->timestamps[cam].push_back(t);
  features_idlookup[id] = f;
}

// FeatureDatabase.cpp:87-123
std::vector<FeatP> FeatureDatabase::features_not_containing_newer(double timestamp, bool remove, bool skip_deleted) {
  std::vector<FeatP> out;
  for (auto it = features_idlookup.begin(); it != features_idlookup.end();) {
    if (skip_deleted && it->second->to_delete) {
      it++;
      continue;
    }
    bool has_newer = false;
    for (auto const &pair : it->second->timestamps) {
      has_newer = (!pair.second.empty() && pair.second.back() >= timestamp);
      if (has_newer) break;
    }
    if (!has_newer) {
      out.push_back(it->second);
      if (remove)
        features_idlookup.erase(it++);
      else
        it++;
    } else {
      it++;
    }
  }
  return out;
}

// FeatureDatabase.cpp:169-208
std::vector<FeatP> FeatureDatabase::features_containing(double timestamp, bool remove, bool skip_deleted) {
  std::vector<FeatP> out;
  for (auto it = features_idlookup.begin(); it != features_idlookup.end();) {
    if (skip_deleted && it->second->to_delete) {
      it++;
      continue;
    }
    bool has = false;
    for (auto const &pair : it->second->timestamps) {
      has = (std::find(pair.second.begin(), pair.second.end(), timestamp) != pair.second.end());
      if (has) break;
    }
    if (has) {
      out.push_back(it->second);
      if (remove)
        features_idlookup.erase(it++);
      else
        it++;
    } else {
      it++;
    }
  }
  return out;
}

// FeatureDatabase.cpp:211-224
void FeatureDatabase::cleanup() {
  for (auto it = features_idlookup.begin(); it != features_idlookup.end();) {
    if (it->second->to_delete)
      features_idlookup.erase(it++);
    else
      it++;
  }
}

// FeatureDatabase.cpp:226-241
void FeatureDatabase::cleanup_measurements(double timestamp) {
  for (auto it = features_idlookup.begin(); it != features_idlookup.end();) {
    it->second->clean_older_measurements(timestamp);
    int ct = 0;
    for (const auto &pair : it->second->timestamps) ct += (int)pair.second.size();
    if (ct < 1)
      features_idlookup.erase(it++);
    else
      it++;
  }
}

// FeatureInitializer.cpp:30-112
bool FeatureInitializer::single_triangulation(Feature &feat, ClonesCam &clonesCAM) {
  size_t anchor_most_meas = 0, most_meas = 0;
  for (auto const &pair : feat.timestamps) {
    if (pair.second.size() > most_meas) {
      anchor_most_meas = pair.first;
      most_meas = pair.second.size();
    }
  }
  feat.anchor_cam_id = (int)anchor_most_meas;
  feat.anchor_clone_timestamp = feat.timestamps.at(feat.anchor_cam_id).back();
  Mat A(3, 3), b(3, 1);
  const ClonePose &anc = clonesCAM.at(feat.anchor_cam_id).at(feat.anchor_clone_timestamp);
  const Mat &R_GtoA = anc.R, &p_AinG = anc.p;
  for (auto const &pair : feat.timestamps) {
    for (size_t m = 0; m < pair.second.size(); m++) {
      const ClonePose &cp = clonesCAM.at(pair.first).at(pair.second[m]);
      Mat R_AtoCi = cp.R * R_GtoA.T();
      Mat p_CiinA = R_GtoA * (cp.p - p_AinG);
      auto un = feat.uvs_norm.at(pair.first)[m];
      Mat b_i = V3(un.first, un.second, 1);
      b_i = R_AtoCi.T() * b_i;
      b_i = (1.0 / norm(b_i)) * b_i;
      Mat Bperp = skew_x(b_i);
      Mat Ai = Bperp.T() * Bperp;
      A = A + Ai;
      b = b + Ai * p_CiinA;
    }
  }
  Mat p_f = colpiv_qr_solve(A, b);
  double sv[3];
  singular_values3(A, sv);
  double condA = sv[0] / sv[2];
  if (std::abs(condA) > o.fi_max_cond_number || p_f[2] < o.fi_min_dist || p_f[2] > o.fi_max_dist ||
      std::isnan(norm(p_f)))
    return false;
  feat.p_FinA = p_f;
  feat.p_FinG = R_GtoA.T() * feat.p_FinA + p_AinG;
  return true;
}

// FeatureInitializer.cpp:114-195
bool FeatureInitializer::single_triangulation_1d(Feature &feat, ClonesCam &clonesCAM) {
  size_t anchor_most_meas = 0, most_meas = 0;
  for (auto const &pair : feat.timestamps) {
    if (pair.second.size() > most_meas) {
      anchor_most_meas = pair.first;
      most_meas = pair.second.size();
    }
  }
  feat.anchor_cam_id = (int)anchor_most_meas;
  feat.anchor_clone_timestamp = feat.timestamps.at(feat.anchor_cam_id).back();
  size_t idx_anchor = feat.timestamps.at(feat.anchor_cam_id).size() - 1;
  double A = 0, b = 0;
  const ClonePose &anc = clonesCAM.at(feat.anchor_cam_id).at(feat.anchor_clone_timestamp);
  const Mat &R_GtoA = anc.R, &p_AinG = anc.p;
  auto un0 = feat.uvs_norm.at(feat.anchor_cam_id)[idx_anchor];
  Mat bearing = V3(un0.first, un0.second, 1);
  bearing = (1.0 / norm(bearing)) * bearing;
  for (auto const &pair : feat.timestamps) {
    for (size_t m = 0; m < pair.second.size(); m++) {
      if ((int)pair.first == feat.anchor_cam_id && m == idx_anchor) continue;
      const ClonePose &cp = clonesCAM.at(pair.first).at(pair.second[m]);
      Mat R_AtoCi = cp.R * R_GtoA.T();
      Mat p_CiinA = R_GtoA * (cp.p - p_AinG);
      auto un = feat.uvs_norm.at(pair.first)[m];
      Mat b_i = V3(un.first, un.second, 1);
      b_i = R_AtoCi.T() * b_i;
      b_i = (1.0 / norm(b_i)) * b_i;
      Mat Bperp = skew_x(b_i);
      Mat BB = Bperp * bearing;
      A += dot(BB, BB);
      b += dot(BB, Bperp * p_CiinA);
    }
  }
  double depth = b / A;
  Mat p_f = depth * bearing;
  if (p_f[2] < o.fi_min_dist || p_f[2] > o.fi_max_dist || std::isnan(norm(p_f))) return false;
  feat.p_FinA = p_f;
  feat.p_FinG = R_GtoA.T() * feat.p_FinA + p_AinG;
  return true;
}

// FeatureInitializer.cpp:377-423 (residuals in float, as in the reference)
double FeatureInitializer::compute_error(ClonesCam &clonesCAM, Feature &feat, double alpha, double beta, double rho) {
  double err = 0;
  const ClonePose &anc = clonesCAM.at(feat.anchor_cam_id).at(feat.anchor_clone_timestamp);
  const Mat &R_GtoA = anc.R, &p_AinG = anc.p;
  for (auto const &pair : feat.timestamps) {
    for (size_t m = 0; m < pair.second.size(); m++) {
      const ClonePose &cp = clonesCAM.at(pair.first).at(pair.second[m]);
      Mat R_AtoCi = cp.R * R_GtoA.T();
      Mat p_CiinA = R_GtoA * (cp.p - p_AinG);
      Mat p_AinCi = -(R_AtoCi * p_CiinA);
      double hi1 = R_AtoCi(0, 0) * alpha + R_AtoCi(0, 1) * beta + R_AtoCi(0, 2) + rho * p_AinCi[0];
      double hi2 = R_AtoCi(1, 0) * alpha + R_AtoCi(1, 1) * beta + R_AtoCi(1, 2) + rho * p_AinCi[1];
      double hi3 = R_AtoCi(2, 0) * alpha + R_AtoCi(2, 1) * beta + R_AtoCi(2, 2) + rho * p_AinCi[2];
      float z1 = fcast(hi1 / hi3), z2 = fcast(hi2 / hi3);
      auto un = feat.uvs_norm.at(pair.first)[m];
      float r1 = un.first - z1, r2 = un.second - z2;
      float nrm = std::sqrt(r1 * r1 + r2 * r2);
      err += std::pow((double)nrm, 2);
    }
  }
  return err;
}

// FeatureInitializer.cpp:197-375
bool FeatureInitializer::single_gaussnewton(Feature &feat, ClonesCam &clonesCAM) {
  double rho = 1 / feat.p_FinA[2];
  double alpha = feat.p_FinA[0] / feat.p_FinA[2];
  double beta = feat.p_FinA[1] / feat.p_FinA[2];
  double lam = o.fi_init_lamda;
  double eps = 10000;
  int runs = 0;
  bool recompute = true;
  Mat Hess(3, 3), grad(3, 1);
  double cost_old = compute_error(clonesCAM, feat, alpha, beta, rho);
  const ClonePose &anc = clonesCAM.at(feat.anchor_cam_id).at(feat.anchor_clone_timestamp);
  const Mat R_GtoA = anc.R, p_AinG = anc.p;
  while (runs < o.fi_max_runs && lam < o.fi_max_lamda && eps > o.fi_min_dx) {
    if (recompute) {
      Hess = Mat(3, 3);
      grad = Mat(3, 1);
      for (auto const &pair : feat.timestamps) {
        for (size_t m = 0; m < pair.second.size(); m++) {
          const ClonePose &cp = clonesCAM.at(pair.first).at(pair.second[m]);
          Mat R_AtoCi = cp.R * R_GtoA.T();
          Mat p_CiinA = R_GtoA * (cp.p - p_AinG);
          Mat p_AinCi = -(R_AtoCi * p_CiinA);
          double hi1 = R_AtoCi(0, 0) * alpha + R_AtoCi(0, 1) * beta + R_AtoCi(0, 2) + rho * p_AinCi[0];
          double hi2 = R_AtoCi(1, 0) * alpha + R_AtoCi(1, 1) * beta + R_AtoCi(1, 2) + rho * p_AinCi[1];
          double hi3 = R_AtoCi(2, 0) * alpha + R_AtoCi(2, 1) * beta + R_AtoCi(2, 2) + rho * p_AinCi[2];
          double h3s = std::pow(hi3, 2);
          Mat H(2, 3);
          H(0, 0) = (R_AtoCi(0, 0) * hi3 - hi1 * R_AtoCi(2, 0)) / h3s;
          H(0, 1) = (R_AtoCi(0, 1) * hi3 - hi1 * R_AtoCi(2, 1)) / h3s;
          H(0, 2) = (p_AinCi[0] * hi3 - hi1 * p_AinCi[2]) / h3s;
          H(1, 0) = (R_AtoCi(1, 0) * hi3 - hi2 * R_AtoCi(2, 0)) / h3s;
          H(1, 1) = (R_AtoCi(1, 1) * hi3 - hi2 * R_AtoCi(2, 1)) / h3s;
          H(1, 2) = (p_AinCi[1] * hi3 - hi2 * p_AinCi[2]) / h3s;
          float z1 = fcast(hi1 / hi3), z2 = fcast(hi2 / hi3);
          auto un = feat.uvs_norm.at(pair.first)[m];
          float r1 = un.first - z1, r2 = un.second - z2;
          Mat res(2, 1);
          res[0] = (double)r1;
          res[1] = (double)r2;
          grad = grad + H.T() * res;
          Hess = Hess + H.T() * H;
        }
      }
    }
    Mat Hess_l = Hess;
    for (int r = 0; r < 3; r++) Hess_l(r, r) *= (1.0 + lam);
    Mat dx = colpiv_qr_solve(Hess_l, grad);
    double cost = compute_error(clonesCAM, feat, alpha + dx[0], beta + dx[1], rho + dx[2]);
    if (cost <= cost_old && (cost_old - cost) / cost_old < o.fi_min_dcost) {
      alpha += dx[0];
      beta += dx[1];
      rho += dx[2];
      eps = 0;
      break;
    }
    if (cost <= cost_old) {
      recompute = true;
      cost_old = cost;
      alpha += dx[0];
      beta += dx[1];
      rho += dx[2];
      runs++;
      lam = lam / o.fi_lam_mult;
      eps = norm(dx);
    } else {
      recompute = false;
      lam = lam * o.fi_lam_mult;
      continue;
    }
  }
  feat.p_FinA[0] = alpha / rho;
  feat.p_FinA[1] = beta / rho;
  feat.p_FinA[2] = 1 / rho;
  // Max baseline: ||Q(:,1:2)^T p_CiinA|| with Q from HouseholderQR(p_FinA) == the norm of the
  // component of p_CiinA orthogonal to p_FinA (basis-independent).
  Mat vhat = (1.0 / norm(feat.p_FinA)) * feat.p_FinA;
  double base_line_max = 0.0;
  for (auto const &pair : feat.timestamps) {
    for (size_t m = 0; m < pair.second.size(); m++) {
      const ClonePose &cp = clonesCAM.at(pair.first).at(pair.second[m]);
      Mat p_CiinA = R_GtoA * (cp.p - p_AinG);
      Mat perp = p_CiinA - dot(p_CiinA, vhat) * vhat;
      double base_line = norm(perp);
      if (base_line > base_line_max) base_line_max = base_line;
    }
  }
  if (feat.p_FinA[2] < o.fi_min_dist || feat.p_FinA[2] > o.fi_max_dist ||
      (norm(feat.p_FinA) / base_line_max) > o.fi_max_baseline || std::isnan(norm(feat.p_FinA)))
    return false;
  feat.p_FinG = R_GtoA.T() * feat.p_FinA + p_AinG;
  return true;
}

}  // namespace orc
