// Engine: IMU propagation.  The mean integration and the (15+intrinsics)-sized state transition /
// noise accumulation run on the host (a serial chain of ~10 IMU intervals of 15x15 math per frame);
// the N x 15 covariance propagation and cloning run on the device.
// Reference: Propagator.cpp:33-138 (propagate_and_clone), :269-393 (select_imu_readings),
// :395-480 (predict_and_compute), :507-586 (RK4), :588-665 (Xi_sum), :683-962 (F, G),
// :964-1015 (H_Dw/H_Da/H_Tg); UVioPropagator.cpp:27-115.
#include <algorithm>
#include <cstring>

#include "engine.h"

namespace uvhp {

namespace {

// small dense row-major helpers
struct Mx {
  int r, c;
  std::vector<double> d;
  Mx(int r_ = 0, int c_ = 0) : r(r_), c(c_), d((size_t)r_ * c_, 0.0) {}
  double &operator()(int i, int j) { return d[(size_t)i * c + j]; }
  double operator()(int i, int j) const { return d[(size_t)i * c + j]; }
};
Mx mul(const Mx &A, const Mx &B) {
  Mx C(A.r, B.c);
  for (int i = 0; i < A.r; i++)
    for (int k = 0; k < A.c; k++) {
      double a = A(i, k);
      if (a == 0.0) continue;
      for (int j = 0; j < B.c; j++) C(i, j) += a * B(k, j);
    }
  return C;
}
Mx mulT(const Mx &A, const Mx &B) {  // A * B^T
  // B's nonzero columns per row, once: F and G of the IMU propagation are mostly zero (39 x 39 with the IMU
  // intrinsics and g-sensitivity), and a zero term adds nothing to the ascending-k sum, so skipping it leaves
  // every C(i, j) bit-identical (finite operands)
  std::vector<int> nzk;
  std::vector<int> nzo(B.r + 1, 0);
  nzk.reserve((size_t)B.r * B.c);
  for (int j = 0; j < B.r; j++) {
    for (int k = 0; k < B.c; k++)
      if (B(j, k) != 0.0) nzk.push_back(k);
    nzo[j + 1] = (int)nzk.size();
  }
  Mx C(A.r, B.r);
  for (int i = 0; i < A.r; i++)
    for (int j = 0; j < B.r; j++) {
      double s = 0;
      for (int e = nzo[j]; e < nzo[j + 1]; e++) {
        const int k = nzk[e];
        s += A(i, k) * B(j, k);
      }
      C(i, j) = s;
    }
  return C;
}
void setb(Mx &M, int i0, int j0, const double *b33, double s = 1.0) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) M(i0 + i, j0 + j) = s * b33[3 * i + j];
}
void setb36(Mx &M, int i0, int j0, const double *b, int nc, double s = 1.0) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < nc; j++) M(i0 + i, j0 + j) = s * b[nc * i + j];
}
// 3x3 helpers
void M3(const double *A, const double *B, double *C) { m3_mul(A, B, C); }
void M3s(double s, const double *A, double *C) {
  for (int i = 0; i < 9; i++) C[i] = s * A[i];
}
void M3add(const double *A, const double *B, double *C) {
  for (int i = 0; i < 9; i++) C[i] = A[i] + B[i];
}
void eye3(double *I) {
  for (int i = 0; i < 9; i++) I[i] = (i % 4 == 0) ? 1.0 : 0.0;
}
// 3 x nc = A(3x3) * B(3 x nc)
void M3xN(const double *A, const double *B, int nc, double *C) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < nc; j++) C[nc * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[nc + j] + A[3 * i + 2] * B[2 * nc + j];
}

void exp_so3(const double *w, double *R) {
  double th = norm3(w), A, B;
  if (th < 1e-7) {
    A = 1;
    B = 0.5;
  } else {
    A = sin(th) / th;
    B = (1 - cos(th)) / (th * th);
  }
  if (th == 0) {
    eye3(R);
    return;
  }
  double S[9], S2[9];
  skew(w, S);
  M3(S, S, S2);
  for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0) ? 1.0 : 0.0) + A * S[i] + B * S2[i];
}
void Jl_so3(const double *w, double *J) {
  double th = norm3(w);
  if (th < 1e-6) {
    eye3(J);
    return;
  }
  double a[3] = {w[0] / th, w[1] / th, w[2] / th}, S[9];
  skew(a, S);
  double c1 = sin(th) / th, c2 = 1 - sin(th) / th, c3 = (1 - cos(th)) / th;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) J[3 * i + j] = ((i == j) ? c1 : 0.0) + c2 * a[i] * a[j] + c3 * S[3 * i + j];
}
void log_so3(const double *R, double *w) {
  double R11 = R[0], R12 = R[1], R13 = R[2], R21 = R[3], R22 = R[4], R23 = R[5], R31 = R[6], R32 = R[7], R33 = R[8];
  double tr = R11 + R22 + R33;
  if (tr + 1.0 < 1e-10) {
    if (std::abs(R33 + 1.0) > 1e-5) {
      double s = M_PI / sqrt(2.0 + 2.0 * R33);
      w[0] = s * R13; w[1] = s * R23; w[2] = s * (1.0 + R33);
    } else if (std::abs(R22 + 1.0) > 1e-5) {
      double s = M_PI / sqrt(2.0 + 2.0 * R22);
      w[0] = s * R12; w[1] = s * (1.0 + R22); w[2] = s * R32;
    } else {
      double s = M_PI / sqrt(2.0 + 2.0 * R11);
      w[0] = s * (1.0 + R11); w[1] = s * R21; w[2] = s * R31;
    }
  } else {
    double mag, tr_3 = tr - 3.0;
    if (tr_3 < -1e-7) {
      double th = acos((tr - 1.0) / 2.0);
      mag = th / (2.0 * sin(th));
    } else {
      mag = 0.5 - tr_3 / 12.0;
    }
    w[0] = mag * (R32 - R23); w[1] = mag * (R13 - R31); w[2] = mag * (R21 - R12);
  }
}

// State::Dm / State::Tg (State.h:92-111)
void Dm(int model, const double *v, double *D) {
  for (int i = 0; i < 9; i++) D[i] = 0;
  if (model == 0) {
    D[0] = v[0];
    D[3] = v[1]; D[4] = v[3];
    D[6] = v[2]; D[7] = v[4]; D[8] = v[5];
  } else {
    D[0] = v[0]; D[1] = v[1]; D[2] = v[3];
    D[4] = v[2]; D[5] = v[4];
    D[8] = v[5];
  }
}
void TgM(const double *v, double *T) {
  T[0] = v[0]; T[1] = v[3]; T[2] = v[6];
  T[3] = v[1]; T[4] = v[4]; T[5] = v[7];
  T[6] = v[2]; T[7] = v[5]; T[8] = v[8];
}
// compute_H_Dw / compute_H_Da (3x6), compute_H_Tg (3x9)
void H_D(int model, const double *w, double *H) {
  for (int i = 0; i < 18; i++) H[i] = 0;
  if (model == 0) {
    H[0 * 6 + 0] = w[0]; H[1 * 6 + 1] = w[0]; H[2 * 6 + 2] = w[0];
    H[1 * 6 + 3] = w[1]; H[2 * 6 + 4] = w[1]; H[2 * 6 + 5] = w[2];
  } else {
    H[0 * 6 + 0] = w[0]; H[0 * 6 + 1] = w[1]; H[1 * 6 + 2] = w[1];
    H[0 * 6 + 3] = w[2]; H[1 * 6 + 4] = w[2]; H[2 * 6 + 5] = w[2];
  }
}
void H_Tg(const double *a, double *H) {
  for (int i = 0; i < 27; i++) H[i] = 0;
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) H[9 * i + 3 * k + i] = a[k];
}

}  // namespace

std::vector<ImuSample> Engine::select_imu_readings(double time0, double time1) {
  std::vector<ImuSample> imu;
  {
    std::lock_guard<std::mutex> lk(imu_mtx_);
    imu = imu_data_;
  }
  return select_imu(imu, time0, time1);
}

// Propagator::select_imu_readings (Propagator.cpp:269-393) on a given buffer
std::vector<ImuSample> Engine::select_imu(const std::vector<ImuSample> &imu, double time0, double time1) {
  auto interp = [](const ImuSample &a, const ImuSample &b, double t) {
    double lambda = (t - a.t) / (b.t - a.t);
    ImuSample d;
    d.t = t;
    for (int k = 0; k < 3; k++) {
      d.am[k] = (1 - lambda) * a.am[k] + lambda * b.am[k];
      d.wm[k] = (1 - lambda) * a.wm[k] + lambda * b.wm[k];
    }
    return d;
  };
  std::vector<ImuSample> prop;
  if (imu.empty()) return prop;
  for (size_t i = 0; i < imu.size() - 1; i++) {
    if (imu[i + 1].t > time0 && imu[i].t < time0) {
      prop.push_back(interp(imu[i], imu[i + 1], time0));
      continue;
    }
    if (imu[i].t >= time0 && imu[i + 1].t <= time1) {
      prop.push_back(imu[i]);
      continue;
    }
    if (imu[i + 1].t > time1) {
      if (imu[i].t > time1 && i == 0) {
        break;
      } else if (imu[i].t > time1) {
        prop.push_back(interp(imu[i - 1], imu[i], time1));
      } else {
        prop.push_back(imu[i]);
      }
      if (prop.back().t != time1) prop.push_back(interp(imu[i], imu[i + 1], time1));
      break;
    }
  }
  if (prop.empty()) return prop;
  if (prop.back().t != time1) prop.push_back(interp(imu[imu.size() - 2], imu[imu.size() - 1], time1));
  for (size_t i = 0; i + 1 < prop.size(); i++)
    if (std::abs(prop[i + 1].t - prop[i].t) < 1e-12) {
      prop.erase(prop.begin() + i);
      i--;
    }
  return prop;
}

void Engine::predict_and_compute(const ImuSample &dm, const ImuSample &dp, double *Fout, double *Qdout, int n) {
  const double dt = dp.t - dm.t;
  double Dw[9], Da[9], Tg[9], Ra[9], Rw[9];
  Dm(o_.imu_model, dw_->val, Dw);
  Dm(o_.imu_model, da_->val, Da);
  TgM(tg_->val, Tg);
  quat_2_Rot(qa_->val, Ra);
  quat_2_Rot(qg_->val, Rw);
  const double *bg = imu_->val + 10, *ba = imu_->val + 13;
  double a1[3], a2[3], aavg[3], aunc[3];
  for (int k = 0; k < 3; k++) {
    a1[k] = dm.am[k] - ba[k];
    a2[k] = dp.am[k] - ba[k];
    aavg[k] = .5 * (a1[k] + a2[k]);
    aunc[k] = aavg[k];
  }
  double RaDa[9], t3[3];
  M3(Ra, Da, RaDa);
  m3_vec(RaDa, a1, t3); std::memcpy(a1, t3, sizeof(t3));
  m3_vec(RaDa, a2, t3); std::memcpy(a2, t3, sizeof(t3));
  m3_vec(RaDa, aavg, t3); std::memcpy(aavg, t3, sizeof(t3));
  double w1[3], w2[3], wavg[3], wunc[3], Ta1[3], Ta2[3];
  m3_vec(Tg, a1, Ta1);
  m3_vec(Tg, a2, Ta2);
  for (int k = 0; k < 3; k++) {
    w1[k] = dm.wm[k] - bg[k] - Ta1[k];
    w2[k] = dp.wm[k] - bg[k] - Ta2[k];
    wavg[k] = .5 * (w1[k] + w2[k]);
    wunc[k] = wavg[k];
  }
  double RwDw[9];
  M3(Rw, Dw, RwDw);
  m3_vec(RwDw, w1, t3); std::memcpy(w1, t3, sizeof(t3));
  m3_vec(RwDw, w2, t3); std::memcpy(w2, t3, sizeof(t3));
  m3_vec(RwDw, wavg, t3); std::memcpy(wavg, t3, sizeof(t3));
  const double g[3] = {0, 0, o_.gravity_mag};

  // ---- Xi_sum (Propagator.cpp:588-665) ----
  double R_ktok1[9], Xi1[9], Xi2[9], Jr[9], Xi3[9], Xi4[9];
  bool use_xi = (o_.integration == 1 || o_.integration == 2);
  if (use_xi) {
    double w_norm = norm3(wavg), d_th = w_norm * dt;
    double k_hat[3] = {0, 0, 0};
    if (w_norm > 1e-12)
      for (int k = 0; k < 3; k++) k_hat[k] = wavg[k] / w_norm;
    double I3[9];
    eye3(I3);
    double d_t2 = dt * dt, d_t3 = dt * dt * dt, w2n = w_norm * w_norm, w3n = w2n * w_norm;
    double cs = cos(d_th), sn = sin(d_th), dth2 = d_th * d_th, dth3 = dth2 * d_th;
    double sK[9], sK2[9], sA[9];
    skew(k_hat, sK);
    M3(sK, sK, sK2);
    skew(aavg, sA);
    double mw[3] = {-wavg[0] * dt, -wavg[1] * dt, -wavg[2] * dt};
    exp_so3(mw, R_ktok1);
    double pw[3] = {wavg[0] * dt, wavg[1] * dt, wavg[2] * dt};
    Jl_so3(pw, Jr);  // Jr(-w dt) = Jl(w dt)
    double ka = dot3(k_hat, aavg);
    double sAsK[9], sKsA[9], sAsK2[9], sK2sA[9];
    M3(sA, sK, sAsK);
    M3(sK, sA, sKsA);
    M3(sA, sK2, sAsK2);
    M3(sK2, sA, sK2sA);
    bool small_w = (w_norm < 1.0 / 180 * M_PI / 2);
    for (int i = 0; i < 9; i++) {
      if (!small_w) {
        Xi1[i] = dt * I3[i] + ((1.0 - cs) / w_norm) * sK[i] + (dt - sn / w_norm) * sK2[i];
        Xi2[i] = (1.0 / 2 * d_t2) * I3[i] + ((d_th - sn) / w2n) * sK[i] + (1.0 / 2 * d_t2 - (1.0 - cs) / w2n) * sK2[i];
        Xi3[i] = (1.0 / 2 * d_t2) * sA[i] + ((sn - d_th) / w2n) * sAsK[i] + ((sn - d_th * cs) / w2n) * sKsA[i] +
                 (1.0 / 2 * d_t2 - (1.0 - cs) / w2n) * sAsK2[i] +
                 (1.0 / 2 * d_t2 + (1.0 - cs - d_th * sn) / w2n) * (sK2sA[i] + ka * sK[i]) -
                 ((3 * sn - 2 * d_th - d_th * cs) / w2n * ka) * sK2[i];
        Xi4[i] = (1.0 / 6 * d_t3) * sA[i] + ((2 * (1.0 - cs) - dth2) / (2 * w3n)) * sAsK[i] +
                 ((2 * (1.0 - cs) - d_th * sn) / w3n) * sKsA[i] + ((sn - d_th) / w3n + d_t3 / 6) * sAsK2[i] +
                 ((d_th - 2 * sn + 1.0 / 6 * dth3 + d_th * cs) / w3n) * (sK2sA[i] + ka * sK[i]) +
                 ((4 * cs - 4 + dth2 + d_th * sn) / w3n * ka) * sK2[i];
      } else {
        Xi1[i] = dt * (I3[i] + sn * sK[i] + (1.0 - cs) * sK2[i]);
      }
    }
    if (small_w)
      for (int i = 0; i < 9; i++) {
        Xi2[i] = (1.0 / 2 * dt) * Xi1[i];
        Xi3[i] = (1.0 / 2 * d_t2) * (sA[i] + sn * (-sAsK[i] + sKsA[i] + ka * sK2[i]) +
                                      (1.0 - cs) * (sAsK2[i] + sK2sA[i] + ka * sK[i]));
        Xi4[i] = (1.0 / 3 * dt) * Xi3[i];
      }
  }

  // ---- mean ----
  double *q0 = imu_->val, *p0 = imu_->val + 4, *v0 = imu_->val + 7;
  double nq[4], np[3], nv[3];
  double Rk0[9];
  quat_2_Rot(q0, Rk0);
  if (o_.integration == 2) {
    double qk[4];
    rot_2_quat(R_ktok1, qk);
    quat_multiply(qk, q0, nq);
    double t1[3], t2[3];
    m3_vec(Xi1, aavg, t1);
    m3t_vec(Rk0, t1, t2);
    for (int k = 0; k < 3; k++) nv[k] = v0[k] + t2[k] - g[k] * dt;
    m3_vec(Xi2, aavg, t1);
    m3t_vec(Rk0, t1, t2);
    for (int k = 0; k < 3; k++) np[k] = p0[k] + v0[k] * dt + t2[k] - 0.5 * g[k] * dt * dt;
  } else if (o_.integration == 1) {
    // predict_mean_rk4 (Propagator.cpp:507-586)
    double w_hat[3] = {w1[0], w1[1], w1[2]}, a_hat[3] = {a1[0], a1[1], a1[2]};
    double w_alpha[3], a_jerk[3];
    for (int k = 0; k < 3; k++) {
      w_alpha[k] = (w2[k] - w1[k]) / dt;
      a_jerk[k] = (a2[k] - a1[k]) / dt;
    }
    double dq0[4] = {0, 0, 0, 1};
    auto qdot = [](const double *w, const double *dq, double *o) {
      // 0.5 * Omega(w) * dq ; Omega = [-skew(w) w; -w^T 0]
      o[0] = 0.5 * (0 * dq[0] + w[2] * dq[1] - w[1] * dq[2] + w[0] * dq[3]);
      o[1] = 0.5 * (-w[2] * dq[0] + 0 * dq[1] + w[0] * dq[2] + w[1] * dq[3]);
      o[2] = 0.5 * (w[1] * dq[0] - w[0] * dq[1] + 0 * dq[2] + w[2] * dq[3]);
      o[3] = 0.5 * (-w[0] * dq[0] - w[1] * dq[1] - w[2] * dq[2]);
    };
    auto vdot = [&](const double *dq, const double *a, double *o) {
      double qq[4], R[9], t[3];
      quat_multiply(dq, q0, qq);
      quat_2_Rot(qq, R);
      m3t_vec(R, a, t);
      for (int k = 0; k < 3; k++) o[k] = t[k] - g[k];
    };
    double k1q[4], k1p[3], k1v[3], k2q[4], k2p[3], k2v[3], k3q[4], k3p[3], k3v[3], k4q[4], k4p[3], k4v[3];
    double qd[4], vd[3];
    qdot(w_hat, dq0, qd);
    vdot(dq0, a_hat, vd);
    for (int k = 0; k < 4; k++) k1q[k] = qd[k] * dt;
    for (int k = 0; k < 3; k++) k1p[k] = v0[k] * dt, k1v[k] = vd[k] * dt;
    for (int k = 0; k < 3; k++) w_hat[k] += 0.5 * w_alpha[k] * dt, a_hat[k] += 0.5 * a_jerk[k] * dt;
    double dq1[4], v1[3];
    for (int k = 0; k < 4; k++) dq1[k] = dq0[k] + 0.5 * k1q[k];
    quatnorm(dq1);
    for (int k = 0; k < 3; k++) v1[k] = v0[k] + 0.5 * k1v[k];
    qdot(w_hat, dq1, qd);
    vdot(dq1, a_hat, vd);
    for (int k = 0; k < 4; k++) k2q[k] = qd[k] * dt;
    for (int k = 0; k < 3; k++) k2p[k] = v1[k] * dt, k2v[k] = vd[k] * dt;
    double dq2[4], v2[3];
    for (int k = 0; k < 4; k++) dq2[k] = dq0[k] + 0.5 * k2q[k];
    quatnorm(dq2);
    for (int k = 0; k < 3; k++) v2[k] = v0[k] + 0.5 * k2v[k];
    qdot(w_hat, dq2, qd);
    vdot(dq2, a_hat, vd);
    for (int k = 0; k < 4; k++) k3q[k] = qd[k] * dt;
    for (int k = 0; k < 3; k++) k3p[k] = v2[k] * dt, k3v[k] = vd[k] * dt;
    for (int k = 0; k < 3; k++) w_hat[k] += 0.5 * w_alpha[k] * dt, a_hat[k] += 0.5 * a_jerk[k] * dt;
    double dq3[4], v3[3];
    for (int k = 0; k < 4; k++) dq3[k] = dq0[k] + k3q[k];
    quatnorm(dq3);
    for (int k = 0; k < 3; k++) v3[k] = v0[k] + k3v[k];
    qdot(w_hat, dq3, qd);
    vdot(dq3, a_hat, vd);
    for (int k = 0; k < 4; k++) k4q[k] = qd[k] * dt;
    for (int k = 0; k < 3; k++) k4p[k] = v3[k] * dt, k4v[k] = vd[k] * dt;
    double dq[4];
    for (int k = 0; k < 4; k++)
      dq[k] = dq0[k] + (1.0 / 6.0) * k1q[k] + (1.0 / 3.0) * k2q[k] + (1.0 / 3.0) * k3q[k] + (1.0 / 6.0) * k4q[k];
    quatnorm(dq);
    quat_multiply(dq, q0, nq);
    for (int k = 0; k < 3; k++) {
      np[k] = p0[k] + (1.0 / 6.0) * k1p[k] + (1.0 / 3.0) * k2p[k] + (1.0 / 3.0) * k3p[k] + (1.0 / 6.0) * k4p[k];
      nv[k] = v0[k] + (1.0 / 6.0) * k1v[k] + (1.0 / 3.0) * k2v[k] + (1.0 / 3.0) * k3v[k] + (1.0 / 6.0) * k4v[k];
    }
  } else {
    // predict_mean_discrete
    double w_norm = norm3(wavg);
    double O[16] = {0, wavg[2], -wavg[1], wavg[0], -wavg[2], 0, wavg[0], wavg[1],
                    wavg[1], -wavg[0], 0, wavg[2], -wavg[0], -wavg[1], -wavg[2], 0};
    double c0, c1;
    if (w_norm > 1e-12) {
      c0 = cos(0.5 * w_norm * dt);
      c1 = 1 / w_norm * sin(0.5 * w_norm * dt);
    } else {
      c0 = 1;
      c1 = 0.5 * dt;
    }
    for (int i = 0; i < 4; i++) {
      double s = c0 * q0[i];
      for (int j = 0; j < 4; j++) s += c1 * O[4 * i + j] * q0[j];
      nq[i] = s;
    }
    quatnorm(nq);
    double t[3];
    m3t_vec(Rk0, aavg, t);
    for (int k = 0; k < 3; k++) {
      nv[k] = v0[k] + t[k] * dt - g[k] * dt;
      np[k] = p0[k] + v0[k] * dt + 0.5 * t[k] * dt * dt - 0.5 * g[k] * dt * dt;
    }
  }

  // ---- F and G ----
  int th = 0, pi = 3, vi = 6, bgi = 9, bai = 12, ls = 15;
  int Dw_id = -1, Da_id = -1, Tg_id = -1, atoI = -1, wtoI = -1;
  if (o_.do_calib_imu_intrinsics) {
    Dw_id = ls; ls += 6;
    Da_id = ls; ls += 6;
    if (o_.do_calib_imu_g_sensitivity) { Tg_id = ls; ls += 9; }
    if (o_.imu_model == 0) { wtoI = ls; ls += 3; }
    else { atoI = ls; ls += 3; }
  }
  double Rk[9], vk[3], pk[3];
  if (o_.do_fej) {
    quat_2_Rot(imu_->fej, Rk);
    for (int k = 0; k < 3; k++) vk[k] = imu_->fej[7 + k], pk[k] = imu_->fej[4 + k];
  } else {
    std::memcpy(Rk, Rk0, sizeof(Rk));
    for (int k = 0; k < 3; k++) vk[k] = v0[k], pk[k] = p0[k];
  }
  double Rnq[9], dR[9], RkT[9];
  quat_2_Rot(nq, Rnq);
  m3_mul_bt(Rnq, Rk, dR);
  m3_transpose(Rk, RkT);
  double ak[3], wk[3];
  m3_vec(RaDa, aunc, ak);
  m3_vec(RwDw, wunc, wk);
  if (!use_xi) {
    double lw[3];
    log_so3(dR, lw);
    double mlw[3] = {-lw[0], -lw[1], -lw[2]};
    Jl_so3(mlw, Jr);  // Jr_so3(log(dR)) = Jl(-log)
  }
  Mx F(n, n), G(n, 12);
  double I3[9];
  eye3(I3);
  double dRJdt[9], tmp[9], tmp2[9], tmp3[9];
  M3(dR, Jr, tmp);
  M3s(dt, tmp, dRJdt);
  double RwDwTg[9], RwDwTgRaDa[9];
  M3(RwDw, Tg, RwDwTg);
  M3(RwDwTg, RaDa, RwDwTgRaDa);
  setb(F, th, th, dR);
  {
    double v1[3] = {np[0] - pk[0] - vk[0] * dt + 0.5 * g[0] * dt * dt, np[1] - pk[1] - vk[1] * dt + 0.5 * g[1] * dt * dt,
                    np[2] - pk[2] - vk[2] * dt + 0.5 * g[2] * dt * dt};
    skew(v1, tmp);
    M3(tmp, RkT, tmp2);
    setb(F, pi, th, tmp2, -1.0);
    double v2[3] = {nv[0] - vk[0] + g[0] * dt, nv[1] - vk[1] + g[1] * dt, nv[2] - vk[2] + g[2] * dt};
    skew(v2, tmp);
    M3(tmp, RkT, tmp2);
    setb(F, vi, th, tmp2, -1.0);
  }
  setb(F, pi, pi, I3);
  setb(F, pi, vi, I3, dt);
  setb(F, vi, vi, I3);
  setb(F, bgi, bgi, I3);
  setb(F, bai, bai, I3);
  M3(dRJdt, RwDw, tmp);
  setb(F, th, bgi, tmp, -1.0);
  setb(G, th, 0, tmp, -1.0);
  M3(dRJdt, RwDwTgRaDa, tmp);
  setb(F, th, bai, tmp);
  setb(G, th, 3, tmp);
  if (use_xi) {
    M3(Xi4, RwDw, tmp); M3(RkT, tmp, tmp2);
    setb(F, pi, bgi, tmp2); setb(G, pi, 0, tmp2);
    M3(Xi3, RwDw, tmp); M3(RkT, tmp, tmp2);
    setb(F, vi, bgi, tmp2); setb(G, vi, 0, tmp2);
    // -R_k^T (Xi_2 + Xi_4 RwDwTg) RaDa
    M3(Xi4, RwDwTg, tmp); M3add(Xi2, tmp, tmp3); M3(tmp3, RaDa, tmp); M3(RkT, tmp, tmp2);
    setb(F, pi, bai, tmp2, -1.0); setb(G, pi, 3, tmp2, -1.0);
    M3(Xi3, RwDwTg, tmp); M3add(Xi1, tmp, tmp3); M3(tmp3, RaDa, tmp); M3(RkT, tmp, tmp2);
    setb(F, vi, bai, tmp2, -1.0); setb(G, vi, 3, tmp2, -1.0);
  } else {
    M3(RkT, RaDa, tmp);
    setb(F, pi, bai, tmp, -0.5 * dt * dt); setb(G, pi, 3, tmp, -0.5 * dt * dt);
    setb(F, vi, bai, tmp, -dt); setb(G, vi, 3, tmp, -dt);
  }
  double b36[27], b33[9];
  if (Dw_id != -1) {
    double Hd[18];
    H_D(o_.imu_model, wunc, Hd);
    double RwH[18];
    M3xN(Rw, Hd, 6, RwH);
    M3xN(dRJdt, RwH, 6, b36);
    setb36(F, th, Dw_id, b36, 6);
    if (use_xi) {
      M3(RkT, Xi4, tmp); M3xN(tmp, RwH, 6, b36); setb36(F, pi, Dw_id, b36, 6, -1.0);
      M3(RkT, Xi3, tmp); M3xN(tmp, RwH, 6, b36); setb36(F, vi, Dw_id, b36, 6, -1.0);
    }
    for (int k = 0; k < 6; k++) F(Dw_id + k, Dw_id + k) = 1.0;
  }
  if (Da_id != -1) {
    double Hd[18], RaH[18];
    H_D(o_.imu_model, aunc, Hd);
    M3xN(Ra, Hd, 6, RaH);
    if (use_xi) {
      M3(dRJdt, RwDwTg, tmp); M3xN(tmp, RaH, 6, b36); setb36(F, th, Da_id, b36, 6, -1.0);
      M3(Xi4, RwDwTg, tmp); M3add(Xi2, tmp, tmp3); M3(RkT, tmp3, tmp); M3xN(tmp, RaH, 6, b36);
      setb36(F, pi, Da_id, b36, 6);
      M3(Xi3, RwDwTg, tmp); M3add(Xi1, tmp, tmp3); M3(RkT, tmp3, tmp); M3xN(tmp, RaH, 6, b36);
      setb36(F, vi, Da_id, b36, 6);
    } else {
      double RwTg[9];
      M3(Rw, Tg, RwTg);
      M3(dRJdt, RwTg, tmp); M3xN(tmp, RaH, 6, b36); setb36(F, th, Da_id, b36, 6, -1.0);
      M3xN(RkT, RaH, 6, b36); setb36(F, pi, Da_id, b36, 6, 0.5 * dt * dt);
      setb36(F, vi, Da_id, b36, 6, dt);
    }
    for (int k = 0; k < 6; k++) F(Da_id + k, Da_id + k) = 1.0;
  }
  if (Tg_id != -1) {
    double Ht[27];
    H_Tg(ak, Ht);
    M3(dRJdt, RwDw, tmp); M3xN(tmp, Ht, 9, b36); setb36(F, th, Tg_id, b36, 9, -1.0);
    if (use_xi) {
      M3(Xi4, RwDw, tmp2); M3(RkT, tmp2, tmp); M3xN(tmp, Ht, 9, b36); setb36(F, pi, Tg_id, b36, 9);
      M3(Xi3, RwDw, tmp2); M3(RkT, tmp2, tmp); M3xN(tmp, Ht, 9, b36); setb36(F, vi, Tg_id, b36, 9);
    }
    for (int k = 0; k < 9; k++) F(Tg_id + k, Tg_id + k) = 1.0;
  }
  if (atoI != -1) {
    double sa[9];
    skew(ak, sa);
    M3(dRJdt, RwDwTg, tmp); M3(tmp, sa, b33); setb(F, th, atoI, b33, -1.0);
    if (use_xi) {
      M3(Xi4, RwDwTg, tmp); M3add(Xi2, tmp, tmp3); M3(RkT, tmp3, tmp); M3(tmp, sa, b33); setb(F, pi, atoI, b33);
      M3(Xi3, RwDwTg, tmp); M3add(Xi1, tmp, tmp3); M3(RkT, tmp3, tmp); M3(tmp, sa, b33); setb(F, vi, atoI, b33);
    } else {
      M3(RkT, sa, b33);
      setb(F, pi, atoI, b33, 0.5 * dt * dt);
      setb(F, vi, atoI, b33, dt);
    }
    setb(F, atoI, atoI, I3);
  }
  if (wtoI != -1) {
    double sw[9];
    skew(wk, sw);
    M3(dRJdt, sw, b33); setb(F, th, wtoI, b33);
    if (use_xi) {
      M3(RkT, Xi4, tmp); M3(tmp, sw, b33); setb(F, pi, wtoI, b33, -1.0);
      M3(RkT, Xi3, tmp); M3(tmp, sw, b33); setb(F, vi, wtoI, b33, -1.0);
    }
    setb(F, wtoI, wtoI, I3);
  }
  setb(G, bgi, 6, I3, dt);
  setb(G, bai, 9, I3, dt);
  // Qd = G Qc G^T, symmetrized
  Mx Qc(12, 12);
  for (int k = 0; k < 3; k++) {
    Qc(k, k) = o_.sigma_w * o_.sigma_w / dt;
    Qc(3 + k, 3 + k) = o_.sigma_a * o_.sigma_a / dt;
    Qc(6 + k, 6 + k) = o_.sigma_wb * o_.sigma_wb / dt;
    Qc(9 + k, 9 + k) = o_.sigma_ab * o_.sigma_ab / dt;
  }
  Mx GQ = mul(G, Qc);  // (zero G entries skipped: Qc is diagonal, so this is G(i, j) Qc(j, j))
  Mx Qd = mulT(GQ, G);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) Qdout[(size_t)i * n + j] = 0.5 * (Qd(i, j) + Qd(j, i));
  std::memcpy(Fout, F.d.data(), sizeof(double) * n * n);
  // state / fej <- propagated values
  for (int k = 0; k < 4; k++) imu_->val[k] = nq[k];
  for (int k = 0; k < 3; k++) imu_->val[4 + k] = np[k], imu_->val[7 + k] = nv[k];
  std::memcpy(imu_->fej, imu_->val, sizeof(double) * 16);
}

void Engine::accumulate_phi(const std::vector<ImuSample> &prop, std::vector<double> &Phi, std::vector<double> &Qd, int n) {
  // Propagator.cpp:87-130: Phi = F Phi, Qd = F Qd F^T + Qdi, symmetrized, per IMU interval.  F is mostly zero (39 x
  // 39 with the IMU intrinsics and g-sensitivity), so the products run over its nonzeros (one compressed-row list
  // per interval) in the order mul / mulT sum them (ascending k, zero terms skipped, which add nothing): the same
  // bits, without the per-interval allocations of dense temporaries
  const size_t nn = (size_t)n * n;
  std::vector<double> P(nn, 0.0), Q(nn, 0.0), F(nn), Qi(nn), T(nn), T2(nn);
  for (int i = 0; i < n; i++) P[(size_t)i * n + i] = 1.0;
  std::vector<int> nzk(nn), nzo(n + 1);
  std::vector<double> nzv(nn);
  auto f_times = [&](const std::vector<double> &B, std::vector<double> &C) {  // C = F B
    for (int i = 0; i < n; i++) {
      double *c = C.data() + (size_t)i * n;
      for (int j = 0; j < n; j++) c[j] = 0.0;
      for (int e = nzo[i]; e < nzo[i + 1]; e++) {
        const double a = nzv[e];
        const double *b = B.data() + (size_t)nzk[e] * n;
        for (int j = 0; j < n; j++) c[j] += a * b[j];
      }
    }
  };
  if (prop.size() > 1) {
    for (size_t s = 0; s + 1 < prop.size(); s++) {
      predict_and_compute(prop[s], prop[s + 1], F.data(), Qi.data(), n);
      int m = 0;
      for (int i = 0; i < n; i++) {
        nzo[i] = m;
        for (int k = 0; k < n; k++) {
          const double v = F[(size_t)i * n + k];
          if (v != 0.0) nzk[m] = k, nzv[m++] = v;
        }
      }
      nzo[n] = m;
      f_times(P, T);
      P.swap(T);
      f_times(Q, T);  // F Q
      for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) {  // (F Q) F^T + Qdi
          double sum = 0;
          for (int e = nzo[b]; e < nzo[b + 1]; e++) sum += T[(size_t)a * n + nzk[e]] * nzv[e];
          T2[(size_t)a * n + b] = sum + Qi[(size_t)a * n + b];
        }
      for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) Q[(size_t)a * n + b] = 0.5 * (T2[(size_t)a * n + b] + T2[(size_t)b * n + a]);
    }
  }
  Phi.swap(P);
  Qd.swap(Q);
}

void Engine::last_w(const std::vector<ImuSample> &prop, double *w) {
  w[0] = w[1] = w[2] = 0;
  if (prop.empty()) return;
  double Dw[9], Da[9], Tg[9], Ra[9], Rw[9];
  Dm(o_.imu_model, dw_->val, Dw);
  Dm(o_.imu_model, da_->val, Da);
  TgM(tg_->val, Tg);
  quat_2_Rot(qa_->val, Ra);
  quat_2_Rot(qg_->val, Rw);
  const ImuSample &L = prop.back();
  double a[3], t[3], la[3], RaDa[9], RwDw[9];
  for (int k = 0; k < 3; k++) a[k] = L.am[k] - imu_->val[13 + k];
  M3(Ra, Da, RaDa);
  m3_vec(RaDa, a, la);
  m3_vec(Tg, la, t);
  double ww[3];
  for (int k = 0; k < 3; k++) ww[k] = L.wm[k] - imu_->val[10 + k] - t[k];
  M3(Rw, Dw, RwDw);
  m3_vec(RwDw, ww, w);
}

std::vector<int> Engine::phi_order_ids(int *n) {
  std::vector<VarP> order = {imu_};
  if (o_.do_calib_imu_intrinsics) {
    order.push_back(dw_);
    order.push_back(da_);
    if (o_.do_calib_imu_g_sensitivity) order.push_back(tg_);
    order.push_back(o_.imu_model == 0 ? qg_ : qa_);
  }
  std::vector<int> ids;
  for (auto &v : order)
    for (int k = 0; k < v->size; k++) ids.push_back(v->id + k);
  *n = (int)ids.size();
  return ids;
}

int Engine::propagate_and_clone(double timestamp) {
  stage_ = "Propagator::propagate_and_clone";
  if (timestamp_ >= timestamp) return UVIO_HP_E_ORDER;
  if (!have_last_prop_time_offset_) {
    last_prop_time_offset_ = calib_dt_->val[0];
    have_last_prop_time_offset_ = true;
  }
  double t_off_new = calib_dt_->val[0];
  std::vector<ImuSample> prop;
  {
    HPROF("prop.select");
    prop = select_imu_readings(timestamp_ + last_prop_time_offset_, timestamp + t_off_new);
  }
  int n;
  std::vector<int> ids = phi_order_ids(&n);
  std::vector<double> Phi, Qd;
  {
    HPROF("prop.phi");
    accumulate_phi(prop, Phi, Qd, n);
  }
  double lw[3];
  last_w(prop, lw);
  // the clone's time-offset column (augment_clone, StateHelper.cpp:579-616) goes up with Phi / Qd
  double dnc[6] = {lw[0], lw[1], lw[2], imu_->val[7], imu_->val[8], imu_->val[9]};
  const bool do_dt = o_.do_calib_camera_timeoffset != 0;
  const double *ddnc = do_dt ? stage(dnc, 6) : nullptr;
  // propagation and clone in one launch unless the clone is refused below (a clone at this time exists)
  if (clones_.find(timestamp) == clones_.end() && cov_propagate_clone(imu_->id, n, ids, Phi, Qd, do_dt, ddnc)) {
    timestamp_ = timestamp;
    last_prop_time_offset_ = t_off_new;
    clones_[timestamp_] = add_clone_var();
    return 0;
  }
  cov_propagate(imu_->id, n, ids, Phi, Qd);
  timestamp_ = timestamp;
  last_prop_time_offset_ = t_off_new;
  if (clones_.find(timestamp_) != clones_.end()) return UVIO_HP_E_STATE;
  VarP pose = clone_imu_pose(dnc, do_dt, ddnc);
  clones_[timestamp_] = pose;
  return 0;
}

// UVioPropagator::propagate (UVioPropagator.cpp:27-115); quirks kept: time1 has no cam-imu offset and
// last_prop_time_offset is not updated.
int Engine::propagate_uwb(double timestamp) {
  stage_ = "UVioPropagator::propagate";
  if (timestamp_ >= timestamp) return UVIO_HP_E_ORDER;
  std::vector<ImuSample> prop = select_imu_readings(timestamp_ + last_prop_time_offset_, timestamp);
  int n;
  std::vector<int> ids = phi_order_ids(&n);
  std::vector<double> Phi, Qd;
  accumulate_phi(prop, Phi, Qd, n);
  cov_propagate(imu_->id, n, ids, Phi, Qd);
  timestamp_ = timestamp;
  return 0;
}

}  // namespace uvhp

namespace uvhp {

namespace {
// UpdaterHelper::measurement_compress_inplace (UpdaterHelper.cpp:456-487): Givens QR of the stacked rows
// [H | res] (Eigen makeGivens / applyOnTheLeft(0, 1, G.adjoint()) conventions), keeping min(m, n) rows
void givens_compress(std::vector<double> &H, std::vector<double> &res, int &m, int n) {
  if (m <= n) return;
  for (int c = 0; c < n; c++)
    for (int r = m - 1; r > c; r--) {
      const double p = H[(size_t)(r - 1) * n + c], q = H[(size_t)r * n + c];
      double cs = 1, sn = 0;
      if (q == 0) {
        cs = p < 0 ? -1.0 : 1.0;
        sn = 0;
      } else if (p == 0) {
        cs = 0;
        sn = q < 0 ? 1.0 : -1.0;
      } else if (std::abs(p) > std::abs(q)) {
        const double t = q / p;
        double u = std::sqrt(1.0 + t * t);
        if (p < 0) u = -u;
        cs = 1.0 / u;
        sn = -t * cs;
      } else {
        const double t = p / q;
        double u = std::sqrt(1.0 + t * t);
        if (q < 0) u = -u;
        sn = -1.0 / u;
        cs = -t * sn;
      }
      auto rot = [&](double &x, double &y) {
        const double xi = x, yi = y;
        x = cs * xi - sn * yi;
        y = sn * xi + cs * yi;
      };
      for (int j = c; j < n; j++) rot(H[(size_t)(r - 1) * n + j], H[(size_t)r * n + j]);
      rot(res[r - 1], res[r]);
    }
  m = n;
  H.resize((size_t)m * n);
  res.resize(m);
}
}  // namespace

// UpdaterZeroVelocity::try_update (UpdaterZeroVelocity.cpp:65-329) with the reference's defaults
// (integrated_accel_constraint = false, model_time_varying_bias = true, override_with_disparity_check = true,
// explicitly_enforce_zero_motion = false).  The residual / Jacobian over the IMU readings (6 rows per
// interval, 9 columns [theta, bg, ba]) and their Givens compression are host math on ~60 x 9; the chi2 test
// reads the 9 x 9 marginal covariance from the device; the bias propagation and the EKF update run on the
// device like every other covariance operation.
int Engine::zupt_try_update(double timestamp) {
  stage_ = "UpdaterZeroVelocity::try_update";
  std::vector<ImuSample> imu;
  {
    std::lock_guard<std::mutex> lk(imu_mtx_);
    imu = zupt_imu_;
  }
  if (imu.empty()) {
    last_zupt_state_timestamp_ = 0.0;
    return 0;
  }
  if (timestamp_ == timestamp) {
    last_zupt_state_timestamp_ = 0.0;
    return 0;
  }
  if (!zupt_have_last_off_) {
    zupt_last_off_ = calib_dt_->val[0];
    zupt_have_last_off_ = true;
  }
  const double t_off_new = calib_dt_->val[0];
  // Propagator::select_imu_readings on the ZUPT's own buffer
  std::vector<ImuSample> recent = select_imu(imu, timestamp_ + zupt_last_off_, timestamp + t_off_new);
  zupt_last_off_ = t_off_new;
  if (recent.size() < 2) {
    last_zupt_state_timestamp_ = 0.0;
    return 0;
  }
  const int n = 9;
  int m = 6 * ((int)recent.size() - 1);
  std::vector<double> H((size_t)m * n, 0.0), res(m, 0.0);
  double Dw[9], Da[9], Tg[9], Ra[9], Rw[9], R[9], Rj[9], g[3] = {0, 0, o_.gravity_mag};
  Dm(o_.imu_model, dw_->val, Dw);
  Dm(o_.imu_model, da_->val, Da);
  TgM(tg_->val, Tg);
  quat_2_Rot(qa_->val, Ra);
  quat_2_Rot(qg_->val, Rw);
  quat_2_Rot(imu_->val, R);
  quat_2_Rot(o_.do_fej ? imu_->fej : imu_->val, Rj);
  const double *bg = imu_->val + 10, *ba = imu_->val + 13;
  double dt_summed = 0;
  for (size_t i = 0; i + 1 < recent.size(); i++) {
    const double dt = recent[i + 1].t - recent[i].t;
    double t1[3], t2[3], a_hat[3], w_hat[3], Ta[3], Rg[3], Sg[9];
    for (int k = 0; k < 3; k++) t1[k] = recent[i].am[k] - ba[k];
    m3_vec(Da, t1, t2);
    m3_vec(Ra, t2, a_hat);
    m3_vec(Tg, a_hat, Ta);
    for (int k = 0; k < 3; k++) t1[k] = recent[i].wm[k] - bg[k] - Ta[k];
    m3_vec(Dw, t1, t2);
    m3_vec(Rw, t2, w_hat);
    const double w_omega = std::sqrt(dt) / o_.sigma_w, w_accel = std::sqrt(dt) / o_.sigma_a;
    m3_vec(R, g, Rg);
    const size_t r0 = 6 * i;
    for (int k = 0; k < 3; k++) {
      res[r0 + k] = -w_omega * w_hat[k];
      res[r0 + 3 + k] = -w_accel * (a_hat[k] - Rg[k]);
    }
    m3_vec(Rj, g, Rg);
    skew(Rg, Sg);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        H[(r0 + a) * n + 3 + b] = (a == b) ? -w_omega : 0.0;
        H[(r0 + 3 + a) * n + b] = -w_accel * Sg[3 * a + b];
        H[(r0 + 3 + a) * n + 6 + b] = (a == b) ? -w_accel : 0.0;
      }
    dt_summed += dt;
  }
  givens_compress(H, res, m, n);
  if (m < 1) return 0;
  const double Rn = o_.zupt_noise_multiplier;
  double Qb[36] = {0};
  for (int k = 0; k < 3; k++) {
    Qb[7 * k] = dt_summed * o_.sigma_wb * o_.sigma_wb;
    Qb[7 * (k + 3)] = dt_summed * o_.sigma_ab * o_.sigma_ab;
  }
  // chi2 with P_marg of [theta, bg, ba] (+ the bias evolution the update would apply)
  std::vector<double> Pimu(15 * 15);
  HP_HIP(hipMemcpy2DAsync(Pimu.data(), sizeof(double) * 15, d_.P + (size_t)imu_->id * d_.ldp + imu_->id,
                          sizeof(double) * d_.ldp, sizeof(double) * 15, 15, hipMemcpyDeviceToHost, d_.stream));
  dev_sync();
  const int idx[9] = {0, 1, 2, 9, 10, 11, 12, 13, 14};
  double Pm[81];
  for (int a = 0; a < 9; a++)
    for (int b = 0; b < 9; b++) Pm[9 * a + b] = Pimu[15 * idx[a] + idx[b]];
  for (int a = 0; a < 6; a++)
    for (int b = 0; b < 6; b++) Pm[9 * (3 + a) + 3 + b] += Qb[6 * a + b];
  std::vector<double> HP((size_t)m * n, 0.0), S((size_t)m * m, 0.0);
  for (int i = 0; i < m; i++)
    for (int k = 0; k < n; k++) {
      const double h = H[(size_t)i * n + k];
      if (h == 0.0) continue;
      for (int j = 0; j < n; j++) HP[(size_t)i * n + j] += h * Pm[9 * k + j];
    }
  for (int i = 0; i < m; i++)
    for (int j = 0; j < m; j++) {
      double acc = 0;
      for (int k = 0; k < n; k++) acc += HP[(size_t)i * n + k] * H[(size_t)j * n + k];
      S[(size_t)i * m + j] = acc + (i == j ? Rn : 0.0);
    }
  // LLT solve S x = res
  std::vector<double> L((size_t)m * m, 0.0), y(res);
  for (int j = 0; j < m; j++) {
    double d = S[(size_t)j * m + j];
    for (int k = 0; k < j; k++) d -= L[(size_t)j * m + k] * L[(size_t)j * m + k];
    if (!(d > 0)) {
      // S not positive definite (the reference's LLT result is undefined there): take the reference's
      // rejection path, which also resets the ZUPT bookkeeping (UpdaterZeroVelocity.cpp:240-245)
      last_zupt_state_timestamp_ = 0.0;
      last_zupt_count_ = 0;
      return 0;
    }
    L[(size_t)j * m + j] = std::sqrt(d);
    for (int i = j + 1; i < m; i++) {
      double v = S[(size_t)i * m + j];
      for (int k = 0; k < j; k++) v -= L[(size_t)i * m + k] * L[(size_t)j * m + k];
      L[(size_t)i * m + j] = v / L[(size_t)j * m + j];
    }
  }
  for (int i = 0; i < m; i++) {
    for (int k = 0; k < i; k++) y[i] -= L[(size_t)i * m + k] * y[k];
    y[i] /= L[(size_t)i * m + i];
  }
  for (int i = m - 1; i >= 0; i--) {
    for (int k = i + 1; k < m; k++) y[i] -= L[(size_t)k * m + i] * y[k];
    y[i] /= L[(size_t)i * m + i];
  }
  double chi2 = 0;
  for (int i = 0; i < m; i++) chi2 += res[i] * y[i];
  const double chi2_check = chi2_table_[std::min(m, 999)];
  // FeatureHelper::compute_disparity(db, state time, frame time) (FeatureHelper.h:60-108): raw-pixel
  // displacement of every feature seen at both times, in the database's iteration order
  const double time0 = timestamp_, time1 = timestamp;
  std::vector<double> disp;
  for (auto &kv : db_) {
    const Feature &f = *kv.second;
    if (f.to_delete) continue;
    bool has0 = false;
    for (auto &tr : f.tracks)
      for (auto &ms : tr.m) has0 |= (ms.t == time0);
    if (!has0) continue;
    for (auto &tr : f.tracks) {
      int i0 = -1, i1 = -1;
      for (int k = 0; k < (int)tr.m.size(); k++) {
        if (i0 < 0 && tr.m[k].t == time0) i0 = k;
        if (i1 < 0 && tr.m[k].t == time1) i1 = k;
      }
      if (i0 < 0 || i1 < 0) continue;
      const float dx = tr.m[i1].u - tr.m[i0].u, dy = tr.m[i1].v - tr.m[i0].v;
      disp.push_back((double)std::sqrt(dx * dx + dy * dy));
    }
  }
  double disp_avg = 0;
  for (double d : disp) disp_avg += d;
  disp_avg /= (double)disp.size();  // NaN without features, as the reference
  const bool disparity_passed = disp_avg < o_.zupt_max_disparity && (int)disp.size() > 20;
  const double vnorm = norm3(imu_->val + 7);
  if (!disparity_passed && (chi2 > o_.zupt_chi2_multipler * chi2_check || vnorm > o_.zupt_max_velocity)) {
    last_zupt_state_timestamp_ = 0.0;
    last_zupt_count_ = 0;
    return 0;
  }
  // FeatureDatabase::cleanup_measurements_exact (FeatureDatabase.cpp:245-263)
  if (last_zupt_count_ >= 2) {
    const double te = last_zupt_state_timestamp_;
    for (auto it = db_.begin(); it != db_.end();) {
      int ct = 0;
      for (auto &tr : it->second->tracks) {
        tr.m.erase(std::remove_if(tr.m.begin(), tr.m.end(), [te](const FeatMeas &x) { return x.t == te; }), tr.m.end());
        ct += (int)tr.m.size();
      }
      if (ct < 1)
        it = db_erase(it);
      else
        it++;
    }
  }
  // bias random walk over the window (EKFPropagation with Phi = I), then the EKF update with R = mult I
  std::vector<int> bias_ids;
  for (int k = 9; k < 15; k++) bias_ids.push_back(imu_->id + k);
  std::vector<double> Phi(36, 0.0), Q(Qb, Qb + 36);
  for (int k = 0; k < 6; k++) Phi[7 * k] = 1.0;
  cov_propagate(imu_->id + 9, 6, bias_ids, Phi, Q);
  std::vector<double> Hr((size_t)m * (n + 1));
  for (int i = 0; i < m; i++) {
    for (int j = 0; j < n; j++) Hr[(size_t)i * (n + 1) + j] = H[(size_t)i * n + j];
    Hr[(size_t)i * (n + 1) + n] = res[i];
  }
  std::vector<int> hidx;
  for (int k : idx) hidx.push_back(imu_->id + k);
  const double *dH = stage(Hr.data(), Hr.size());
  stage_flush();
  ekf_update_rows(dH, n + 1, m, n, hidx, dH + n, n + 1, Rn);
  timestamp_ = timestamp;
  last_zupt_state_timestamp_ = timestamp;
  last_zupt_count_++;
  return 1;
}

}  // namespace uvhp
