// Small fixed-size FP64 math shared by host orchestration and gfx950 device code.
// JPL quaternion conventions of ov_core/src/utils/quat_ops.h (q = [x y z w], R = quat_2_Rot(q)
// maps global->local); camera models of ov_core/src/cam/CamRadtan.h / CamEqui.h.
// Row-major 3x3 matrices as double[9].
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#define HPD __host__ __device__ __forceinline__

namespace uvhp {

HPD void m3_mul(const double *A, const double *B, double *C) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
// C = A * B^T
HPD void m3_mul_bt(const double *A, const double *B, double *C) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) C[3 * i + j] = A[3 * i] * B[3 * j] + A[3 * i + 1] * B[3 * j + 1] + A[3 * i + 2] * B[3 * j + 2];
}
// C = A^T * B
HPD void m3_mul_at(const double *A, const double *B, double *C) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) C[3 * i + j] = A[i] * B[j] + A[3 + i] * B[3 + j] + A[6 + i] * B[6 + j];
}
HPD void m3_vec(const double *A, const double *x, double *y) {
  for (int i = 0; i < 3; i++) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}
HPD void m3t_vec(const double *A, const double *x, double *y) {
  for (int i = 0; i < 3; i++) y[i] = A[i] * x[0] + A[3 + i] * x[1] + A[6 + i] * x[2];
}
HPD void m3_transpose(const double *A, double *T) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) T[3 * j + i] = A[3 * i + j];
}
HPD void skew(const double *w, double *S) {
  S[0] = 0; S[1] = -w[2]; S[2] = w[1];
  S[3] = w[2]; S[4] = 0; S[5] = -w[0];
  S[6] = -w[1]; S[7] = w[0]; S[8] = 0;
}
HPD double dot3(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
HPD double norm3(const double *a) { return sqrt(dot3(a, a)); }
// inverse of a 3x3 (row-major) by cofactors; host and device give identical results (no contraction)
HPD void inv3_cofactor(const double *A, double *R) {
  const double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                     A[2] * (A[3] * A[7] - A[4] * A[6]);
  R[0] = (A[4] * A[8] - A[5] * A[7]) / det;
  R[1] = (A[2] * A[7] - A[1] * A[8]) / det;
  R[2] = (A[1] * A[5] - A[2] * A[4]) / det;
  R[3] = (A[5] * A[6] - A[3] * A[8]) / det;
  R[4] = (A[0] * A[8] - A[2] * A[6]) / det;
  R[5] = (A[2] * A[3] - A[0] * A[5]) / det;
  R[6] = (A[3] * A[7] - A[4] * A[6]) / det;
  R[7] = (A[1] * A[6] - A[0] * A[7]) / det;
  R[8] = (A[0] * A[4] - A[1] * A[3]) / det;
}

// quat_ops.h:152
HPD void quat_2_Rot(const double *q, double *R) {
  double w = q[3];
  double a = 2 * w * w - 1;
  double x = q[0], y = q[1], z = q[2];
  // a*I - 2w*skew(v) + 2 v v^T
  R[0] = a + 2 * x * x;       R[1] = 2 * w * z + 2 * x * y; R[2] = -2 * w * y + 2 * x * z;
  R[3] = -2 * w * z + 2 * y * x; R[4] = a + 2 * y * y;    R[5] = 2 * w * x + 2 * y * z;
  R[6] = 2 * w * y + 2 * z * x;  R[7] = -2 * w * x + 2 * z * y; R[8] = a + 2 * z * z;
}
// quat_ops.h:180  (q (x) p, normalized, w >= 0)
HPD void quat_multiply(const double *q, const double *p, double *out) {
  double qx = q[0], qy = q[1], qz = q[2], qw = q[3];
  // Qm = [qw*I - skew(qv), qv; -qv^T, qw]
  double t0 = qw * p[0] + qz * p[1] - qy * p[2] + qx * p[3];
  double t1 = -qz * p[0] + qw * p[1] + qx * p[2] + qy * p[3];
  double t2 = qy * p[0] - qx * p[1] + qw * p[2] + qz * p[3];
  double t3 = -qx * p[0] - qy * p[1] - qz * p[2] + qw * p[3];
  if (t3 < 0) {
    t0 = -t0; t1 = -t1; t2 = -t2; t3 = -t3;
  }
  double n = sqrt(t0 * t0 + t1 * t1 + t2 * t2 + t3 * t3);
  out[0] = t0 / n; out[1] = t1 / n; out[2] = t2 / n; out[3] = t3 / n;
}
// quat_ops.h:496
HPD void quatnorm(double *q) {
  if (q[3] < 0) {
    q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3];
  }
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}
// JPLQuat::update (JPLQuat.h:114): q <- quatnorm([dth/2, 1]) (x) q
HPD void quat_boxplus(double *q, const double *dth) {
  double dq[4] = {0.5 * dth[0], 0.5 * dth[1], 0.5 * dth[2], 1.0};
  quatnorm(dq);
  double o[4];
  quat_multiply(dq, q, o);
  q[0] = o[0]; q[1] = o[1]; q[2] = o[2]; q[3] = o[3];
}

// rot_2_quat (quat_ops.h:88) on a row-major 3x3
inline void rot_2_quat(const double *r, double *q) {
  auto R = [&](int i, int j) { return r[3 * i + j]; };
  double T = R(0, 0) + R(1, 1) + R(2, 2);
  if ((R(0, 0) >= T) && (R(0, 0) >= R(1, 1)) && (R(0, 0) >= R(2, 2))) {
    q[0] = std::sqrt((1 + (2 * R(0, 0)) - T) / 4);
    q[1] = (1 / (4 * q[0])) * (R(0, 1) + R(1, 0));
    q[2] = (1 / (4 * q[0])) * (R(0, 2) + R(2, 0));
    q[3] = (1 / (4 * q[0])) * (R(1, 2) - R(2, 1));
  } else if ((R(1, 1) >= T) && (R(1, 1) >= R(0, 0)) && (R(1, 1) >= R(2, 2))) {
    q[1] = std::sqrt((1 + (2 * R(1, 1)) - T) / 4);
    q[0] = (1 / (4 * q[1])) * (R(0, 1) + R(1, 0));
    q[2] = (1 / (4 * q[1])) * (R(1, 2) + R(2, 1));
    q[3] = (1 / (4 * q[1])) * (R(2, 0) - R(0, 2));
  } else if ((R(2, 2) >= T) && (R(2, 2) >= R(0, 0)) && (R(2, 2) >= R(1, 1))) {
    q[2] = std::sqrt((1 + (2 * R(2, 2)) - T) / 4);
    q[0] = (1 / (4 * q[2])) * (R(0, 2) + R(2, 0));
    q[1] = (1 / (4 * q[2])) * (R(1, 2) + R(2, 1));
    q[3] = (1 / (4 * q[2])) * (R(0, 1) - R(1, 0));
  } else {
    q[3] = std::sqrt((1 + T) / 4);
    q[0] = (1 / (4 * q[3])) * (R(1, 2) - R(2, 1));
    q[1] = (1 / (4 * q[3])) * (R(2, 0) - R(0, 2));
    q[2] = (1 / (4 * q[3])) * (R(0, 1) - R(1, 0));
  }
  if (q[3] < 0) {
    q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3];
  }
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int k = 0; k < 4; k++) q[k] /= n;
}

// ---- camera models (CamRadtan.h:127-198, CamEqui.h:136-230) ----
struct CamParams {
  int model;  // 0 radtan, 1 equidistant
  int w, h;
  double v[8];
};

// distort_f with the reference's float interface: inputs rounded to float, outputs float
HPD void cam_distort_f(const CamParams &c, float xf, float yf, float &uf, float &vf) {
  double x = xf, y = yf;
  const double *v = c.v;
  if (c.model == 0) {
    double r = sqrt(x * x + y * y);
    double r_2 = r * r, r_4 = r_2 * r_2;
    double x1 = x * (1 + v[4] * r_2 + v[5] * r_4) + 2 * v[6] * x * y + v[7] * (r_2 + 2 * x * x);
    double y1 = y * (1 + v[4] * r_2 + v[5] * r_4) + v[6] * (r_2 + 2 * y * y) + 2 * v[7] * x * y;
    uf = (float)(v[0] * x1 + v[2]);
    vf = (float)(v[1] * y1 + v[3]);
  } else {
    double r = sqrt(x * x + y * y);
    double th = atan(r);
    double th2 = th * th;
    double th3 = th2 * th, th5 = th3 * th2, th7 = th5 * th2, th9 = th7 * th2;
    double theta_d = th + v[4] * th3 + v[5] * th5 + v[6] * th7 + v[7] * th9;
    double inv_r = (r > 1e-8) ? 1.0 / r : 1.0;
    double cdist = (r > 1e-8) ? theta_d * inv_r : 1.0;
    uf = (float)(v[0] * (x * cdist) + v[2]);
    vf = (float)(v[1] * (y * cdist) + v[3]);
  }
}

// H_dz_dzn (2x2 row-major) and H_dz_dzeta (2x8 row-major)
HPD void cam_distort_jac(const CamParams &c, double x, double y, double *dzn, double *dzeta) {
  const double *v = c.v;
  for (int k = 0; k < 16; k++) dzeta[k] = 0;
  if (c.model == 0) {
    double r_2 = x * x + y * y;
    double r = sqrt(r_2);
    r_2 = r * r;
    double r_4 = r_2 * r_2;
    double x_2 = x * x, y_2 = y * y, x_y = x * y;
    dzn[0] = v[0] * ((1 + v[4] * r_2 + v[5] * r_4) + (2 * v[4] * x_2 + 4 * v[5] * x_2 * r_2) + 2 * v[6] * y +
                     (2 * v[7] * x + 4 * v[7] * x));
    dzn[1] = v[0] * (2 * v[4] * x_y + 4 * v[5] * x_y * r_2 + 2 * v[6] * x + 2 * v[7] * y);
    dzn[2] = v[1] * (2 * v[4] * x_y + 4 * v[5] * x_y * r_2 + 2 * v[6] * x + 2 * v[7] * y);
    dzn[3] = v[1] * ((1 + v[4] * r_2 + v[5] * r_4) + (2 * v[4] * y_2 + 4 * v[5] * y_2 * r_2) + 2 * v[7] * x +
                     (2 * v[6] * y + 4 * v[6] * y));
    double x1 = x * (1 + v[4] * r_2 + v[5] * r_4) + 2 * v[6] * x * y + v[7] * (r_2 + 2 * x * x);
    double y1 = y * (1 + v[4] * r_2 + v[5] * r_4) + v[6] * (r_2 + 2 * y * y) + 2 * v[7] * x * y;
    dzeta[0] = x1;
    dzeta[2] = 1;
    dzeta[4] = v[0] * x * r_2;
    dzeta[5] = v[0] * x * r_4;
    dzeta[6] = 2 * v[0] * x * y;
    dzeta[7] = v[0] * (r_2 + 2 * x * x);
    dzeta[8 + 1] = y1;
    dzeta[8 + 3] = 1;
    dzeta[8 + 4] = v[1] * y * r_2;
    dzeta[8 + 5] = v[1] * y * r_4;
    dzeta[8 + 6] = v[1] * (r_2 + 2 * y * y);
    dzeta[8 + 7] = 2 * v[1] * x * y;
  } else {
    double r = sqrt(x * x + y * y);
    double th = atan(r);
    double th2 = th * th;
    double th3 = th2 * th, th4 = th2 * th2, th5 = th3 * th2, th6 = th4 * th2, th7 = th5 * th2, th8 = th6 * th2,
           th9 = th7 * th2;
    double theta_d = th + v[4] * th3 + v[5] * th5 + v[6] * th7 + v[7] * th9;
    double inv_r = (r > 1e-8) ? 1.0 / r : 1.0;
    double cdist = (r > 1e-8) ? theta_d * inv_r : 1.0;
    double dthd_dth = 1 + 3 * v[4] * th2 + 5 * v[5] * th4 + 7 * v[6] * th6 + 9 * v[7] * th8;
    double dth_dr = 1 / (r * r + 1);
    // duv_dxy * (dxy_dxyn + (dxy_dr + dxy_dthd*dthd_dth*dth_dr) * dr_dxyn)
    double a0 = -x * theta_d * inv_r * inv_r + x * inv_r * dthd_dth * dth_dr;
    double a1 = -y * theta_d * inv_r * inv_r + y * inv_r * dthd_dth * dth_dr;
    double b0 = x * inv_r, b1 = y * inv_r;
    dzn[0] = v[0] * (theta_d * inv_r + a0 * b0);
    dzn[1] = v[0] * (a0 * b1);
    dzn[2] = v[1] * (a1 * b0);
    dzn[3] = v[1] * (theta_d * inv_r + a1 * b1);
    dzeta[0] = x * cdist;
    dzeta[2] = 1;
    dzeta[4] = v[0] * x * inv_r * th3;
    dzeta[5] = v[0] * x * inv_r * th5;
    dzeta[6] = v[0] * x * inv_r * th7;
    dzeta[7] = v[0] * x * inv_r * th9;
    dzeta[8 + 1] = y * cdist;
    dzeta[8 + 3] = 1;
    dzeta[8 + 4] = v[1] * y * inv_r * th3;
    dzeta[8 + 5] = v[1] * y * inv_r * th5;
    dzeta[8 + 6] = v[1] * y * inv_r * th7;
    dzeta[8 + 7] = v[1] * y * inv_r * th9;
  }
}

// UpdaterUWB::update_single's row (UVioUpdaterHelper::get_uwb_jacobian_single, UVioUpdaterHelper.cpp:147-241):
// the range from the IMU pose (q_GtoI, p_IinG), p_IinU and the anchor [p_AinG, const_bias, dist_bias];
// H[0..n-1] over the columns [IMU theta (3), IMU p (3), p_IinU (3) if cal, anchor (5) if anc], H[n] = residual.
// Shared by the host and the device (the chained UWB update) so both form the row with the same operations.
HPD int uwb_row(const double *q, const double *pI, const double *pIinU, const double *an, bool cal, bool anc, double range,
                double *H) {
  double R[9], mp[3], t[3], pU[3];
  quat_2_Rot(q, R);
  for (int k = 0; k < 3; k++) mp[k] = -pIinU[k];
  m3t_vec(R, mp, t);
  for (int k = 0; k < 3; k++) pU[k] = t[k] + pI[k];
  const double d[3] = {an[0] - pU[0], an[1] - pU[1], an[2] - pU[2]};
  const double dn = norm3(d);
  const double beta = an[4], gam = an[3];
  const double res = range - ((1 + beta) * dn + gam);
  const double Hn[3] = {d[0] / dn, d[1] / dn, d[2] / dn};
  double S[9], RS[9];
  skew(mp, S);
  m3_mul_at(R, S, RS);  // R^T skew(-p_IinU)
  for (int j = 0; j < 3; j++) {
    H[j] = (1 + beta) * (Hn[0] * RS[j] + Hn[1] * RS[3 + j] + Hn[2] * RS[6 + j]);
    H[3 + j] = (1 + beta) * (-Hn[j]);
  }
  double HnRT[3];  // the row vector H_n R^T
  for (int j = 0; j < 3; j++) HnRT[j] = Hn[0] * R[3 * j] + Hn[1] * R[3 * j + 1] + Hn[2] * R[3 * j + 2];
  int n = 6;
  if (cal) {
    for (int j = 0; j < 3; j++) H[n + j] = (1 + beta) * HnRT[j];
    n += 3;
  }
  if (anc) {
    for (int j = 0; j < 3; j++) H[n + j] = (1 + beta) * HnRT[j];  // reference quirk (UVioUpdaterHelper.cpp:236), kept
    H[n + 3] = 1;
    H[n + 4] = dn;
    n += 5;
  }
  H[n] = res;
  return n;
}

// True when the float rounding of v is not decided by v's leading 40 bits: a result that differs from v by a
// few ulps (the equidistant model's tan, whose last bit differs between libm and the device) could round to
// the other float.  Away from such a boundary (all but <= 2^-15 of the float spacing) the float is the same.
HPD bool float_round_ambiguous(double v) {
  const double e = fabs(v) * 0x1p-40;
  return (float)(v - e) != (float)(v + e);
}

// undistort_cv: cv::undistortPoints (radtan, 5 iterations) / cv::fisheye::undistortPoints.  Returns true when
// the result depends on tan's last bits (equidistant only: every other step is an IEEE operation in the same
// order on host and device), i.e. when a caller that needs the host's libm result must recompute it there.
HPD bool cam_undistort_f(const CamParams &c, float u, float vv, float &xo, float &yo) {
  const double *v = c.v;
  double px = u, py = vv;
  if (c.model == 0) {
    double x0 = (px - v[2]) * (1.0 / v[0]);
    double y0 = (py - v[3]) * (1.0 / v[1]);
    double x = x0, y = y0;
    for (int j = 0; j < 5; j++) {
      double r2 = x * x + y * y;
      double icdist = 1.0 / (1 + (v[5] * r2 + v[4]) * r2);
      if (icdist < 0) {
        x = x0;
        y = y0;
        break;
      }
      double deltaX = 2 * v[6] * x * y + v[7] * (r2 + 2 * x * x);
      double deltaY = v[6] * (r2 + 2 * y * y) + 2 * v[7] * x * y;
      x = (x0 - deltaX) * icdist;
      y = (y0 - deltaY) * icdist;
    }
    xo = (float)x;
    yo = (float)y;
    return false;
  } else {
    double pwx = (px - v[2]) / v[0], pwy = (py - v[3]) / v[1];
    double scale = 1.0;
    double theta_d = sqrt(pwx * pwx + pwy * pwy);
    theta_d = fmin(fmax(-M_PI / 2., theta_d), M_PI / 2.);
    if (theta_d > 1e-8) {
      double theta = theta_d;
      for (int j = 0; j < 10; j++) {
        double t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t6 * t2;
        double k0 = v[4] * t2, k1 = v[5] * t4, k2 = v[6] * t6, k3 = v[7] * t8;
        double fix = (theta * (1 + k0 + k1 + k2 + k3) - theta_d) / (1 + 3 * k0 + 5 * k1 + 7 * k2 + 9 * k3);
        theta = theta - fix;
        if (fabs(fix) < 1e-8) break;
      }
      scale = tan(theta) / theta_d;
    }
    const double xs = pwx * scale, ys = pwy * scale;
    xo = (float)xs;
    yo = (float)ys;
    return theta_d > 1e-8 && (float_round_ambiguous(xs) || float_round_ambiguous(ys));
  }
}

}  // namespace uvhp
