// ORACLE — test infrastructure only (see la.h header).
// Restatement of ov_core/src/cam/CamRadtan.h and CamEqui.h:
//   distort_f               CamRadtan.h:127 / CamEqui.h:136  (float in/out, double inside)
//   compute_distort_jacobian CamRadtan.h:154 / CamEqui.h:166
//   undistort_f              CamRadtan.h:99 / CamEqui.h:108 -> OpenCV undistortPoints /
//                            fisheye::undistortPoints (OpenCV 4.2, not in /root/reference;
//                            restated from SURVEY Appendix A)
#pragma once
#include "flip.h"
#include "la.h"

namespace orc {

struct Camera {
  int model = 0;  // 0 radtan, 1 equidistant
  int w = 0, h = 0;
  double v[8] = {0};  // fx fy cx cy d0..d3

  // CamBase::distort_d (CamBase.h:130): double -> float -> distort_f -> float -> double
  void distort_d(double xn, double yn, double &u, double &vv) const {
    float xf = fcast(xn), yf = fcast(yn);
    float uf, vf;
    distort_f(xf, yf, uf, vf);
    u = (double)uf;
    vv = (double)vf;
  }

  void distort_f(float xf, float yf, float &uf, float &vf) const {
    double x = xf, y = yf;
    if (model == 0) {
      double r = std::sqrt(x * x + y * y);
      double r_2 = r * r, r_4 = r_2 * r_2;
      double x1 = x * (1 + v[4] * r_2 + v[5] * r_4) + 2 * v[6] * x * y + v[7] * (r_2 + 2 * x * x);
      double y1 = y * (1 + v[4] * r_2 + v[5] * r_4) + v[6] * (r_2 + 2 * y * y) + 2 * v[7] * x * y;
      uf = fcast(v[0] * x1 + v[2]);
      vf = fcast(v[1] * y1 + v[3]);
    } else {
      double r = std::sqrt(x * x + y * y);
      double theta = std::atan(r);
      double theta_d = theta + v[4] * std::pow(theta, 3) + v[5] * std::pow(theta, 5) + v[6] * std::pow(theta, 7) +
                       v[7] * std::pow(theta, 9);
      double inv_r = (r > 1e-8) ? 1.0 / r : 1.0;
      double cdist = (r > 1e-8) ? theta_d * inv_r : 1.0;
      double x1 = x * cdist, y1 = y * cdist;
      uf = fcast(v[0] * x1 + v[2]);
      vf = fcast(v[1] * y1 + v[3]);
    }
  }

  // H_dz_dzn (2x2) and H_dz_dzeta (2x8)
  void distort_jacobian(double x, double y, Mat &dz_dzn, Mat &dz_dzeta) const {
    dz_dzn = Mat(2, 2);
    dz_dzeta = Mat(2, 8);
    if (model == 0) {
      double r = std::sqrt(x * x + y * y);
      double r_2 = r * r, r_4 = r_2 * r_2;
      double x_2 = x * x, y_2 = y * y, x_y = x * y;
      dz_dzn(0, 0) = v[0] * ((1 + v[4] * r_2 + v[5] * r_4) + (2 * v[4] * x_2 + 4 * v[5] * x_2 * r_2) + 2 * v[6] * y +
                             (2 * v[7] * x + 4 * v[7] * x));
      dz_dzn(0, 1) = v[0] * (2 * v[4] * x_y + 4 * v[5] * x_y * r_2 + 2 * v[6] * x + 2 * v[7] * y);
      dz_dzn(1, 0) = v[1] * (2 * v[4] * x_y + 4 * v[5] * x_y * r_2 + 2 * v[6] * x + 2 * v[7] * y);
      dz_dzn(1, 1) = v[1] * ((1 + v[4] * r_2 + v[5] * r_4) + (2 * v[4] * y_2 + 4 * v[5] * y_2 * r_2) + 2 * v[7] * x +
                             (2 * v[6] * y + 4 * v[6] * y));
      double x1 = x * (1 + v[4] * r_2 + v[5] * r_4) + 2 * v[6] * x * y + v[7] * (r_2 + 2 * x * x);
      double y1 = y * (1 + v[4] * r_2 + v[5] * r_4) + v[6] * (r_2 + 2 * y * y) + 2 * v[7] * x * y;
      dz_dzeta(0, 0) = x1;
      dz_dzeta(0, 2) = 1;
      dz_dzeta(0, 4) = v[0] * x * r_2;
      dz_dzeta(0, 5) = v[0] * x * r_4;
      dz_dzeta(0, 6) = 2 * v[0] * x * y;
      dz_dzeta(0, 7) = v[0] * (r_2 + 2 * x * x);
      dz_dzeta(1, 1) = y1;
      dz_dzeta(1, 3) = 1;
      dz_dzeta(1, 4) = v[1] * y * r_2;
      dz_dzeta(1, 5) = v[1] * y * r_4;
      dz_dzeta(1, 6) = v[1] * (r_2 + 2 * y * y);
      dz_dzeta(1, 7) = 2 * v[1] * x * y;
    } else {
      double r = std::sqrt(x * x + y * y);
      double theta = std::atan(r);
      double theta_d = theta + v[4] * std::pow(theta, 3) + v[5] * std::pow(theta, 5) + v[6] * std::pow(theta, 7) +
                       v[7] * std::pow(theta, 9);
      double inv_r = (r > 1e-8) ? 1.0 / r : 1.0;
      double cdist = (r > 1e-8) ? theta_d * inv_r : 1.0;
      Mat duv_dxy(2, 2);
      duv_dxy(0, 0) = v[0];
      duv_dxy(1, 1) = v[1];
      Mat dxy_dxyn(2, 2);
      dxy_dxyn(0, 0) = theta_d * inv_r;
      dxy_dxyn(1, 1) = theta_d * inv_r;
      Mat dxy_dr(2, 1);
      dxy_dr[0] = -x * theta_d * inv_r * inv_r;
      dxy_dr[1] = -y * theta_d * inv_r * inv_r;
      Mat dr_dxyn(1, 2);
      dr_dxyn[0] = x * inv_r;
      dr_dxyn[1] = y * inv_r;
      Mat dxy_dthd(2, 1);
      dxy_dthd[0] = x * inv_r;
      dxy_dthd[1] = y * inv_r;
      double dthd_dth = 1 + 3 * v[4] * std::pow(theta, 2) + 5 * v[5] * std::pow(theta, 4) + 7 * v[6] * std::pow(theta, 6) +
                        9 * v[7] * std::pow(theta, 8);
      double dth_dr = 1 / (r * r + 1);
      dz_dzn = duv_dxy * (dxy_dxyn + (dxy_dr + (dthd_dth * dth_dr) * dxy_dthd) * dr_dxyn);
      double x1 = x * cdist, y1 = y * cdist;
      dz_dzeta(0, 0) = x1;
      dz_dzeta(0, 2) = 1;
      dz_dzeta(0, 4) = v[0] * x * inv_r * std::pow(theta, 3);
      dz_dzeta(0, 5) = v[0] * x * inv_r * std::pow(theta, 5);
      dz_dzeta(0, 6) = v[0] * x * inv_r * std::pow(theta, 7);
      dz_dzeta(0, 7) = v[0] * x * inv_r * std::pow(theta, 9);
      dz_dzeta(1, 1) = y1;
      dz_dzeta(1, 3) = 1;
      dz_dzeta(1, 4) = v[1] * y * inv_r * std::pow(theta, 3);
      dz_dzeta(1, 5) = v[1] * y * inv_r * std::pow(theta, 5);
      dz_dzeta(1, 6) = v[1] * y * inv_r * std::pow(theta, 7);
      dz_dzeta(1, 7) = v[1] * y * inv_r * std::pow(theta, 9);
    }
  }

  // undistort_cv: cv::undistortPoints (radtan, 5 fixed iterations) or cv::fisheye::undistortPoints
  void undistort_f(float u, float vv, float &xo, float &yo) const {
    double px = u, py = vv;
    if (model == 0) {
      double x0 = (px - v[2]) * (1.0 / v[0]);
      double y0 = (py - v[3]) * (1.0 / v[1]);
      double x = x0, y = y0;
      double k0 = v[4], k1 = v[5], p0 = v[6], p1 = v[7];
      for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        double icdist = 1.0 / (1 + (k1 * r2 + k0) * r2);
        if (icdist < 0) {
          x = x0;
          y = y0;
          break;
        }
        double deltaX = 2 * p0 * x * y + p1 * (r2 + 2 * x * x);
        double deltaY = p0 * (r2 + 2 * y * y) + 2 * p1 * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
      }
      xo = (float)x;
      yo = (float)y;
    } else {
      double pwx = (px - v[2]) / v[0], pwy = (py - v[3]) / v[1];
      double scale = 1.0;
      double theta_d = std::sqrt(pwx * pwx + pwy * pwy);
      theta_d = std::min(std::max(-M_PI / 2., theta_d), M_PI / 2.);
      if (theta_d > 1e-8) {
        double theta = theta_d;
        for (int j = 0; j < 10; j++) {
          double theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2, theta8 = theta6 * theta2;
          double k0t = v[4] * theta2, k1t = v[5] * theta4, k2t = v[6] * theta6, k3t = v[7] * theta8;
          double theta_fix = (theta * (1 + k0t + k1t + k2t + k3t) - theta_d) / (1 + 3 * k0t + 5 * k1t + 7 * k2t + 9 * k3t);
          theta = theta - theta_fix;
          if (std::fabs(theta_fix) < 1e-8) break;
        }
        scale = std::tan(theta) / theta_d;
      }
      xo = (float)(pwx * scale);
      yo = (float)(pwy * scale);
    }
  }
};

}  // namespace orc
