// ORACLE — test infrastructure only. CPU restatement of the reference algorithm; never linked
// into the product (uvio_amd/). Used by tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg as the checker / CPU baseline.
//
// Dense FP64 helpers standing in for the Eigen operations the reference calls (Eigen is a
// third-party dependency absent from /root/reference; ~3.3.7 per SURVEY §8c). Restated:
//   * Eigen JacobiRotation::makeGivens / applyOnTheLeft(G.adjoint()) — SURVEY Appendix A
//   * LLT solve (upper triangle read)  — StateHelper.cpp:160-162, UpdaterMSCKF.cpp:212
//   * colPivHouseholderQr solve 3x3    — FeatureInitializer.cpp:88,294
//   * JacobiSVD singular values 3x3    — FeatureInitializer.cpp:91
// and ov_core/src/utils/quat_ops.h (JPL quaternion ops) verbatim in math.
#pragma once
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstring>
#include <vector>

namespace orc {

struct Mat {
  int r = 0, c = 0;
  std::vector<double> d;
  Mat() {}
  Mat(int r_, int c_) : r(r_), c(c_), d((size_t)r_ * c_, 0.0) {}
  double &operator()(int i, int j) { return d[(size_t)i * c + j]; }
  double operator()(int i, int j) const { return d[(size_t)i * c + j]; }
  double &operator[](int i) { return d[i]; }
  double operator[](int i) const { return d[i]; }
  static Mat Zero(int r, int c) { return Mat(r, c); }
  static Mat Identity(int n) {
    Mat m(n, n);
    for (int i = 0; i < n; i++) m(i, i) = 1.0;
    return m;
  }
  Mat block(int i0, int j0, int nr, int nc) const {
    Mat b(nr, nc);
    for (int i = 0; i < nr; i++)
      for (int j = 0; j < nc; j++) b(i, j) = (*this)(i0 + i, j0 + j);
    return b;
  }
  void set_block(int i0, int j0, const Mat &b) {
    for (int i = 0; i < b.r; i++)
      for (int j = 0; j < b.c; j++) (*this)(i0 + i, j0 + j) = b(i, j);
  }
  void add_block(int i0, int j0, const Mat &b) {
    for (int i = 0; i < b.r; i++)
      for (int j = 0; j < b.c; j++) (*this)(i0 + i, j0 + j) += b(i, j);
  }
  Mat T() const {
    Mat t(c, r);
    for (int i = 0; i < r; i++)
      for (int j = 0; j < c; j++) t(j, i) = (*this)(i, j);
    return t;
  }
  // conservativeResizeLike(Zero): keep the top-left overlap, zero the rest
  void conservative_resize(int nr, int nc) {
    Mat n(nr, nc);
    for (int i = 0; i < std::min(r, nr); i++)
      for (int j = 0; j < std::min(c, nc); j++) n(i, j) = (*this)(i, j);
    *this = n;
  }
};

inline Mat operator*(const Mat &a, const Mat &b) {
  assert(a.c == b.r);
  Mat o(a.r, b.c);
  for (int i = 0; i < a.r; i++)
    for (int k = 0; k < a.c; k++) {
      double aik = a(i, k);
      if (aik == 0.0) continue;
      const double *br = &b.d[(size_t)k * b.c];
      double *orow = &o.d[(size_t)i * o.c];
      for (int j = 0; j < b.c; j++) orow[j] += aik * br[j];
    }
  return o;
}
inline Mat operator+(const Mat &a, const Mat &b) {
  Mat o = a;
  for (size_t i = 0; i < o.d.size(); i++) o.d[i] += b.d[i];
  return o;
}
inline Mat operator-(const Mat &a, const Mat &b) {
  Mat o = a;
  for (size_t i = 0; i < o.d.size(); i++) o.d[i] -= b.d[i];
  return o;
}
inline Mat operator*(double s, const Mat &a) {
  Mat o = a;
  for (auto &v : o.d) v *= s;
  return o;
}
inline Mat operator-(const Mat &a) { return -1.0 * a; }

// ---- small fixed 3-vectors / 3x3 as Mat for brevity ----
inline Mat V3(double a, double b, double c) {
  Mat v(3, 1);
  v[0] = a; v[1] = b; v[2] = c;
  return v;
}
inline double dot(const Mat &a, const Mat &b) {
  double s = 0;
  for (size_t i = 0; i < a.d.size(); i++) s += a.d[i] * b.d[i];
  return s;
}
inline double norm(const Mat &a) { return std::sqrt(dot(a, a)); }

// quat_ops.h:135
inline Mat skew_x(const Mat &w) {
  Mat m(3, 3);
  m(0, 1) = -w[2]; m(0, 2) = w[1];
  m(1, 0) = w[2];  m(1, 2) = -w[0];
  m(2, 0) = -w[1]; m(2, 1) = w[0];
  return m;
}
// quat_ops.h:152 (JPL, q = [x y z w])
inline Mat quat_2_Rot(const Mat &q) {
  Mat qv = q.block(0, 0, 3, 1);
  Mat R = (2 * q[3] * q[3] - 1) * Mat::Identity(3) - (2 * q[3]) * skew_x(qv) + 2.0 * (qv * qv.T());
  return R;
}
// quat_ops.h:88
inline Mat rot_2_quat(const Mat &rot) {
  Mat q(4, 1);
  double T = rot(0, 0) + rot(1, 1) + rot(2, 2);
  if ((rot(0, 0) >= T) && (rot(0, 0) >= rot(1, 1)) && (rot(0, 0) >= rot(2, 2))) {
    q[0] = std::sqrt((1 + (2 * rot(0, 0)) - T) / 4);
    q[1] = (1 / (4 * q[0])) * (rot(0, 1) + rot(1, 0));
    q[2] = (1 / (4 * q[0])) * (rot(0, 2) + rot(2, 0));
    q[3] = (1 / (4 * q[0])) * (rot(1, 2) - rot(2, 1));
  } else if ((rot(1, 1) >= T) && (rot(1, 1) >= rot(0, 0)) && (rot(1, 1) >= rot(2, 2))) {
    q[1] = std::sqrt((1 + (2 * rot(1, 1)) - T) / 4);
    q[0] = (1 / (4 * q[1])) * (rot(0, 1) + rot(1, 0));
    q[2] = (1 / (4 * q[1])) * (rot(1, 2) + rot(2, 1));
    q[3] = (1 / (4 * q[1])) * (rot(2, 0) - rot(0, 2));
  } else if ((rot(2, 2) >= T) && (rot(2, 2) >= rot(0, 0)) && (rot(2, 2) >= rot(1, 1))) {
    q[2] = std::sqrt((1 + (2 * rot(2, 2)) - T) / 4);
    q[0] = (1 / (4 * q[2])) * (rot(0, 2) + rot(2, 0));
    q[1] = (1 / (4 * q[2])) * (rot(1, 2) + rot(2, 1));
    q[3] = (1 / (4 * q[2])) * (rot(0, 1) - rot(1, 0));
  } else {
    q[3] = std::sqrt((1 + T) / 4);
    q[0] = (1 / (4 * q[3])) * (rot(1, 2) - rot(2, 1));
    q[1] = (1 / (4 * q[3])) * (rot(2, 0) - rot(0, 2));
    q[2] = (1 / (4 * q[3])) * (rot(0, 1) - rot(1, 0));
  }
  if (q[3] < 0) q = -q;
  return (1.0 / norm(q)) * q;
}
// quat_ops.h:180
inline Mat quat_multiply(const Mat &q, const Mat &p) {
  Mat Qm(4, 4);
  Mat qv = q.block(0, 0, 3, 1);
  Qm.set_block(0, 0, q[3] * Mat::Identity(3) - skew_x(qv));
  Qm.set_block(0, 3, qv);
  Qm.set_block(3, 0, -qv.T());
  Qm(3, 3) = q[3];
  Mat qt = Qm * p;
  if (qt[3] < 0) qt = -qt;
  return (1.0 / norm(qt)) * qt;
}
// quat_ops.h:231
inline Mat exp_so3(const Mat &w) {
  Mat wx = skew_x(w);
  double theta = norm(w);
  double A, B;
  if (theta < 1e-7) {
    A = 1; B = 0.5;
  } else {
    A = std::sin(theta) / theta;
    B = (1 - std::cos(theta)) / (theta * theta);
  }
  if (theta == 0) return Mat::Identity(3);
  return Mat::Identity(3) + A * wx + B * (wx * wx);
}
// quat_ops.h:482
inline Mat Omega(const Mat &w) {
  Mat m(4, 4);
  m.set_block(0, 0, -skew_x(w));
  m.set_block(3, 0, -w.T());
  m.set_block(0, 3, w);
  return m;
}
// quat_ops.h:496
inline Mat quatnorm(Mat q) {
  if (q[3] < 0) q = -q;
  return (1.0 / norm(q)) * q;
}
// quat_ops.h:515
inline Mat Jl_so3(const Mat &w) {
  double theta = norm(w);
  if (theta < 1e-6) return Mat::Identity(3);
  Mat a = (1.0 / theta) * w;
  return (std::sin(theta) / theta) * Mat::Identity(3) + (1 - std::sin(theta) / theta) * (a * a.T()) +
         ((1 - std::cos(theta)) / theta) * skew_x(a);
}
inline Mat Jr_so3(const Mat &w) { return Jl_so3(-w); }

// ---- Eigen::JacobiRotation<double>::makeGivens(p, q) (real case), SURVEY Appendix A ----
struct Givens {
  double c = 1, s = 0;
  void make(double p, double q) {
    if (q == 0) {
      c = p < 0 ? -1.0 : 1.0;
      s = 0;
    } else if (p == 0) {
      c = 0;
      s = q < 0 ? 1.0 : -1.0;
    } else if (std::abs(p) > std::abs(q)) {
      double t = q / p;
      double u = std::sqrt(1.0 + t * t);
      if (p < 0) u = -u;
      c = 1.0 / u;
      s = -t * c;
    } else {
      double t = p / q;
      double u = std::sqrt(1.0 + t * t);
      if (q < 0) u = -u;
      s = -1.0 / u;
      c = -t * s;
    }
  }
  // applyOnTheLeft(i, i+1, G.adjoint()) on rows x (=i), y (=i+1): x' = c x - s y, y' = s x + c y
  inline void apply(double &x, double &y) const {
    double xi = x, yi = y;
    x = c * xi - s * yi;
    y = s * xi + c * yi;
  }
};

// LLT of the upper triangle of S (symmetric), solve S x = b in place. Returns false if not PD.
inline bool llt_solve(const Mat &S, Mat &b) {
  int n = S.r;
  Mat L(n, n);
  for (int j = 0; j < n; j++) {
    double s = S(j, j);
    for (int k = 0; k < j; k++) s -= L(j, k) * L(j, k);
    if (!(s > 0)) return false;
    double ljj = std::sqrt(s);
    L(j, j) = ljj;
    for (int i = j + 1; i < n; i++) {
      double v = S(j, i);  // upper triangle read (selfadjointView<Upper>)
      for (int k = 0; k < j; k++) v -= L(i, k) * L(j, k);
      L(i, j) = v / ljj;
    }
  }
  for (int col = 0; col < b.c; col++) {
    for (int i = 0; i < n; i++) {
      double v = b(i, col);
      for (int k = 0; k < i; k++) v -= L(i, k) * b(k, col);
      b(i, col) = v / L(i, i);
    }
    for (int i = n - 1; i >= 0; i--) {
      double v = b(i, col);
      for (int k = i + 1; k < n; k++) v -= L(k, i) * b(k, col);
      b(i, col) = v / L(i, i);
    }
  }
  return true;
}

// Column-pivoting Householder QR solve for small square systems (colPivHouseholderQr().solve)
inline Mat colpiv_qr_solve(const Mat &A_in, const Mat &b_in) {
  int n = A_in.r;
  Mat A = A_in, b = b_in;
  std::vector<int> perm(n);
  for (int i = 0; i < n; i++) perm[i] = i;
  std::vector<double> colnorm(n);
  for (int j = 0; j < n; j++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += A(i, j) * A(i, j);
    colnorm[j] = s;
  }
  int rank = n;
  double maxpivot = 0;
  for (int k = 0; k < n; k++) {
    int best = k;
    for (int j = k + 1; j < n; j++)
      if (colnorm[j] > colnorm[best]) best = j;
    if (best != k) {
      for (int i = 0; i < n; i++) std::swap(A(i, k), A(i, best));
      std::swap(colnorm[k], colnorm[best]);
      std::swap(perm[k], perm[best]);
    }
    double alpha = 0;
    for (int i = k; i < n; i++) alpha += A(i, k) * A(i, k);
    alpha = std::sqrt(alpha);
    if (k == 0) maxpivot = alpha;
    if (alpha <= maxpivot * 1e-15 || alpha == 0) {
      rank = k;
      break;
    }
    if (A(k, k) > 0) alpha = -alpha;
    std::vector<double> v(n, 0.0);
    for (int i = k; i < n; i++) v[i] = A(i, k);
    v[k] -= alpha;
    double vn = 0;
    for (int i = k; i < n; i++) vn += v[i] * v[i];
    if (vn > 0) {
      for (int j = k; j < n; j++) {
        double s = 0;
        for (int i = k; i < n; i++) s += v[i] * A(i, j);
        s = 2 * s / vn;
        for (int i = k; i < n; i++) A(i, j) -= s * v[i];
      }
      for (int j = 0; j < b.c; j++) {
        double s = 0;
        for (int i = k; i < n; i++) s += v[i] * b(i, j);
        s = 2 * s / vn;
        for (int i = k; i < n; i++) b(i, j) -= s * v[i];
      }
    }
    for (int j = k + 1; j < n; j++) {
      double s = 0;
      for (int i = k + 1; i < n; i++) s += A(i, j) * A(i, j);
      colnorm[j] = s;
    }
  }
  Mat x(n, b.c);
  for (int j = 0; j < b.c; j++) {
    std::vector<double> y(n, 0.0);
    for (int i = rank - 1; i >= 0; i--) {
      double v = b(i, j);
      for (int k = i + 1; k < rank; k++) v -= A(i, k) * y[k];
      y[i] = v / A(i, i);
    }
    for (int i = 0; i < n; i++) x(perm[i], j) = y[i];
  }
  return x;
}

// Singular values of a 3x3 matrix (descending) via Jacobi eigenvalues of A^T A.
inline void singular_values3(const Mat &A, double sv[3]) {
  Mat M = A.T() * A;
  double a[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) a[i][j] = M(i, j);
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    // converged once the off-diagonal is 1e-18 of the diagonal: further rotations have c == 1 and change no
    // diagonal bit (the full iteration to off < 1e-300 spent ~4 more sweeps on exact-zero moves)
    if (off < 1e-300 || off <= 1e-36 * (a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2])) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        if (a[p][q] == 0) continue;
        double theta = (a[q][q] - a[p][p]) / (2 * a[p][q]);
        double t = (theta >= 0 ? 1.0 : -1.0) / (std::abs(theta) + std::sqrt(theta * theta + 1));
        double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 3; k++) {
          double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; k++) {
          double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
      }
  }
  double e[3] = {std::max(a[0][0], 0.0), std::max(a[1][1], 0.0), std::max(a[2][2], 0.0)};
  std::sort(e, e + 3, [](double x, double y) { return x > y; });
  for (int i = 0; i < 3; i++) sv[i] = std::sqrt(e[i]);
}

}  // namespace orc
