// Per-feature linearization kernel, one 256-thread workgroup (4 waves) per feature.
//
//   wave 0 : FeatureInitializer::single_triangulation  (FeatureInitializer.cpp:30-112)
//            FeatureInitializer::single_gaussnewton    (FeatureInitializer.cpp:197-375, float residuals)
//            one lane per measurement, 64-lane __shfl_xor reductions; every lane ends with the same
//            reduced sums so the LM control flow is wave-uniform.
//   all    : UpdaterHelper::get_feature_jacobian_full (UpdaterHelper.cpp:192-424), one thread per
//            measurement, dense local Jacobian [H_x | res] (2m x (nf+1)) in LDS.
//   all    : left-nullspace projection (UpdaterHelper.cpp:426-454) as 3 Householder reflections of H_f
//            applied to [H_x | res] (any orthonormal basis of the left nullspace gives the same chi2,
//            the same Gram matrix and hence the same EKF update as the reference's Givens sweep).
//   all    : the projected rows [Hhat | rhat] are written to H_all in canonical dense columns (zeros
//            when triangulation / refinement failed).
// The chi2 gate (UpdaterMSCKF.cpp:209-234) runs afterwards for the whole batch (kernels_chi2.hip):
// T = H_all P_can as one GEMM over the shared canonical covariance block, then one workgroup per
// feature forms S = T Hhat^T + s2 I, factors [S | r] and zeroes the rows of rejected features.
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace uvhp {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Sum over the first m lanes in lane (= measurement) order, the order the reference accumulates
// (FeatureInitializer.cpp:76-82, 268-270, 413-416), so the LM accept/stop decisions see the same
// bits.  Values go through LDS (red: 64 * NV + NV doubles); lane k < NV walks series k in lane order
// (one dependent add per measurement, the NV series in parallel) and the sums come back through LDS.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int NV>
__device__ __forceinline__ void ordered_sum(double *red, const double *v, int lane, int m, double *out) {
  wave_sync();
#pragma unroll
  for (int k = 0; k < NV; k++) red[lane * NV + k] = v[k];
  wave_sync();
  if (lane < NV) {
    double s = 0.0;
#pragma unroll 8
    for (int j = 0; j < m; j++) s += red[j * NV + lane];
    red[64 * NV + lane] = s;
  }
  wave_sync();
#pragma unroll
  for (int k = 0; k < NV; k++) out[k] = red[64 * NV + k];
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// colPivHouseholderQr().solve for 3x3 (A row-major), single right-hand side.  Every loop is unrolled and the
// pivot swap / rank cut / permuted store are selects on compile-time indices, so A, b, cn and perm stay in
// registers (a runtime column index would put them in scratch memory, on the LM's critical path).
__device__ __forceinline__ void colpiv_solve3(const double *Ain, const double *bin, double *x) {
  double A[9], b[3];
#pragma unroll
  for (int i = 0; i < 9; i++) A[i] = Ain[i];
#pragma unroll
  for (int i = 0; i < 3; i++) b[i] = bin[i];
  int perm[3] = {0, 1, 2};
  double cn[3];
#pragma unroll
  for (int j = 0; j < 3; j++) cn[j] = A[j] * A[j] + A[3 + j] * A[3 + j] + A[6 + j] * A[6 + j];
  int rank = 3;
  double maxpivot = 0;
  bool stop = false;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (stop) continue;
    int best = k;
    double bv = cn[k];
#pragma unroll
    for (int j = k + 1; j < 3; j++)
      if (cn[j] > bv) {
        best = j;
        bv = cn[j];
      }
#pragma unroll
    for (int c = k + 1; c < 3; c++)
      if (best == c) {
#pragma unroll
        for (int i = 0; i < 3; i++) {
          double t = A[3 * i + k];
          A[3 * i + k] = A[3 * i + c];
          A[3 * i + c] = t;
        }
        double t = cn[k];
        cn[k] = cn[c];
        cn[c] = t;
        int tp = perm[k];
        perm[k] = perm[c];
        perm[c] = tp;
      }
    double alpha = 0;
#pragma unroll
    for (int i = k; i < 3; i++) alpha += A[3 * i + k] * A[3 * i + k];
    alpha = sqrt(alpha);
    if (k == 0) maxpivot = alpha;
    if (alpha <= maxpivot * 1e-15 || alpha == 0) {
      rank = k;
      stop = true;
      continue;
    }
    if (A[3 * k + k] > 0) alpha = -alpha;
    double v[3] = {0, 0, 0};
#pragma unroll
    for (int i = k; i < 3; i++) v[i] = A[3 * i + k];
    v[k] -= alpha;
    double vn = 0;
#pragma unroll
    for (int i = k; i < 3; i++) vn += v[i] * v[i];
    if (vn > 0) {
#pragma unroll
      for (int j = k; j < 3; j++) {
        double s = 0;
#pragma unroll
        for (int i = k; i < 3; i++) s += v[i] * A[3 * i + j];
        s = 2 * s / vn;
#pragma unroll
        for (int i = k; i < 3; i++) A[3 * i + j] -= s * v[i];
      }
      double s = 0;
#pragma unroll
      for (int i = k; i < 3; i++) s += v[i] * b[i];
      s = 2 * s / vn;
#pragma unroll
      for (int i = k; i < 3; i++) b[i] -= s * v[i];
    }
#pragma unroll
    for (int j = k + 1; j < 3; j++) {
      double s = 0;
#pragma unroll
      for (int i = k + 1; i < 3; i++) s += A[3 * i + j] * A[3 * i + j];
      cn[j] = s;
    }
  }
  double y[3] = {0, 0, 0};
#pragma unroll
  for (int i = 2; i >= 0; i--) {
    if (i < rank) {
      double v = b[i];
#pragma unroll
      for (int k = i + 1; k < 3; k++)
        if (k < rank) v -= A[3 * i + k] * y[k];
      y[i] = v / A[3 * i + i];
    }
  }
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      if (perm[i] == j) x[j] = y[i];
}

// singular values (descending) of 3x3 A via Jacobi eigenvalues of A^T A
__device__ void singular_values3(const double *A, double *sv) {
  double a[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) a[i][j] = A[i] * A[j] + A[3 + i] * A[3 + j] + A[6 + i] * A[6 + j];
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    // converged once the off-diagonal is 1e-18 of the diagonal: a further rotation has c == 1 and moves no
    // diagonal entry by a bit (oracle la.h:singular_values3 stops at the same point)
    if (off < 1e-300 || off <= 1e-36 * (a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2])) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        if (a[p][q] == 0) continue;
        double theta = (a[q][q] - a[p][p]) / (2 * a[p][q]);
        double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
        double c = 1 / sqrt(t * t + 1), s = t * c;
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
  double e0 = fmax(a[0][0], 0.0), e1 = fmax(a[1][1], 0.0), e2 = fmax(a[2][2], 0.0);
  // sort descending
  double t;
  if (e0 < e1) { t = e0; e0 = e1; e1 = t; }
  if (e1 < e2) { t = e1; e1 = e2; e2 = t; }
  if (e0 < e1) { t = e0; e0 = e1; e1 = t; }
  sv[0] = sqrt(e0);
  sv[1] = sqrt(e1);
  sv[2] = sqrt(e2);
}

// camera pose of clone slot s in camera k (UpdaterMSCKF.cpp:98-115): R_GtoCi, p_CiinG
__device__ __forceinline__ void clone_cam_pose(const DClone &c, const DCam &k, double *R_GtoCi, double *p_CiinG) {
  m3_mul(k.R_ItoC, c.R, R_GtoCi);
  double t[3];
  m3t_vec(R_GtoCi, k.p_IinC, t);
  for (int i = 0; i < 3; i++) p_CiinG[i] = c.p[i] - t[i];
}

// per-lane LM terms (FeatureInitializer.cpp:241-271): returns H (2x3) and float residual
__device__ __forceinline__ void lm_terms(const double *R_AtoCi, const double *p_AinCi, double alpha, double beta,
                                         double rho, float un, float vn, double *H, double *res) {
  double hi1 = R_AtoCi[0] * alpha + R_AtoCi[1] * beta + R_AtoCi[2] + rho * p_AinCi[0];
  double hi2 = R_AtoCi[3] * alpha + R_AtoCi[4] * beta + R_AtoCi[5] + rho * p_AinCi[1];
  double hi3 = R_AtoCi[6] * alpha + R_AtoCi[7] * beta + R_AtoCi[8] + rho * p_AinCi[2];
  double h3s = hi3 * hi3;
  if (H) {
    H[0] = (R_AtoCi[0] * hi3 - hi1 * R_AtoCi[6]) / h3s;
    H[1] = (R_AtoCi[1] * hi3 - hi1 * R_AtoCi[7]) / h3s;
    H[2] = (p_AinCi[0] * hi3 - hi1 * p_AinCi[2]) / h3s;
    H[3] = (R_AtoCi[3] * hi3 - hi2 * R_AtoCi[6]) / h3s;
    H[4] = (R_AtoCi[4] * hi3 - hi2 * R_AtoCi[7]) / h3s;
    H[5] = (p_AinCi[1] * hi3 - hi2 * p_AinCi[2]) / h3s;
  }
  float z1 = (float)(hi1 / hi3), z2 = (float)(hi2 / hi3);
  float r1 = un - z1, r2 = vn - z2;
  res[0] = (double)r1;
  res[1] = (double)r2;
}
__device__ __forceinline__ double lm_err(const double *R_AtoCi, const double *p_AinCi, double alpha, double beta,
                                         double rho, float un, float vn) {
  double hi1 = R_AtoCi[0] * alpha + R_AtoCi[1] * beta + R_AtoCi[2] + rho * p_AinCi[0];
  double hi2 = R_AtoCi[3] * alpha + R_AtoCi[4] * beta + R_AtoCi[5] + rho * p_AinCi[1];
  double hi3 = R_AtoCi[6] * alpha + R_AtoCi[7] * beta + R_AtoCi[8] + rho * p_AinCi[2];
  float z1 = (float)(hi1 / hi3), z2 = (float)(hi2 / hi3);
  float r1 = un - z1, r2 = vn - z2;
  float nrm = sqrtf(r1 * r1 + r2 * r2);
  double dn = (double)nrm;
  return dn * dn;
}

// The three reflectors applied to the local Jacobian [Hl | r] (rows x ldl), one column per TPC adjacent threads.
// The column products keep one summation order whatever TPC is: four partial sums w_q over the rows i = q mod 4
// (rows past the last multiple of 4 go to w_0, in order), combined as (w_0 + w_1) + (w_2 + w_3); thread `part`
// of a column accumulates the w_q with q = part mod TPC and the four sums meet through lane shuffles, so the
// projected rows are the same bits for TPC = 1, 2, 4.  The update then splits the rows over the TPC threads.
template <int TPC>
__device__ __forceinline__ void ns_apply(double *Hl, const double *V, int rows, int ldl, int tid, double b1, double b2,
                                         double b3, double g21, double g31, double g32) {
  constexpr int NQ = 4 / TPC;
  const int part = tid & (TPC - 1), lane = tid & 63, base = lane & ~(TPC - 1);
  const int rows4 = rows & ~3;
  for (int j = tid / TPC; j < ldl; j += 256 / TPC) {
    double a1[NQ], a2[NQ], a3[NQ];
#pragma unroll
    for (int k = 0; k < NQ; k++) a1[k] = a2[k] = a3[k] = 0.0;
    for (int i = 0; i < rows4; i += 4) {
#pragma unroll
      for (int k = 0; k < NQ; k++) {
        const int r = i + part + TPC * k;
        const double a = Hl[(size_t)r * ldl + j];
        a1[k] += V[r * 3] * a;
        a2[k] += V[r * 3 + 1] * a;
        a3[k] += V[r * 3 + 2] * a;
      }
    }
    if (part == 0)
      for (int r = rows4; r < rows; r++) {
        const double a = Hl[(size_t)r * ldl + j];
        a1[0] += V[r * 3] * a;
        a2[0] += V[r * 3 + 1] * a;
        a3[0] += V[r * 3 + 2] * a;
      }
    double w1[4], w2[4], w3[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (TPC == 1) {
        w1[q] = a1[q];
        w2[q] = a2[q];
        w3[q] = a3[q];
      } else {
        w1[q] = __shfl(a1[q / TPC], base + q % TPC, 64);
        w2[q] = __shfl(a2[q / TPC], base + q % TPC, 64);
        w3[q] = __shfl(a3[q / TPC], base + q % TPC, 64);
      }
    }
    const double s1 = (w1[0] + w1[1]) + (w1[2] + w1[3]);
    const double s2 = (w2[0] + w2[1]) + (w2[2] + w2[3]);
    const double s3 = (w3[0] + w3[1]) + (w3[2] + w3[3]);
    const double u1 = b1 * s1;
    const double u2 = b2 * (s2 - g21 * u1);
    const double u3 = b3 * (s3 - g31 * u1 - g32 * u2);
#pragma unroll 4
    for (int k = part; k < rows; k += TPC) {
      double *p = Hl + (size_t)k * ldl + j;
      *p -= V[k * 3] * u1 + V[k * 3 + 1] * u2 + V[k * 3 + 2] * u3;
    }
  }
}

struct FeatShared {
  double p_FinA[3], p_FinG[3], p_FinA_fej[3], p_FinG_fej[3];
  int status;
  int nrows_out;
  double beta[3];
  double chi2;
};

// LDS layout helper (doubles)
__host__ __device__ inline size_t feat_lds_doubles(int max_meas, int max_nf) {
  int rows = 2 * max_meas;
  size_t n = 0;
  n += (size_t)rows * (max_nf + 1);  // Hl
  n += (size_t)rows * 3;             // Hf
  n += (size_t)rows * 3;             // V (Householder vectors)
  n += (size_t)max_nf;               // loc2pid (as double-size slots for alignment)
  n += 64;                           // scratch
  return n;
}
size_t feature_lds_bytes(int max_meas, int max_nf) { return feat_lds_doubles(max_meas, max_nf) * sizeof(double); }

__global__ void __launch_bounds__(256) k_feature(DBatchParams bp, const DFeat *__restrict__ feats,
                                                 const DMeas *__restrict__ meas, const DVar *__restrict__ vars,
                                                 const DClone *__restrict__ clones, const DCam *__restrict__ cams,
                                                 const double *__restrict__ P, const double *__restrict__ chi2_table,
                                                 double *__restrict__ H_all, DFeatOut *__restrict__ out, int max_meas,
                                                 int max_nf) {
  extern __shared__ double lds[];
  __shared__ FeatShared sh;
  long long *tsp = bp.dbg_ts ? bp.dbg_ts + (size_t)blockIdx.x * 16 : nullptr;
#define FEAT_TS(k) \
  if (tsp && threadIdx.x == 0) tsp[k] = clock64();
  __shared__ int canon2loc[512];
  __shared__ double red[9 * 64 + 16];
  const int f = blockIdx.x;
  const DFeat F = feats[f];
  const int m = F.nmeas, rows = 2 * m, nf = F.nf, ldl = nf + 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DMeas *Ms = meas + F.meas_off;

  double *Hl = lds;
  double *Hf = Hl + (size_t)2 * max_meas * (max_nf + 1);
  double *V = Hf + 2 * max_meas * 3;
  int *loc2pid = (int *)(V + 2 * max_meas * 3);

  FEAT_TS(0)
  // ---- setup: column maps, zero the local Jacobian ----
  for (int j = tid; j <= bp.n_canon; j += 256) canon2loc[j] = -1;
  for (int e = tid; e < rows * ldl; e += 256) Hl[e] = 0.0;
  __syncthreads();
  // one thread per (variable, element): the variable records load in parallel (sizes are <= 8)
  for (int e = tid; e < F.nvar * 8; e += 256) {
    const DVar dv = vars[F.var_off + (e >> 3)];
    const int k = e & 7;
    if (k < dv.size) {
      loc2pid[dv.loc + k] = dv.pid + k;
      if (dv.canon >= 0) canon2loc[dv.canon + k] = dv.loc + k;
    }
  }
  if (tid == 0) {
    sh.status = 0;
    double pin[3], pinf[3];
    for (int k = 0; k < 3; k++) pin[k] = F.p_in[k], pinf[k] = F.p_in_fej[k];
    if (F.mode == 3 && bp.tri_in) {  // the chained batch triangulation (p_FinA, p_FinG)
      const DFeatOut &t = bp.tri_in[f];
      for (int k = 0; k < 3; k++) pin[k] = t.p_FinA[k], pinf[k] = t.p_FinG[k];
      if (t.status == 1 || t.status == 2) sh.status = 1;
    }
    if (F.mode == 1 && bp.xv && F.lm_pid >= 0) {  // Landmark::get_xyz of the current value (Landmark.cpp:26-63)
      const double *v = bp.xv + F.lm_pid;
      if (F.rep == 4) {
        pin[0] = (1 / v[2]) * v[0];
        pin[1] = (1 / v[2]) * v[1];
        pin[2] = 1 / v[2];
        for (int k = 0; k < 3; k++) pinf[k] = pin[k];  // the reference ignores the fej value here
      } else {
        for (int k = 0; k < 3; k++) pin[k] = v[k];
      }
    }
    for (int k = 0; k < 3; k++) {
      sh.p_FinA[k] = pin[k];
      sh.p_FinA_fej[k] = pinf[k];
      sh.p_FinG[k] = (F.mode == 3) ? pinf[k] : pin[k];
      sh.p_FinG_fej[k] = pinf[k];
      if (F.mode == 3) sh.p_FinA_fej[k] = pin[k];
    }
  }
  __syncthreads();

  FEAT_TS(1)
  // ---- geometry: triangulation (waves 0-1) + Levenberg-Marquardt (all 4 waves; MSCKF / delayed init only) ----
  // Two of three LM trials are rejections (lam *= lam_mult, same Hessian; cfg2: 3.3 rejections and 1.8
  // acceptances per feature), so each iteration evaluates four trials at once: wave w solves with the damping
  // the reference would reach after w more rejections (lam multiplied w times, in the reference's order) and
  // forms its cost; every wave then replays the reference's control flow over the four results in order
  // (FeatureInitializer.cpp:197-375), so the accepted step, lam, runs and eps are the sequential ones.
  if (F.mode == 0 || F.mode == 2) {
    __shared__ double lm_H[9], lm_pf[3], lm_cond, lm_cand[2][4][4];
    const DClone &ca = clones[F.anchor_slot];
    const DCam &ka = cams[F.anchor_cam];
    double R_GtoA[9], p_AinG[3];
    clone_cam_pose(ca, ka, R_GtoA, p_AinG);
    double R_AtoCi[9] = {0}, p_CiinA[3] = {0, 0, 0}, p_AinCi[3] = {0, 0, 0};
    float un = 0.f, vn = 0.f;
    bool act = lane < m;
    if (act) {
      const DMeas &mm = Ms[lane];
      double R_GtoCi[9], p_CiinG[3];
      clone_cam_pose(clones[mm.slot], cams[mm.cam], R_GtoCi, p_CiinG);
      m3_mul_bt(R_GtoCi, R_GtoA, R_AtoCi);
      double d[3] = {p_CiinG[0] - p_AinG[0], p_CiinG[1] - p_AinG[1], p_CiinG[2] - p_AinG[2]};
      m3_vec(R_GtoA, d, p_CiinA);
      double t[3];
      m3_vec(R_AtoCi, p_CiinA, t);
      p_AinCi[0] = -t[0];
      p_AinCi[1] = -t[1];
      p_AinCi[2] = -t[2];
      un = mm.un;
      vn = mm.vn;
    }
    if (wave == 0) {
      // linear triangulation
      double Ai[6] = {0, 0, 0, 0, 0, 0}, bi[3] = {0, 0, 0};
      if (act) {
        double b0[3] = {(double)un, (double)vn, 1.0}, b[3];
        m3t_vec(R_AtoCi, b0, b);
        double nb = norm3(b);
        b[0] /= nb; b[1] /= nb; b[2] /= nb;
        double Bp[9], A9[9];
        skew(b, Bp);
        m3_mul_at(Bp, Bp, A9);
        Ai[0] = A9[0]; Ai[1] = A9[1]; Ai[2] = A9[2]; Ai[3] = A9[4]; Ai[4] = A9[5]; Ai[5] = A9[8];
        m3_vec(A9, p_CiinA, bi);
      }
      double v9[9] = {Ai[0], Ai[1], Ai[2], Ai[3], Ai[4], Ai[5], bi[0], bi[1], bi[2]}, s9[9];
      ordered_sum<9>(red, v9, lane, m, s9);
      if (lane == 0)
        for (int k = 0; k < 9; k++) lm_H[k] = s9[k];
    }
    __syncthreads();
    // the solve (wave 0) and the condition number (wave 1) of A p = b side by side
    if (wave < 2) {
      const double A[9] = {lm_H[0], lm_H[1], lm_H[2], lm_H[1], lm_H[3], lm_H[4], lm_H[2], lm_H[4], lm_H[5]};
      if (wave == 0) {
        const double bb[3] = {lm_H[6], lm_H[7], lm_H[8]};
        double p3[3];
        colpiv_solve3(A, bb, p3);
        if (lane == 0)
          for (int k = 0; k < 3; k++) lm_pf[k] = p3[k];
      } else {
        double sv[3];
        singular_values3(A, sv);
        if (lane == 0) lm_cond = sv[0] / sv[2];
      }
    }
    __syncthreads();
    double pf[3] = {lm_pf[0], lm_pf[1], lm_pf[2]};
    int st = 0;
    {
      const double condA = lm_cond;
      const double npf = norm3(pf);
      if (fabs(condA) > bp.fi_max_cond || pf[2] < bp.fi_min_dist || pf[2] > bp.fi_max_dist || isnan(npf)) st = 1;
    }
    if (st == 0 && bp.fi_refine) {  // block-uniform from here to the end of the LM loop
      double *wred = red + 72 * wave;  // this wave's ordered_sum<1> slots (wave 0's <9> sums run between barriers)
      double rho = 1 / pf[2], alpha = pf[0] / pf[2], beta = pf[1] / pf[2];
      double lam = bp.fi_init_lamda, eps = 10000;
      int runs = 0, par = 0;
      bool recompute = true, done = false;
      double Hs[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
      double cost_old;
      {
        double e1 = act ? lm_err(R_AtoCi, p_AinCi, alpha, beta, rho, un, vn) : 0.0;
        ordered_sum<1>(wred, &e1, lane, m, &cost_old);
      }
      __syncthreads();
      while (!done && runs < bp.fi_max_runs && lam < bp.fi_max_lamda && eps > bp.fi_min_dx) {
        if (recompute) {
          if (wave == 0) {
            double h[6] = {0, 0, 0, 0, 0, 0}, gg[3] = {0, 0, 0};
            if (act) {
              double H[6], r[2];
              lm_terms(R_AtoCi, p_AinCi, alpha, beta, rho, un, vn, H, r);
              // H^T H (upper 6) and H^T r
              h[0] = H[0] * H[0] + H[3] * H[3];
              h[1] = H[0] * H[1] + H[3] * H[4];
              h[2] = H[0] * H[2] + H[3] * H[5];
              h[3] = H[1] * H[1] + H[4] * H[4];
              h[4] = H[1] * H[2] + H[4] * H[5];
              h[5] = H[2] * H[2] + H[5] * H[5];
              gg[0] = H[0] * r[0] + H[3] * r[1];
              gg[1] = H[1] * r[0] + H[4] * r[1];
              gg[2] = H[2] * r[0] + H[5] * r[1];
            }
            double v9[9] = {h[0], h[1], h[2], h[3], h[4], h[5], gg[0], gg[1], gg[2]}, s9[9];
            ordered_sum<9>(red, v9, lane, m, s9);
            if (lane == 0)
              for (int k = 0; k < 9; k++) lm_H[k] = s9[k];
          }
          __syncthreads();
          for (int k = 0; k < 6; k++) Hs[k] = lm_H[k];
          for (int k = 0; k < 3; k++) g[k] = lm_H[6 + k];
        }
        // trial of this wave: the damping after `wave` further rejections
        double lw = lam;
        for (int k = 0; k < wave; k++) lw = lw * bp.fi_lam_mult;
        double Hl3[9] = {Hs[0], Hs[1], Hs[2], Hs[1], Hs[3], Hs[4], Hs[2], Hs[4], Hs[5]};
        Hl3[0] *= (1.0 + lw);
        Hl3[4] *= (1.0 + lw);
        Hl3[8] *= (1.0 + lw);
        double dx[3];
        colpiv_solve3(Hl3, g, dx);
        double cost;
        {
          double e1 = act ? lm_err(R_AtoCi, p_AinCi, alpha + dx[0], beta + dx[1], rho + dx[2], un, vn) : 0.0;
          ordered_sum<1>(wred, &e1, lane, m, &cost);
        }
        if (lane == 0) {
          double *c = lm_cand[par][wave];
          c[0] = cost;
          c[1] = dx[0];
          c[2] = dx[1];
          c[3] = dx[2];
        }
        __syncthreads();
        // the reference's sequence over the four trials (the loop condition is re-checked before each)
        for (int w = 0; w < 4; w++) {
          if (w > 0 && !(runs < bp.fi_max_runs && lam < bp.fi_max_lamda && eps > bp.fi_min_dx)) {
            done = true;
            break;
          }
          const double *c = lm_cand[par][w];
          const double cw = c[0], d0 = c[1], d1 = c[2], d2 = c[3];
          if (cw <= cost_old && (cost_old - cw) / cost_old < bp.fi_min_dcost) {
            alpha += d0;
            beta += d1;
            rho += d2;
            eps = 0;
            done = true;
            break;
          }
          if (cw <= cost_old) {
            recompute = true;
            cost_old = cw;
            alpha += d0;
            beta += d1;
            rho += d2;
            runs++;
            lam = lam / bp.fi_lam_mult;
            eps = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
            break;
          }
          recompute = false;
          lam = lam * bp.fi_lam_mult;
        }
        par ^= 1;
      }
      pf[0] = alpha / rho;
      pf[1] = beta / rho;
      pf[2] = 1 / rho;
      if (wave == 0) {
        double np = norm3(pf);
        double vh[3] = {pf[0] / np, pf[1] / np, pf[2] / np};
        double bl = 0.0;
        if (act) {
          double dd = dot3(p_CiinA, vh);
          double perp[3] = {p_CiinA[0] - dd * vh[0], p_CiinA[1] - dd * vh[1], p_CiinA[2] - dd * vh[2]};
          bl = norm3(perp);
        }
        double base_line_max = wave_max(bl);
        if (pf[2] < bp.fi_min_dist || pf[2] > bp.fi_max_dist || (np / base_line_max) > bp.fi_max_baseline ||
            isnan(np))
          st = 2;
      }
    }
    if (tid == 0) {
      sh.status = st;
      double pG[3];
      m3t_vec(R_GtoA, pf, pG);
      for (int k = 0; k < 3; k++) {
        sh.p_FinA[k] = pf[k];
        sh.p_FinA_fej[k] = pf[k];
        sh.p_FinG[k] = pG[k] + p_AinG[k];
        sh.p_FinG_fej[k] = sh.p_FinG[k];
      }
    }
  }
  __syncthreads();
  const int status0 = sh.status;
  if (F.mode == 2) {  // batch triangulation for the delayed initialization: no rows are formed
    if (tid == 0) {
      DFeatOut o;
      for (int k = 0; k < 3; k++) o.p_FinA[k] = sh.p_FinA[k], o.p_FinG[k] = sh.p_FinG[k];
      o.chi2 = -1.0;
      for (int k = 0; k < 9; k++) o.HfR[k] = 0.0;
      o.status = status0;
      o.rows = 0;
      out[f] = o;
    }
    return;
  }

  FEAT_TS(2)
  // ---- Jacobians (one thread per measurement) ----
  if (status0 == 0 && tid < m) {
    const DMeas &mm = Ms[tid];
    const DClone &cl = clones[mm.slot];
    const DCam &ck = cams[mm.cam];
    const bool rel = (F.rep == 2 || F.rep == 3 || F.rep == 4 || F.rep == 5);
    double p_FinG[3], p_FinG_fej[3];
    // representation Jacobian (UpdaterHelper.cpp:32-190) and anchor terms
    double dl[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};  // dpfg_dlambda
    double Hanc[18], Hcal[18];                   // 3x6 each
    int ncolf = (F.rep == 5) ? 1 : 3;
    if (!rel) {
      for (int k = 0; k < 3; k++) {
        p_FinG[k] = sh.p_FinG[k];
        p_FinG_fej[k] = sh.p_FinG_fej[k];
      }
      if (F.rep == 1) {  // GLOBAL_FULL_INVERSE_DEPTH
        const double *pg = bp.do_fej ? p_FinG_fej : p_FinG;
        double g_rho = 1 / norm3(pg), g_phi = acos(g_rho * pg[2]), g_theta = atan2(pg[1], pg[0]);
        double sth = sin(g_theta), cth = cos(g_theta), sph = sin(g_phi), cph = cos(g_phi), rho = g_rho;
        dl[0] = -(1.0 / rho) * sth * sph; dl[1] = (1.0 / rho) * cth * cph; dl[2] = -(1.0 / (rho * rho)) * cth * sph;
        dl[3] = (1.0 / rho) * cth * sph;  dl[4] = (1.0 / rho) * sth * cph; dl[5] = -(1.0 / (rho * rho)) * sth * sph;
        dl[6] = 0.0; dl[7] = -(1.0 / rho) * sph; dl[8] = -(1.0 / (rho * rho)) * cph;
      }
    } else {
      const DClone &an = clones[F.anchor_slot];
      const DCam &ak = cams[F.anchor_cam];
      const double *pA = sh.p_FinA;
      // p_FinG = R_GtoI^T R_ItoC^T (p_FinA - p_IinC) + p_IinG (UpdaterHelper.cpp:271-283)
      double d0[3] = {pA[0] - ak.p_IinC[0], pA[1] - ak.p_IinC[1], pA[2] - ak.p_IinC[2]}, t1[3], t2[3];
      m3t_vec(ak.R_ItoC, d0, t1);
      m3t_vec(an.R, t1, t2);
      for (int k = 0; k < 3; k++) {
        p_FinG[k] = t2[k] + an.p[k];
        p_FinG_fej[k] = p_FinG[k];
      }
      double R_GtoI[9], p_IinG[3], pFA[3];
      for (int k = 0; k < 9; k++) R_GtoI[k] = an.R[k];
      for (int k = 0; k < 3; k++) {
        p_IinG[k] = an.p[k];
        pFA[k] = pA[k];
      }
      if (bp.do_fej) {
        for (int k = 0; k < 9; k++) R_GtoI[k] = an.Rf[k];
        for (int k = 0; k < 3; k++) p_IinG[k] = an.pf[k];
        // p_FinA = (R_GtoI^T R_ItoC^T)^T (p_FinG_best - p_IinG) + p_IinC
        double RCG[9], RCG_T[9], dd[3], tt[3];
        double RIT[9], RCT[9];
        m3_transpose(R_GtoI, RIT);
        m3_transpose(ak.R_ItoC, RCT);
        m3_mul(RIT, RCT, RCG);
        m3_transpose(RCG, RCG_T);
        for (int k = 0; k < 3; k++) dd[k] = p_FinG[k] - p_IinG[k];
        m3_vec(RCG_T, dd, tt);
        for (int k = 0; k < 3; k++) pFA[k] = tt[k] + ak.p_IinC[k];
      }
      double RIT[9], RCT[9], R_CtoG[9];
      m3_transpose(R_GtoI, RIT);
      m3_transpose(ak.R_ItoC, RCT);
      m3_mul(RIT, RCT, R_CtoG);
      // H_anc = [-R_GtoI^T skew(R_ItoC^T (p_FinA - p_IinC)), I]
      double dd[3] = {pFA[0] - ak.p_IinC[0], pFA[1] - ak.p_IinC[1], pFA[2] - ak.p_IinC[2]}, w[3], Sk[9], Tm[9];
      m3t_vec(ak.R_ItoC, dd, w);
      skew(w, Sk);
      m3_mul(RIT, Sk, Tm);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          Hanc[6 * i + j] = -Tm[3 * i + j];
          Hanc[6 * i + 3 + j] = (i == j) ? 1.0 : 0.0;
        }
      // H_calib = [-R_CtoG skew(p_FinA - p_IinC), -R_CtoG]
      skew(dd, Sk);
      m3_mul(R_CtoG, Sk, Tm);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          Hcal[6 * i + j] = -Tm[3 * i + j];
          Hcal[6 * i + 3 + j] = -R_CtoG[3 * i + j];
        }
      if (F.rep == 2) {
        for (int k = 0; k < 9; k++) dl[k] = R_CtoG[k];
      } else if (F.rep == 4 || F.rep == 5) {
        double alpha = pFA[0] / pFA[2], beta = pFA[1] / pFA[2], rho = 1 / pFA[2];
        double d[9] = {1.0 / rho, 0.0, -(1.0 / (rho * rho)) * alpha, 0.0, 1.0 / rho, -(1.0 / (rho * rho)) * beta,
                       0.0, 0.0, -(1.0 / (rho * rho))};
        if (F.rep == 4) {
          m3_mul(R_CtoG, d, dl);
        } else {
          double bear[3] = {rho * pFA[0], rho * pFA[1], rho * pFA[2]};
          double dr[3] = {-(1.0 / (rho * rho)) * bear[0], -(1.0 / (rho * rho)) * bear[1], -(1.0 / (rho * rho)) * bear[2]};
          double o[3];
          m3_vec(R_CtoG, dr, o);
          dl[0] = o[0]; dl[3] = o[1]; dl[6] = o[2];
        }
      } else if (F.rep == 3) {
        double a_rho = 1 / norm3(pFA), a_phi = acos(a_rho * pFA[2]), a_theta = atan2(pFA[1], pFA[0]);
        double sth = sin(a_theta), cth = cos(a_theta), sph = sin(a_phi), cph = cos(a_phi), rho = a_rho;
        double d[9] = {-(1.0 / rho) * sth * sph, (1.0 / rho) * cth * cph, -(1.0 / (rho * rho)) * cth * sph,
                       (1.0 / rho) * cth * sph,  (1.0 / rho) * sth * cph, -(1.0 / (rho * rho)) * sth * sph,
                       0.0, -(1.0 / rho) * sph, -(1.0 / (rho * rho)) * cph};
        m3_mul(R_CtoG, d, dl);
      }
    }
    // measurement model (UpdaterHelper.cpp:310-404)
    double R_GtoIi[9], p_IiinG[3];
    for (int k = 0; k < 9; k++) R_GtoIi[k] = cl.R[k];
    for (int k = 0; k < 3; k++) p_IiinG[k] = cl.p[k];
    double d1[3] = {p_FinG[0] - p_IiinG[0], p_FinG[1] - p_IiinG[1], p_FinG[2] - p_IiinG[2]}, p_FinIi[3], p_FinCi[3];
    m3_vec(R_GtoIi, d1, p_FinIi);
    m3_vec(ck.R_ItoC, p_FinIi, p_FinCi);
    for (int k = 0; k < 3; k++) p_FinCi[k] += ck.p_IinC[k];
    double xn = p_FinCi[0] / p_FinCi[2], yn = p_FinCi[1] / p_FinCi[2];
    float ud, vd;
    cam_distort_f(ck.cam, (float)xn, (float)yn, ud, vd);
    double res0 = (double)mm.u - (double)ud, res1 = (double)mm.v - (double)vd;
    if (bp.dbg) {
      double *d = bp.dbg + (size_t)(F.meas_off + tid) * 8;
      d[0] = mm.cam; d[1] = xn; d[2] = yn; d[3] = ud; d[4] = vd; d[5] = mm.u; d[6] = mm.v; d[7] = p_FinCi[2];
    }
    if (bp.do_fej) {
      for (int k = 0; k < 9; k++) R_GtoIi[k] = cl.Rf[k];
      for (int k = 0; k < 3; k++) p_IiinG[k] = cl.pf[k];
      double d2[3] = {p_FinG_fej[0] - p_IiinG[0], p_FinG_fej[1] - p_IiinG[1], p_FinG_fej[2] - p_IiinG[2]};
      m3_vec(R_GtoIi, d2, p_FinIi);
      m3_vec(ck.R_ItoC, p_FinIi, p_FinCi);
      for (int k = 0; k < 3; k++) p_FinCi[k] += ck.p_IinC[k];
    }
    double dzn[4], dzeta[16];
    cam_distort_jac(ck.cam, xn, yn, dzn, dzeta);
    double iz = 1 / p_FinCi[2];
    double dzn_dpfc[6] = {iz, 0, -p_FinCi[0] / (p_FinCi[2] * p_FinCi[2]), 0, iz, -p_FinCi[1] / (p_FinCi[2] * p_FinCi[2])};
    double dpfc_dpfg[9];
    m3_mul(ck.R_ItoC, R_GtoIi, dpfc_dpfg);
    double Sk[9], RS[9];
    skew(p_FinIi, Sk);
    m3_mul(ck.R_ItoC, Sk, RS);
    double dz_dpfc[6];  // 2x3
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 3; j++) dz_dpfc[3 * i + j] = dzn[2 * i] * dzn_dpfc[j] + dzn[2 * i + 1] * dzn_dpfc[3 + j];
    double dz_dpfg[6];
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 3; j++)
        dz_dpfg[3 * i + j] = dz_dpfc[3 * i] * dpfc_dpfg[j] + dz_dpfc[3 * i + 1] * dpfc_dpfg[3 + j] +
                             dz_dpfc[3 * i + 2] * dpfc_dpfg[6 + j];
    for (int i = 0; i < 2; i++) {
      double *row = Hl + (size_t)(2 * tid + i) * ldl;
      double *hf = Hf + (2 * tid + i) * 3;
      // H_f = dz_dpfg * dpfg_dlambda
#pragma unroll
      for (int j = 0; j < 3; j++)  // compile-time columns: dl stays in registers
        hf[j] = (j < ncolf) ? dz_dpfg[3 * i] * dl[j] + dz_dpfg[3 * i + 1] * dl[3 + j] + dz_dpfg[3 * i + 2] * dl[6 + j] : 0.0;
      // clone block: dz_dpfc * [R_ItoC skew(p_FinIi), -dpfc_dpfg]
      for (int j = 0; j < 3; j++) {
        row[mm.lc_clone + j] =
            dz_dpfc[3 * i] * RS[j] + dz_dpfc[3 * i + 1] * RS[3 + j] + dz_dpfc[3 * i + 2] * RS[6 + j];
        row[mm.lc_clone + 3 + j] = -(dz_dpfc[3 * i] * dpfc_dpfg[j] + dz_dpfc[3 * i + 1] * dpfc_dpfg[3 + j] +
                                     dz_dpfc[3 * i + 2] * dpfc_dpfg[6 + j]);
      }
      if (rel) {
        for (int j = 0; j < 6; j++)
          row[F.lc_anchor_clone + j] +=
              dz_dpfg[3 * i] * Hanc[j] + dz_dpfg[3 * i + 1] * Hanc[6 + j] + dz_dpfg[3 * i + 2] * Hanc[12 + j];
        if (bp.calib_ext)
          for (int j = 0; j < 6; j++)
            row[F.lc_anchor_ext + j] +=
                dz_dpfg[3 * i] * Hcal[j] + dz_dpfg[3 * i + 1] * Hcal[6 + j] + dz_dpfg[3 * i + 2] * Hcal[12 + j];
      }
      if (bp.calib_ext && mm.lc_ext >= 0) {
        double pc[3] = {p_FinCi[0] - ck.p_IinC[0], p_FinCi[1] - ck.p_IinC[1], p_FinCi[2] - ck.p_IinC[2]}, Sc[9];
        skew(pc, Sc);
        for (int j = 0; j < 3; j++) {
          row[mm.lc_ext + j] += dz_dpfc[3 * i] * Sc[j] + dz_dpfc[3 * i + 1] * Sc[3 + j] + dz_dpfc[3 * i + 2] * Sc[6 + j];
          row[mm.lc_ext + 3 + j] += dz_dpfc[3 * i + j];
        }
      }
      if (bp.calib_intr && mm.lc_intr >= 0)
        for (int j = 0; j < 8; j++) row[mm.lc_intr + j] = dzeta[8 * i + j];
      row[nf] = (i == 0) ? res0 : res1;
      // SLAM update: landmark columns hold H_f (UpdaterSLAM.cpp:355-358)
      if (F.mode == 1)
        for (int j = 0; j < ncolf; j++) row[F.lm_loc + j] = hf[j];
    }
  }
  __syncthreads();

  FEAT_TS(3)
  // ---- left-nullspace projection: 3 Householder reflections of H_f (MSCKF) ----
  // Wave 0 forms the reflectors v_c (beta_c) on H_f's 3 columns in sequence.  The local Jacobian
  // [Hl | r] then takes all three in one read and one write pass per column: with w_c = v_c^T A,
  //   u_1 = b_1 w_1,  u_2 = b_2 (w_2 - g21 u_1),  u_3 = b_3 (w_3 - g31 u_1 - g32 u_2),  g_ab = v_a^T v_b,
  // H_3 H_2 H_1 A = A - v_1 u_1 - v_2 u_2 - v_3 u_3.
  int r0 = 0;  // first output row in Hl
  if (status0 == 0 && F.mode != 1) {
    if (wave == 0) {
      for (int c = 0; c < 3; c++) {
        // v = x - alpha e_c over rows c..rows-1 (zero above)
        double ss = 0.0;
        for (int i = c + lane; i < rows; i += 64) {
          double x = Hf[i * 3 + c];
          ss += x * x;
        }
        ss = wave_sum(ss);
        const double x0 = Hf[c * 3 + c];
        const double alpha = (x0 > 0) ? -sqrt(ss) : sqrt(ss);
        for (int i = lane; i < rows; i += 64) {
          V[i * 3 + c] = (i < c) ? 0.0 : (i == c) ? (x0 - alpha) : Hf[i * 3 + c];
          // the reflected column c is alpha e_c (H_finit = the upper 3x3 of the reflected H_f)
          if (i >= c) Hf[i * 3 + c] = (i == c) ? alpha : 0.0;
        }
        const double vn = ss - x0 * x0 + (x0 - alpha) * (x0 - alpha);
        const double b = (vn > 0) ? 2.0 / vn : 0.0;
        if (lane == 0) sh.beta[c] = b;
        wave_sync();
        for (int j = c + 1; j < 3; j++) {  // reflect H_f's later columns
          double d = 0.0;
          for (int i = c + lane; i < rows; i += 64) d += V[i * 3 + c] * Hf[i * 3 + j];
          d = b * wave_sum(d);
          for (int i = c + lane; i < rows; i += 64) Hf[i * 3 + j] -= d * V[i * 3 + c];
        }
        wave_sync();
      }
      double g0 = 0.0, g1 = 0.0, g2 = 0.0;
      for (int i = lane; i < rows; i += 64) {
        const double a = V[i * 3], bq = V[i * 3 + 1], cq = V[i * 3 + 2];
        g0 += bq * a;
        g1 += cq * a;
        g2 += cq * bq;
      }
      g0 = wave_sum(g0);
      g1 = wave_sum(g1);
      g2 = wave_sum(g2);
      if (lane == 0) red[0] = g0, red[1] = g1, red[2] = g2;
      if (F.mode == 3) FEAT_TS(8)  // debug sub-phases of a single candidate (no chi2 stamps there)
    }
    __syncthreads();
    if (F.mode == 3) FEAT_TS(9)
    const double b1 = sh.beta[0], b2 = sh.beta[1], b3 = sh.beta[2];
    const double g21 = red[0], g31 = red[1], g32 = red[2];
    if (ldl <= 64)
      ns_apply<4>(Hl, V, rows, ldl, tid, b1, b2, b3, g21, g31, g32);
    else if (ldl <= 128)
      ns_apply<2>(Hl, V, rows, ldl, tid, b1, b2, b3, g21, g31, g32);
    else
      ns_apply<1>(Hl, V, rows, ldl, tid, b1, b2, b3, g21, g31, g32);
    if (F.mode == 3) FEAT_TS(10)
    __syncthreads();
    r0 = 3;
  }
  const int R = rows - r0;

  FEAT_TS(4)
  FEAT_TS(5)
  const int status = sh.status;  // 0 or a triangulation / refinement failure; chi2 is k_chi2's
  FEAT_TS(6)
  // ---- output rows (canonical dense columns; zeros when rejected) ----
  const int out_r0 = (F.mode == 0) ? 3 : 0;
  const int nrows_out = max(rows - out_r0, 0);
  {
    // one wave per row, lanes over the canonical columns (n_canon + 1 <= 512: 8 column slots per lane,
    // their local column cached in registers); rejected features write zero rows
    const int nc = bp.n_canon + 1;
    int lcs[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int j = lane + 64 * q;
      lcs[q] = (status != 0 || j >= nc) ? -1 : (j == bp.n_canon) ? nf : canon2loc[j];
    }
    for (int i = wave; i < nrows_out; i += 4) {
      const double *src = Hl + (size_t)(out_r0 + i) * ldl;
      double *dst = H_all + (size_t)(F.row_off + i) * bp.ldh;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int j = lane + 64 * q;
        if (j < nc) dst[j] = (lcs[q] >= 0) ? src[lcs[q]] : 0.0;
      }
    }
  }
  if (tid == 0) {
    DFeatOut o;
    for (int k = 0; k < 3; k++) {
      o.p_FinA[k] = sh.p_FinA[k];
      o.p_FinG[k] = sh.p_FinG[k];
    }
    o.chi2 = -1.0;
    for (int k = 0; k < 9; k++) o.HfR[k] = (F.mode >= 2 && status0 == 0) ? Hf[(k / 3) * 3 + (k % 3)] : 0.0;
    o.status = status;
    o.rows = status == 0 ? nrows_out : 0;
    out[f] = o;
    if (bp.gate_out) *bp.gate_out = (status == 0) ? 1 : 0;
  }
  FEAT_TS(7)
#undef FEAT_TS
}

void launch_feature_linearize(hipStream_t s, const DBatchParams &bp, const DFeat *feats, const DMeas *meas,
                              const DVar *vars, const DClone *clones, const DCam *cams, const double *P,
                              const double *chi2_table, double *H_all, DFeatOut *out, int max_meas, int max_nf) {
  if (bp.nfeat <= 0) return;
  if (bp.n_canon >= 512 || max_meas > 64)  // canon2loc[512]; one lane per measurement
    throw std::runtime_error("k_feature: n_canon " + std::to_string(bp.n_canon) + " / measurements per feature " +
                             std::to_string(max_meas) + " beyond the kernel's limits (511 / 64)");
  size_t bytes = feature_lds_bytes(max_meas, max_nf);
  static int granted = -1;
  if (granted < 0) granted = set_dyn_lds((const void *)k_feature, 156 * 1024);
  if (bytes > 64 * 1024 && (int)bytes > granted)
    throw std::runtime_error("k_feature needs " + std::to_string(bytes) + " B of LDS, granted " + std::to_string(granted));
  hipLaunchKernelGGL(k_feature, dim3(bp.nfeat), dim3(256), bytes, s, bp, feats, meas, vars, clones, cams, P,
                     chi2_table, H_all, out, max_meas, max_nf);
}

// ---------------------------------------------------------------------------------------------------
// VioManager::retriangulate_active_tracks (VioManagerHelper.cpp:190-388).  The reference walks the frame's
// observations camera by camera; per track it sets A_new = A_i + A_old (A_old: the track's system of the
// LAST frame, so a second camera's observation overwrites the first's, a reference quirk kept here), count_new
// = 1 + count_old, and once count_new > 3 solves A_new p = b_new (colPivHouseholderQr) and keeps p if cond(A)
// <= max_cond and the depth in the observing camera lies in [min_dist, max_dist]; a later observation's
// result overwrites an earlier one's.  Here every observation is one thread (k_retri_obs: hash lookup of the
// track's old system, insertion of its new slot, its own A_new / solve; atomicMax marks the track's last
// observation and its last successful one), then k_retri_final keeps those two per track and k_retri_uvd
// projects the tracks and the SLAM landmarks seen by camera 0 into it.
__device__ __forceinline__ unsigned retri_hash(unsigned long long k, int cap) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (unsigned)(k & (unsigned long long)(cap - 1));
}
__device__ int retri_find(const unsigned long long *keys, int cap, unsigned long long id) {
  unsigned h = retri_hash(id, cap);
  for (int p = 0; p < cap; p++, h = (h + 1) & (cap - 1)) {
    const unsigned long long k = keys[h];
    if (k == id) return (int)h;
    if (k == kRetriEmpty) return -1;
  }
  return -1;
}
__device__ int retri_insert(unsigned long long *keys, int cap, unsigned long long id) {
  unsigned h = retri_hash(id, cap);
  for (int p = 0; p < cap; p++, h = (h + 1) & (cap - 1)) {
    const unsigned long long prev = atomicCAS(&keys[h], kRetriEmpty, id);
    if (prev == kRetriEmpty || prev == id) return (int)h;
  }
  return -1;
}

__global__ void __launch_bounds__(256) k_retri_reset(RetriJob job) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < job.cap) {
    job.keys_new[i] = kRetriEmpty;
    DRetriEntry &e = job.ent_new[i];
    e.last_obs = e.last_pass = -1;
    e.first_obs = 0x7fffffff;
    e.has_uv0 = 0;
    e.uvd_valid = 0;
  }
  if (i < job.nslam) {
    job.slam[i].has_uv0 = 0;
    job.slam[i].uvd_valid = 0;
  }
}

__global__ void __launch_bounds__(256) k_retri_obs(RetriJob job) {
  // the SLAM landmarks' ids in LDS: every observation scans them (the scan over global memory was ~50
  // dependent loads per thread)
  extern __shared__ unsigned long long sh_slam_id[];
  for (int s = threadIdx.x; s < job.nslam; s += blockDim.x) sh_slam_id[s] = job.slam[s].featid;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= job.nobs) return;
  const DRetriObs o = job.obs[i];
  // feat_uvs_in_cam0 is recorded before the SLAM skip
  for (int s = 0; s < job.nslam; s++)
    if (sh_slam_id[s] == o.featid) {
      if (o.cam == 0) {
        job.slam[s].u0 = o.u;
        job.slam[s].v0 = o.v;
        job.slam[s].has_uv0 = 1;
      }
      return;
    }
  const int slot = retri_insert(job.keys_new, job.cap, o.featid);
  if (slot < 0) return;
  DRetriEntry &e = job.ent_new[slot];
  if (o.cam == 0) {
    e.u0 = o.u;
    e.v0 = o.v;
    e.has_uv0 = 1;
  }
  const double *R = job.R_GtoC[o.cam], *pC = job.p_CinG[o.cam];
  double b0[3] = {(double)o.un, (double)o.vn, 1.0}, bi[3];
  m3t_vec(R, b0, bi);
  const double inv = 1.0 / norm3(bi);
  for (int k = 0; k < 3; k++) bi[k] = inv * bi[k];
  double Bp[9], Ai[9], bb[3];
  skew(bi, Bp);
  m3_mul_at(Bp, Bp, Ai);
  m3_vec(Ai, pC, bb);
  double *sc = job.scratch + (size_t)17 * i;
  const int old = retri_find(job.keys_old, job.cap, o.featid);
  int cnt = 1;
  if (old >= 0) {
    const DRetriEntry &eo = job.ent_old[old];
    for (int k = 0; k < 9; k++) Ai[k] = Ai[k] + eo.A[k];
    for (int k = 0; k < 3; k++) bb[k] = bb[k] + eo.b[k];
    cnt = 1 + eo.cnt;
  }
  for (int k = 0; k < 9; k++) sc[k] = Ai[k];
  for (int k = 0; k < 3; k++) sc[9 + k] = bb[k];
  int pass = 0;
  if (cnt > 3) {
    double p[3], d[3], pc[3], sv[3];
    colpiv_solve3(Ai, bb, p);
    for (int k = 0; k < 3; k++) d[k] = p[k] - pC[k];
    m3_vec(R, d, pc);
    singular_values3(Ai, sv);
    const double cond = sv[0] / sv[2];
    if (fabs(cond) <= job.max_cond && pc[2] >= job.min_dist && pc[2] <= job.max_dist && !isnan(norm3(pc))) {
      pass = 1;
      for (int k = 0; k < 3; k++) sc[13 + k] = p[k];
    }
  }
  sc[16] = pass;
  sc[12] = (double)cnt + (old >= 0 ? 0.5 : 0.0);  // the fraction marks a track with an old system
  atomicMax(&e.last_obs, i);
  atomicMin(&e.first_obs, i);
  if (pass) atomicMax(&e.last_pass, i);
}

__global__ void __launch_bounds__(256) k_retri_final(RetriJob job) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= job.nobs) return;
  const DRetriObs o = job.obs[i];
  const int slot = retri_find(job.keys_new, job.cap, o.featid);
  if (slot < 0) return;  // a SLAM landmark (never inserted)
  DRetriEntry &e = job.ent_new[slot];
  const double *sc = job.scratch + (size_t)17 * i;
  // a track with an old system keeps its last observation's (operator[] overwrites), a new one its first
  const bool had_old = sc[12] != (double)(int)sc[12];
  if ((had_old ? e.last_obs : e.first_obs) == i) {
    for (int k = 0; k < 9; k++) e.A[k] = sc[k];
    for (int k = 0; k < 3; k++) e.b[k] = sc[9 + k];
    e.cnt = (int)sc[12];
  }
  if (e.last_pass == i)
    for (int k = 0; k < 3; k++) e.pos[k] = sc[13 + k];
}

__device__ __forceinline__ int retri_uvd(const RetriJob &job, const double *pos, float u0, float v0, double *uvd) {
  double d[3], pI[3], pC[3];
  for (int k = 0; k < 3; k++) d[k] = pos[k] - job.p_IinG[k];
  m3_vec(job.R_GtoI, d, pI);
  m3_vec(job.R_ItoC0, pI, pC);
  for (int k = 0; k < 3; k++) pC[k] = pC[k] + job.p_IinC0[k];
  const double depth = pC[2], u = (double)u0, v = (double)v0;
  if (depth < 0.1) return 0;
  if (u < 0 || (int)u >= job.w0 || v < 0 || (int)v >= job.h0) return 0;
  uvd[0] = u;
  uvd[1] = v;
  uvd[2] = depth;
  return 1;
}

__global__ void __launch_bounds__(256) k_retri_uvd(RetriJob job) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < job.cap) {
    DRetriEntry &e = job.ent_new[i];
    if (job.keys_new[i] != kRetriEmpty && e.last_pass >= 0 && e.has_uv0)
      e.uvd_valid = retri_uvd(job, e.pos, e.u0, e.v0, e.uvd);
  }
  if (i < job.nslam) {
    DRetriSlam &sl = job.slam[i];
    if (sl.has_uv0) sl.uvd_valid = retri_uvd(job, sl.pos, sl.u0, sl.v0, sl.uvd);
  }
}

void launch_retriangulate(hipStream_t s, const RetriJob &job) {
  const int nr = std::max(job.cap, job.nslam);
  hipLaunchKernelGGL(k_retri_reset, dim3((nr + 255) / 256), dim3(256), 0, s, job);
  if (job.nobs > 0) {
    if (job.nslam > 8192) throw std::runtime_error("retriangulation: more SLAM landmarks than the LDS id table");
    hipLaunchKernelGGL(k_retri_obs, dim3((job.nobs + 255) / 256), dim3(256),
                       sizeof(unsigned long long) * (size_t)std::max(job.nslam, 1), s, job);
    hipLaunchKernelGGL(k_retri_final, dim3((job.nobs + 255) / 256), dim3(256), 0, s, job);
  }
  hipLaunchKernelGGL(k_retri_uvd, dim3((nr + 255) / 256), dim3(256), 0, s, job);
}

}  // namespace uvhp
