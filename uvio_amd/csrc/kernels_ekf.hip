// StateHelper::EKFUpdate (StateHelper.cpp:116-197) for a direct (uncompressed) batch of r rows, as three
// launches whose products all run on the FP64 matrix cores (v_mfma_f64_16x16x4f64):
//
//   k_ekf_MS   grid:  M = P[:, I] H^T (N x r; one 16-row block per workgroup, the P rows gathered once
//                     into LDS) and, in the same launch, S_up = H P_II H^T + s2 I (one 16-column block of S
//                     per workgroup: T = P_II H_b^T into LDS, then the upper tiles H_a T)
//   k_ekf_fact one workgroup: LDL^T of [S ; r^T] in LDS with the unit-lower inverse alongside (dense_lds.h
//                     ldl_wave) -> L^-1, y = L^-1 r, and StateHelper::initialize's chi2 gate on y
//   k_ekf_WP   grid over the upper 16x16 tile pairs (bi <= bj) of P: W_b = M_b L^-T for both row blocks
//                     (a GEMM with the explicit inverse, recomputed per tile pair instead of a separate
//                     launch), P_ij -= W_bi W_bj^T (written to both triangles), dx = W y on diagonal tiles
//
// The reference computes K = P H^T S^-1 through an LLT solve and P -= K M^T; here P -= (M L^-T)(M L^-T)^T
// and dx = (M L^-T)(L^-1 r): the same update (S = L L^T), every product on MFMA tiles.  The earlier chain
// (k_ekf_M, k_ekf_S, k_ekf_small, k_trinv16, k_trsm_lt, k_ekf_P: six launches, VALU tiles for the four
// products) cost 96 us per update at cfg2 in rocprof (profiles/r01g_cfg2_per_frame.txt).
//
// MFMA operand layout (f64 16x16x4): A (16x4) lane l holds A[l & 15][l >> 4]; B (4x16) lane l holds
// B[l >> 4][l & 15]; C/D register q of lane l is D[(l >> 4) + 4 q][l & 15].
#include <cstdlib>
#include <algorithm>
#include <stdexcept>

#include "dense_lds.h"
#include "kernels.h"

namespace uvhp {

// ---------------------------------------------------------------------------------------------------
// K1: M (blocks 0 .. nbM-1) and S_up (blocks nbM .. nbM + ceil(r/16) - 1; none when Sup is null)
constexpr int kMSThreads = 512;  // 8 waves: one M column tile / one S tile pair per wave at cfg2's r ~ 100
__global__ void __launch_bounds__(kMSThreads) k_ekf_MS(const double *__restrict__ P, int ldp, int N,
                                                const double *__restrict__ H, int ldh, int r, int n,
                                                const int *__restrict__ hidx, double s2, double *__restrict__ M,
                                                double *__restrict__ Sup, int nbM, int *zero,
                                                const double *__restrict__ Tall, int ldt) {
  extern __shared__ double sh[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;  // the update's negative-diagonal count
  if ((int)blockIdx.x < nbM) {
    // M rows i0 .. i0+15: Ps[i][k] = P[i0 + i][hidx[k]] staged once, each wave takes column tiles of M
    const int i0 = blockIdx.x * 16, lds = n | 1;
    double *Ps = sh;
    staged_copy(
        16 * n,
        [&](int e) {
          const int i = e / n, k = e - i * n;
          return (i0 + i < N) ? P[(size_t)(i0 + i) * ldp + hidx[k]] : 0.0;
        },
        [&](int e, double v) {
          const int i = e / n, k = e - i * n;
          Ps[i * lds + k] = v;
        });
    __syncthreads();
    const int nct = (r + 15) / 16;
    for (int t = wid; t < nct; t += kMSThreads / 64) {
      const int j0 = 16 * t, jr = j0 + r16;
      const double *Hr = H + (size_t)min(jr, r - 1) * ldh;
      const bool jv = jr < r;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = tile_chain<16>(
          0, n, kq, [&](int k) { return Ps[r16 * lds + k]; }, [&](int k) { return jv ? Hr[k] : 0.0; }, acc);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = i0 + kq + 4 * q, col = j0 + r16;
        if (row < N && col < r) M[(size_t)row * r + col] = acc[q];
      }
    }
    return;
  }
  if (Tall) {
    // T = H P_II is already in HBM from the batch's chi2 gate (k_gemm_HPg, rejected features' rows zeroed
    // there with their H rows), so S_up[a][b] = H_a T_b^T directly: one upper tile pair (a <= b) per wave,
    // one chain of loads instead of forming T_b first (same products, same ascending k order).
    // ldt < 0: Tall is this update's M = P[:, I] H^T (N x r, launched after the M blocks), whose rows hidx are
    // T^T: T[b][k] = M[hidx[k]][b], the products and k order with which the column blocks below form T.
    const bool gath = ldt < 0;
    int *hs = (int *)sh;
    if (gath) {
      for (int k = threadIdx.x; k < n; k += blockDim.x) hs[k] = hidx[k];
      __syncthreads();
    }
    const int nt = (r + 15) / 16;
    int pair = (blockIdx.x - nbM) * (kMSThreads / 64) + wid, at = 0;
    if (pair >= nt * (nt + 1) / 2) return;
    while (pair >= nt - at) {
      pair -= nt - at;
      at++;
    }
    const int bt = at + pair;
    const int ar = 16 * at + r16, br = 16 * bt + r16;
    const double *Ha = H + (size_t)min(ar, r - 1) * ldh;
    const double *Tb = gath ? Tall + min(br, r - 1) : Tall + (size_t)min(br, r - 1) * ldt;
    const bool av = ar < r, bv = br < r;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = tile_chain<16>(
        0, n, kq, [&](int k) { return av ? Ha[k] : 0.0; },
        [&](int k) { return bv ? (gath ? Tb[(size_t)hs[k] * r] : Tb[k]) : 0.0; }, acc);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = 16 * at + kq + 4 * q, col = 16 * bt + r16;
      if (row < r && col < r) Sup[(size_t)row * r + col] = acc[q] + (row == col ? s2 : 0.0);
    }
    return;
  }
  // S column block b: T = P_II H_b^T (n x 16) into LDS, then S_up[a-tile][b] = H_a T for a <= b
  const int jb = blockIdx.x - nbM, j0 = 16 * jb;
  const int npad = (n + 15) / 16 * 16;
  double *Ts = sh;                                  // npad x 17
  int *hs = (int *)(sh + (size_t)npad * 17);        // hidx
  for (int k = threadIdx.x; k < n; k += blockDim.x) hs[k] = hidx[k];
  __syncthreads();
  {
    const int jr = j0 + r16;
    const double *Hb = H + (size_t)min(jr, r - 1) * ldh;
    const bool jv = jr < r;
    for (int kt = wid; kt < npad / 16; kt += kMSThreads / 64) {
      const int row = 16 * kt + r16;
      const double *Prow = P + (size_t)hs[min(row, n - 1)] * ldp;
      const bool rv = row < n;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = tile_chain<16>(
          0, n, kq, [&](int l) { return rv ? Prow[hs[l]] : 0.0; }, [&](int l) { return jv ? Hb[l] : 0.0; }, acc);
#pragma unroll
      for (int q = 0; q < 4; q++) Ts[(16 * kt + kq + 4 * q) * 17 + r16] = acc[q];
    }
  }
  __syncthreads();
  for (int at = wid; at <= jb; at += kMSThreads / 64) {
    const int ar = 16 * at + r16;
    const double *Ha = H + (size_t)min(ar, r - 1) * ldh;
    const bool av = ar < r;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = tile_chain<16>(
        0, n, kq, [&](int k) { return av ? Ha[k] : 0.0; }, [&](int k) { return Ts[k * 17 + r16]; }, acc);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = 16 * at + kq + 4 * q, col = j0 + r16;
      if (row < r && col < r) Sup[(size_t)row * r + col] = acc[q] + (row == col ? s2 : 0.0);
    }
  }
}

// M = P[:, I] H^T for r <= 4 rows (initialize_invertible's 3 x n block): a GEMV per covariance row, one
// wavefront per row with the lanes over the columns and a butterfly reduction (the 16-row MFMA blocks of
// k_ekf_MS would waste 13 of 16 output columns and serialize their loads per tile)
constexpr int kSmallMRows = 4;
__global__ void __launch_bounds__(256) k_ekf_M_small(const double *__restrict__ P, int ldp, int N,
                                                     const double *__restrict__ H, int ldh, int r, int n,
                                                     const int *__restrict__ hidx, double *__restrict__ M, int *zero) {
  if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const double *Pr = P + (size_t)row * ldp;
  double acc[kSmallMRows] = {0.0, 0.0, 0.0, 0.0};
  for (int k = lane; k < n; k += 64) {
    const double p = Pr[hidx[k]];
#pragma unroll
    for (int b = 0; b < kSmallMRows; b++)
      if (b < r) acc[b] = fma(p, H[(size_t)b * ldh + k], acc[b]);
  }
#pragma unroll
  for (int b = 0; b < kSmallMRows; b++)
    for (int o = 32; o > 0; o >>= 1) acc[b] += __shfl_xor(acc[b], o, 64);
  if (lane < r) {
    double v = acc[0];
#pragma unroll
    for (int b = 1; b < kSmallMRows; b++)
      if (lane == b) v = acc[b];
    M[(size_t)row * r + lane] = v;
  }
}

static size_t ekf_ms_lds_bytes(int n, bool with_S) {
  size_t bm = (size_t)16 * (n | 1) * sizeof(double);
  size_t bs = with_S ? (size_t)(n + 15) / 16 * 16 * 17 * sizeof(double) + (size_t)n * sizeof(int) : 0;
  return bm > bs ? bm : bs;
}

// ---------------------------------------------------------------------------------------------------
// K2: one workgroup.  [S ; r^T] (S from the upper triangle of S_up = selfadjointView<Upper>,
// StateHelper.cpp:160) -> LDL^T with the unit-lower inverse alongside (dense_lds.h ldl_wave), then
// L^-1 = D^-1/2 L_u^-1 (lower, zeros above, ld r) into Linv_out and y = L^-1 r = D^1/2 (D^-1 L_u^-1 r).
// chi2_gate: StateHelper::initialize's test (StateHelper.cpp:458-470) on this factor: chi2 = |y|^2 in a
// fixed order against thr -> *chi2_gate (the P-update gate) and [chi2, accepted] into gate_out[0..1].
// LDS: the factor in LDS (a compile-time choice, so every access of the factorization is a DS instruction;
// a runtime choice makes them all FLAT)
// W: the panel waves of ldl_wave_inv (panel rows 16 + 48 W); one workgroup of kFactThreads.
template <int W, bool LDS>
__global__ void __launch_bounds__(kFactThreads) k_ekf_fact(const double *__restrict__ Sup, int r,
                                                  const double *__restrict__ res, int res_stride,
                                                  double *__restrict__ Linv_out, double *__restrict__ y_out, double *Sg,
                                                  int use_lds, int *chi2_gate, double chi2_thr,
                                                  double *__restrict__ gate_out) {
  extern __shared__ double lds[];
  double *A = LDS ? lds : Sg;
  (void)use_lds;
  const int ld = r | 1;  // odd row stride: conflict-free 64-bit LDS reads down a column
  double *Dd = A + (size_t)(r + 1) * ld, *sd = Dd + r;
  staged_copy(
      r * r + r,
      [&](int e) {
        if (e >= r * r) return res[(size_t)(e - r * r) * res_stride];
        const int a = e / r, b = e - a * r;
        return (b <= a) ? Sup[(size_t)b * r + a] : 0.0;
      },
      [&](int e, double v) {
        if (e >= r * r) {
          A[(size_t)r * ld + e - r * r] = v;
        } else {
          const int a = e / r, b = e - a * r;
          if (b <= a) A[(size_t)a * ld + b] = v;
        }
      });
  __syncthreads();
  ldl_wave_inv<1, SqLayout, W>(A, SqLayout{ld}, r, r + 1, Dd, true);
  for (int k = threadIdx.x; k < r; k += blockDim.x) {
    const double q = sqrt(Dd[k]);
    sd[k] = q;
    y_out[k] = A[(size_t)r * ld + k] * q;
  }
  __syncthreads();
  if (chi2_gate && threadIdx.x < 64) {
    double s = 0.0;
    for (int k = threadIdx.x; k < r; k += 64) {
      const double v = A[(size_t)r * ld + k] * sd[k];
      s += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (threadIdx.x == 0) {
      // the incoming gate (the feature's linearization succeeded) AND the test
      const int acc = (*chi2_gate != 0) && !(s > chi2_thr);
      *chi2_gate = acc;
      gate_out[0] = s;
      gate_out[1] = acc;
    }
  }
  for (int e = threadIdx.x; e < r * r; e += blockDim.x) {
    const int a = e / r, b = e - a * r;
    double v = 0.0;
    if (b < a)
      v = A[(size_t)b * ld + a] / sd[a];
    else if (b == a)
      v = 1.0 / sd[a];
    Linv_out[e] = v;
  }
}
size_t ekf_small_lds_bytes(int r) { return (dense_lds_bytes(r + 1, r) + (size_t)2 * r * sizeof(double)); }

// ---------------------------------------------------------------------------------------------------
// K3: tile pair (bi, bj), bi <= bj, of the nb x nb tile grid of P (blocks enumerated row by row)
__global__ void __launch_bounds__(256) k_ekf_WP(double *__restrict__ P, int ldp, int N, const double *__restrict__ M,
                                                int r, const double *__restrict__ Linv, const double *__restrict__ y,
                                                double *__restrict__ dx, int *neg, const int *gate, int nb) {
  if (gate && *gate == 0) return;  // no accepted rows: the reference makes no update
  extern __shared__ double sh[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  int b = blockIdx.x, bi = 0;
  while (b >= nb - bi) {
    b -= nb - bi;
    bi++;
  }
  const int bj = bi + b;
  const int ldw = r | 1;
  double *Wi = sh, *Wj = sh + 16 * ldw, *red = sh + 32 * ldw;
  // this thread's P element, fetched before the products so its latency is hidden
  const int ei = threadIdx.x >> 4, ej = threadIdx.x & 15;
  const int gi = 16 * bi + ei, gj = 16 * bj + ej;
  const bool pw = gi < N && gj < N && (bi < bj || ej >= ei);
  const double pv = pw ? P[(size_t)gi * ldp + gj] : 0.0;
  // W_b[i][c] = sum_{k <= c} M[16 b + i][k] Linv[c][k]
  const int nct = (r + 15) / 16, ntask = (bi == bj ? 1 : 2) * nct;
  for (int t = wid; t < ntask; t += 4) {
    const int which = t / nct, ct = t - which * nct;
    double *Wd = which ? Wj : Wi;
    const int row = 16 * (which ? bj : bi) + r16, c = 16 * ct + r16;
    const double *Mr = M + (size_t)min(row, N - 1) * r;
    const double *Lr = Linv + (size_t)min(c, r - 1) * r;
    const bool rv = row < N, cv = c < r;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = tile_chain(
        0, min(16 * ct + 16, r), kq, [&](int k) { return rv ? Mr[k] : 0.0; }, [&](int k) { return cv ? Lr[k] : 0.0; },
        acc);
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (cv) Wd[(kq + 4 * q) * ldw + c] = acc[q];
  }
  __syncthreads();
  const double *Wb = (bi == bj) ? Wi : Wj;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 4 * wid; k0 < r; k0 += 16) {  // wave w: k-slabs w, w + 4, ...
    const int k = k0 + kq;
    const double a = (k < r) ? Wi[r16 * ldw + k] : 0.0;
    const double bb = (k < r) ? Wb[r16 * ldw + k] : 0.0;
    acc = mfma4(a, bb, acc);
  }
#pragma unroll
  for (int q = 0; q < 4; q++) red[wid * 256 + (kq + 4 * q) * 16 + r16] = acc[q];
  __syncthreads();
  if (pw) {
    const int e = threadIdx.x;
    const double s = (red[e] + red[256 + e]) + (red[512 + e] + red[768 + e]);
    const double v = pv - s;
    P[(size_t)gi * ldp + gj] = v;
    P[(size_t)gj * ldp + gi] = v;
    if (gi == gj && v < 0.0) atomicAdd(neg, 1);
  }
  if (bi == bj && wid == 1) {
    const int i = lane >> 2, part = lane & 3;
    double a = 0.0;
    for (int k = part; k < r; k += 4) a += Wi[i * ldw + k] * y[k];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (part == 0 && 16 * bi + i < N) dx[16 * bi + i] = a;
  }
}

// Thread t of one workgroup moves clone t (t < ncl) or camera t - ncl by dx: Var::update (PoseJPL: quat_boxplus,
// p += dp; intrinsics +=) and the tables' rotation matrices (quat_2_Rot), the host's formulas
__device__ void chain_tables_apply(int t, const double *__restrict__ dx, DClone *__restrict__ clones,
                                   DPoseVal *__restrict__ cv, int ncl, DCam *__restrict__ cams,
                                   DPoseVal *__restrict__ camv, int ncam, int calib_ext, int calib_intr) {
  if (t < ncl) {  // PoseJPL::update of clone t, then the table's R_GtoI / p_IinG
    DPoseVal &v = cv[t];
    const double *d = dx + v.pid;
    quat_boxplus(v.q, d);
    for (int k = 0; k < 3; k++) v.p[k] += d[3 + k];
    quat_2_Rot(v.q, clones[t].R);
    for (int k = 0; k < 3; k++) clones[t].p[k] = v.p[k];
  } else if (t < ncl + ncam) {
    const int c = t - ncl;
    DCam &dc = cams[c];
    if (calib_ext && dc.pid_ext >= 0) {
      DPoseVal &v = camv[c];
      const double *d = dx + v.pid;
      quat_boxplus(v.q, d);
      for (int k = 0; k < 3; k++) v.p[k] += d[3 + k];
      quat_2_Rot(v.q, dc.R_ItoC);
      for (int k = 0; k < 3; k++) dc.p_IinC[k] = v.p[k];
    }
    if (calib_intr && dc.pid_intr >= 0)
      for (int k = 0; k < 8; k++) dc.cam.v[k] += dx[dc.pid_intr + k];
  }
}

// Delayed-initialization chain step (kernels.h launch_chain_apply).  Block 0 updates the tables (one thread
// per clone / camera) when the candidate was accepted; every block clears a rejected candidate's slot.
__global__ void __launch_bounds__(256) k_chain_apply(const DFeatOut *__restrict__ fout, const int *__restrict__ gate,
                                                     const int *__restrict__ neg, const double *__restrict__ dx,
                                                     DClone *__restrict__ clones, DPoseVal *__restrict__ cv, int ncl,
                                                     DCam *__restrict__ cams, DPoseVal *__restrict__ camv, int ncam,
                                                     int calib_ext, int calib_intr, double *__restrict__ xv, int Nx,
                                                     double *__restrict__ P, int ldp, int Ntot, int slot,
                                                     double *__restrict__ out) {
  const bool acc = (!fout || fout->status == 0) && (!gate || *gate != 0);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (!acc) {
    if (slot >= 0)
      for (int e = t; e < 3 * Ntot; e += gridDim.x * blockDim.x) {
        const int i = e / 3, a = e - 3 * i;
        P[(size_t)(slot + a) * ldp + i] = 0.0;
        P[(size_t)i * ldp + slot + a] = 0.0;
      }
  } else if (dx && xv) {  // the additive mirror (landmarks): Var::update of a vector, val += dx
    for (int e = t; e < Nx; e += gridDim.x * blockDim.x) xv[e] += dx[e];
  }
  if (acc && blockIdx.x == 0 && dx) chain_tables_apply(t, dx, clones, cv, ncl, cams, camv, ncam, calib_ext, calib_intr);
  if (t == 0) {
    out[0] = acc ? 1.0 : 0.0;
    out[1] = neg ? (double)*neg : 0.0;
  }
}

void launch_chain_apply(hipStream_t s, const DFeatOut *fout, const int *gate, const int *neg, const double *dx,
                        DClone *clones, DPoseVal *cv, int ncl, DCam *cams, DPoseVal *camv, int ncam, int calib_ext,
                        int calib_intr, double *xv, int Nx, double *P, int ldp, int Ntot, int slot, double *out) {
  if (ncl + ncam > 256) throw std::runtime_error("update chain: more clones + cameras than one workgroup");
  const int nb = std::max(1, std::min(16, (std::max(3 * Ntot, Nx) + 255) / 256));
  hipLaunchKernelGGL(k_chain_apply, dim3(nb), dim3(256), 0, s, fout, gate, neg, dx, clones, cv, ncl, cams, camv, ncam,
                     calib_ext, calib_intr, xv, Nx, P, ldp, Ntot, slot, out);
}

// ---------------------------------------------------------------------------------------------------
// Chained UWB ranges (kernels.h DUwbState)
__global__ void k_uwb_row(DUwbState *st, int j, const double *__restrict__ prev, double *__restrict__ h,
                          double *__restrict__ region) {
  if (threadIdx.x != 0) return;
  DUwbState &u = *st;
  // a negative covariance diagonal in an earlier range of the message halts the rest of it: the reference stops
  // at that update (StateHelper.cpp:181, std::exit), so no later range may touch P (the host then reports E_NUMERIC)
  const int *pi = reinterpret_cast<const int *>(prev + 1);
  const bool halt = prev && (pi[0] > 0 || pi[1] != 0);
  if (prev && prev[0] != 0.0 && !halt) {
    // Var::update of the previous range's dx (engine_state.cpp): IMU quaternion boxplus + position, p_IinU and
    // the anchors additive
    const double *dx = prev + 4;
    quat_boxplus(u.q, dx + u.id_imu);
    for (int k = 0; k < 3; k++) u.p[k] += dx[u.id_imu + 3 + k];
    if (u.id_cal >= 0)
      for (int k = 0; k < 3; k++) u.pU[k] += dx[u.id_cal + k];
    for (int a = 0; a < u.nr; a++)
      if (u.id_anc[a] >= 0)
        for (int k = 0; k < 5; k++) u.anc[a][k] += dx[u.id_anc[a] + k];
  }
  uwb_row(u.q, u.p, u.pU, u.anc[j], u.id_cal >= 0, u.id_anc[j] >= 0, u.range[j], h);
  region[0] = 0.0;
  region[1] = 0.0;  // the negative-diagonal count (int bits, low word) and the halt flag (high word)
  if (halt) reinterpret_cast<int *>(region + 1)[1] = 1;
  region[2] = region[3] = 0.0;
}

void launch_uwb_row(hipStream_t s, DUwbState *st, int j, const double *prev, double *h, double *region) {
  hipLaunchKernelGGL(k_uwb_row, dim3(1), dim3(64), 0, s, st, j, prev, h, region);
}

__global__ void __launch_bounds__(256) k_uwb_M(const double *__restrict__ P, int ldp, int N, const double *__restrict__ h,
                                               const int *__restrict__ hidx, int n, double *__restrict__ M) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const double *Pr = P + (size_t)i * ldp;
  double a = 0.0;
  for (int k = 0; k < n; k++) a = fma(Pr[hidx[k]], h[k], a);
  M[i] = a;
}

void launch_uwb_M(hipStream_t s, const double *P, int ldp, int N, const double *h, const int *hidx, int n, double *M) {
  hipLaunchKernelGGL(k_uwb_M, dim3((N + 255) / 256), dim3(256), 0, s, P, ldp, N, h, hidx, n, M);
}

// tile pair (bi, bj), bi <= bj, of the 16 x 16 tiles of P, one element per thread
__global__ void __launch_bounds__(256) k_uwb_update(double *__restrict__ P, int ldp, int N, const double *__restrict__ M,
                                                    const double *__restrict__ h, const int *__restrict__ hidx, int n,
                                                    double s2, double thr, double *__restrict__ region, int nb) {
  if (reinterpret_cast<const int *>(region + 1)[1] != 0) return;  // halted (k_uwb_row): not applied, region[0] = 0
  // the innovation variance and the gate, the same arithmetic in every block
  double S = 0.0;
  for (int k = 0; k < n; k++) S = fma(h[k], M[hidx[k]], S);
  S += s2;
  const double res = h[n];
  const double chi2 = res * res / S;
  const bool acc = !(chi2 > thr);  // UpdaterUWB.cpp:73-79: rejected when chi2 > multiplier * chi2_0.95(1)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    region[0] = acc ? 1.0 : 0.0;
    region[2] = chi2;
    region[3] = S;
  }
  if (!acc) return;
  int b = blockIdx.x, bi = 0;
  while (b >= nb - bi) {
    b -= nb - bi;
    bi++;
  }
  const int bj = bi + b;
  const int ei = threadIdx.x >> 4, ej = threadIdx.x & 15;
  const int gi = 16 * bi + ei, gj = 16 * bj + ej;
  const double rs = 1.0 / sqrt(S);
  if (gi < N && gj < N && (bi < bj || ej >= ei)) {
    const double v = P[(size_t)gi * ldp + gj] - (M[gi] * rs) * (M[gj] * rs);
    P[(size_t)gi * ldp + gj] = v;
    P[(size_t)gj * ldp + gi] = v;
    if (gi == gj && v < 0.0) atomicAdd(reinterpret_cast<int *>(region + 1), 1);
  }
  if (bi == bj && ei == 0 && gj < N) region[4 + gj] = (M[gj] * rs) * (res * rs);
}

void launch_uwb_update(hipStream_t s, double *P, int ldp, int N, const double *M, const double *h, const int *hidx,
                       int n, double s2, double thr, double *region) {
  const int nb = (N + 15) / 16;
  hipLaunchKernelGGL(k_uwb_update, dim3(nb * (nb + 1) / 2), dim3(256), 0, s, P, ldp, N, M, h, hidx, n, s2, thr, region,
                     nb);
}

static void ensure_ekf_lds_attrs() {
  static bool done = false;
  if (done) return;
  const void *fns[7] = {(const void *)k_ekf_MS,            (const void *)k_ekf_WP,
                        (const void *)k_ekf_fact<1, true>, (const void *)k_ekf_fact<2, true>,
                        (const void *)k_ekf_fact<3, true>, (const void *)k_ekf_fact<4, true>,
                        (const void *)k_ekf_fact<5, true>};
  for (int k = 0; k < 7; k++)
    if (set_dyn_lds(fns[k], kMaxDynLds) < kMaxDynLds)
      throw std::runtime_error("dynamic LDS limit not granted for an EKF kernel (" + std::to_string(k) + ")");
  done = true;
}

void launch_ekf_M(hipStream_t s, const double *P, int ldp, int N, const double *H, int ldh, int r, int n,
                  const int *hidx, double *M, int *zero) {
  if (r <= kSmallMRows) {
    hipLaunchKernelGGL(k_ekf_M_small, dim3((N + 3) / 4), dim3(256), 0, s, P, ldp, N, H, ldh, r, n, hidx, M, zero);
    return;
  }
  ensure_ekf_lds_attrs();
  const size_t lds = ekf_ms_lds_bytes(n, false);
  if (lds > (size_t)kMaxDynLds) throw std::runtime_error("EKF update with too many columns for k_ekf_MS");
  const int nbM = (N + 15) / 16;
  hipLaunchKernelGGL(k_ekf_MS, dim3(nbM), dim3(kMSThreads), lds, s, P, ldp, N, H, ldh, r, n, hidx, 0.0, M,
                     (double *)nullptr, nbM, zero, (const double *)nullptr, 0);
}

void launch_ekf_phaseA(hipStream_t s, const double *P, int ldp, int N, const double *H, int ldh, int r, int n,
                       const int *hidx, double sigma2, EkfScratch &sc) {
  ensure_ekf_lds_attrs();
  const size_t lds = ekf_ms_lds_bytes(n, true);
  if (lds > (size_t)kMaxDynLds) throw std::runtime_error("EKF update with too many columns for k_ekf_MS");
  const int nbM = (N + 15) / 16, nt = (r + 15) / 16;
  const int wpb = kMSThreads / 64;
  const double *Tall = sc.Tall;
  const int nbS = Tall ? (nt * (nt + 1) / 2 + wpb - 1) / wpb : nt;  // tile pairs, a wave each / column blocks
  double *Sup = sc.S + 2 * (size_t)r * r;
  // No T from a chi2 gate (the delayed initialization's update): S from this update's own M in a second
  // launch (rows hidx of M are T^T) instead of each S column block forming T from P (r04v: 26 us per launch in
  // the cfg3 frame).  UVIO_HP_MS_FROM_P=1: the one-launch form (A/B).
  static const bool from_p = std::getenv("UVIO_HP_MS_FROM_P") != nullptr;
  if (!Tall && !from_p) {
    const int nbG = (nt * (nt + 1) / 2 + wpb - 1) / wpb;
    hipLaunchKernelGGL(k_ekf_MS, dim3(nbM), dim3(kMSThreads), lds, s, P, ldp, N, H, ldh, r, n, hidx, sigma2, sc.M, Sup,
                       nbM, sc.neg, (const double *)nullptr, 0);
    hipLaunchKernelGGL(k_ekf_MS, dim3(nbG), dim3(kMSThreads), lds, s, P, ldp, N, H, ldh, r, n, hidx, sigma2, sc.M, Sup,
                       0, (int *)nullptr, (const double *)sc.M, -1);
    return;
  }
  static const bool split = std::getenv("UVIO_HP_MS_SPLIT") != nullptr;  // diagnostic: M, then S, as two launches
  if (split) {
    hipLaunchKernelGGL(k_ekf_MS, dim3(nbM), dim3(kMSThreads), lds, s, P, ldp, N, H, ldh, r, n, hidx, sigma2, sc.M, Sup,
                       nbM, sc.neg, Tall, sc.ldt);
    hipLaunchKernelGGL(k_ekf_MS, dim3(nbS), dim3(kMSThreads), lds, s, P, ldp, N, H, ldh, r, n, hidx, sigma2, sc.M, Sup,
                       0, (int *)nullptr, Tall, sc.ldt);
    return;
  }
  hipLaunchKernelGGL(k_ekf_MS, dim3(nbM + nbS), dim3(kMSThreads), lds, s, P, ldp, N, H, ldh, r, n, hidx, sigma2, sc.M, Sup,
                     nbM, sc.neg, Tall, sc.ldt);
}

static void launch_ekf_factor(hipStream_t s, int N, int r, const double *res, int res_stride, EkfScratch &sc) {
  ensure_ekf_lds_attrs();
  if (r + 1 > kWaveMaxRows) throw std::runtime_error("direct EKF update with more rows than the factorization panel");
  const size_t bytes = ekf_small_lds_bytes(r);
  const int use_lds = bytes <= (size_t)kMaxDynLds;
  double *Linv = sc.S;
  double *Sup = sc.S + 2 * (size_t)r * r;
  double *Sg = sc.S + 3 * (size_t)r * r;  // (r+1)(r|1) + 2r <= 2 r^2 doubles once r >= 40 (else LDS)
  {
    KScope ks(sc.kp, KC_LDL);
    const int w = panel_waves(r + 1);
    auto *kf = use_lds ? (w == 1 ? k_ekf_fact<1, true> : w == 2 ? k_ekf_fact<2, true> : w == 3 ? k_ekf_fact<3, true>
                          : w == 4 ? k_ekf_fact<4, true> : k_ekf_fact<5, true>)
                       : (w == 1 ? k_ekf_fact<1, false> : w == 2 ? k_ekf_fact<2, false> : w == 3 ? k_ekf_fact<3, false>
                          : w == 4 ? k_ekf_fact<4, false> : k_ekf_fact<5, false>);
    hipLaunchKernelGGL(kf, dim3(1), dim3(kFactThreads), use_lds ? bytes : 0, s, Sup, r, res, res_stride, Linv, sc.y, Sg,
                       use_lds, sc.chi2_gate, sc.chi2_thr, sc.dx + N);
  }
  // LDL^T of the r x r innovation covariance with the residual as an extra row: r^3/3 + r^2 FLOPs; the
  // lower triangle and the residual read, the factor written
  if (sc.kp) sc.kp->credit(KC_LDL, (double)r * r * r / 3.0 + (double)r * r, 8.0 * (1.5 * r * r + 2.0 * r));
  if (sc.chi2_gate) sc.gate = sc.chi2_gate;
}

void launch_ekf_phaseB(hipStream_t s, double *P, int ldp, int N, int r, const double *res, int res_stride,
                       EkfScratch &sc) {
  launch_ekf_factor(s, N, r, res, res_stride, sc);
  const int nb = (N + 15) / 16;
  const size_t lw = (size_t)(32 * (r | 1) + 1024) * sizeof(double);
  hipLaunchKernelGGL(k_ekf_WP, dim3(nb * (nb + 1) / 2), dim3(256), lw, s, P, ldp, N, sc.M, r, sc.S, sc.y, sc.dx,
                     sc.neg, sc.gate, nb);
}

// ---------------------------------------------------------------------------------------------------
// One delayed-initialization candidate (StateHelper::initialize, StateHelper.cpp:393-577: initialize_invertible
// of the landmark's 3 rows, then EKFUpdate of the other nup rows at the same factor that carries the chi2 test)
// in six launches instead of eight (k_ekf_M_small, k_init_invertible, 2 x k_ekf_MS, k_ekf_fact, k_ekf_WP,
// k_chain_apply):
//   k_di_M    grid over the old state's 16-row blocks (rows < Ni): P[i, I] staged once; M_up = P[:, I] H_up^T on
//             k_ekf_MS's tiles and M3 = P[:, I] H_init^T in k_ekf_M_small's GEMV order
//   k_di_S    S_up from M_up's rows I (k_ekf_MS's gathered tile pairs); initialize_invertible (k_init_invertible's
//             blocks: the landmark's cross-covariance columns and 3x3 block); the landmark's rows of M_up, from
//             the same values k_init_invertible writes, on the tiles k_ekf_MS formed from P's new rows
//   k_ekf_fact, k_ekf_WP, k_chain_apply unchanged
// Every value is formed by the same expression, in the same order, as in the eight-launch chain (the old chain
// stays behind UVIO_HP_DI_UNFUSED=1 for A/B runs; the 40-frame state digests of cfg3 and cfg3t are equal).
// Measured and dropped: k_chain_apply folded into k_ekf_WP (the last workgroup to finish, after agent-scope
// release / acquire fences around a completion counter, moving the tables): 22.8 us against 10.7 + 4.7 us.
__global__ void __launch_bounds__(kMSThreads) k_di_M(const double *__restrict__ P, int ldp, int Ni,
                                              const double *__restrict__ H, int ldh, int nup, int n,
                                              const int *__restrict__ hidx, double *__restrict__ M,
                                              double *__restrict__ M3, int *neg) {
  extern __shared__ double sh[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  if (blockIdx.x == 0 && threadIdx.x == 0) *neg = 0;  // the update's negative-diagonal count
  const int i0 = blockIdx.x * 16, lds = n | 1;
  double *Ps = sh;
  staged_copy(
      16 * n,
      [&](int e) {
        const int i = e / n, k = e - i * n;
        return (i0 + i < Ni) ? P[(size_t)(i0 + i) * ldp + hidx[k]] : 0.0;
      },
      [&](int e, double v) {
        const int i = e / n, k = e - i * n;
        Ps[i * lds + k] = v;
      });
  __syncthreads();
  const double *Hup = H + 3 * (size_t)ldh;
  const int nct = (nup + 15) / 16;
  for (int t = wid; t < nct; t += kMSThreads / 64) {
    const int j0 = 16 * t, jr = j0 + r16;
    const double *Hr = Hup + (size_t)min(jr, nup - 1) * ldh;
    const bool jv = jr < nup;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = tile_chain<16>(
        0, n, kq, [&](int k) { return Ps[r16 * lds + k]; }, [&](int k) { return jv ? Hr[k] : 0.0; }, acc);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = i0 + kq + 4 * q, col = j0 + r16;
      if (row < Ni && col < nup) M[(size_t)row * nup + col] = acc[q];
    }
  }
  // M3: one wavefront per row, lanes over the columns, butterfly sum (k_ekf_M_small)
  for (int i = wid; i < 16 && i0 + i < Ni; i += kMSThreads / 64) {
    double acc[kSmallMRows] = {0.0, 0.0, 0.0, 0.0};
    for (int k = lane; k < n; k += 64) {
      const double p = Ps[i * lds + k];
#pragma unroll
      for (int b = 0; b < 3; b++) acc[b] = fma(p, H[(size_t)b * ldh + k], acc[b]);
    }
#pragma unroll
    for (int b = 0; b < kSmallMRows; b++)
      for (int o = 32; o > 0; o >>= 1) acc[b] += __shfl_xor(acc[b], o, 64);
    if (lane < 3) {
      double v = acc[0];
#pragma unroll
      for (int b = 1; b < kSmallMRows; b++)
        if (lane == b) v = acc[b];
      M3[(size_t)(i0 + i) * 3 + lane] = v;
    }
  }
}

constexpr int kDiInitThreads = 512;  // k_di_S's initialize_invertible blocks: (3 Ni + 511) / 512 of them
__global__ void __launch_bounds__(kMSThreads) k_di_S(double *__restrict__ P, int ldp, int Ni,
                                              const double *__restrict__ H, int ldh, int nup, int n,
                                              const int *__restrict__ hidx, double s2, double *__restrict__ M,
                                              const double *__restrict__ M3, double *__restrict__ Sup,
                                              const DFeatOut *__restrict__ fout, const int *__restrict__ gate,
                                              double *__restrict__ resout, int nbG, int nbX) {
  extern __shared__ double sh[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const double *Hup = H + 3 * (size_t)ldh;
  const int b = blockIdx.x;
  if (b < nbG) {
    // S_up[a][b] = H_a T_b^T with T[b][k] = M[hidx[k]][b] (k_ekf_MS, ldt < 0)
    int *hs = (int *)sh;
    for (int k = threadIdx.x; k < n; k += blockDim.x) hs[k] = hidx[k];
    __syncthreads();
    const int nt = (nup + 15) / 16;
    int pair = b * (kMSThreads / 64) + wid, at = 0;
    if (pair >= nt * (nt + 1) / 2) return;
    while (pair >= nt - at) {
      pair -= nt - at;
      at++;
    }
    const int bt = at + pair;
    const int ar = 16 * at + r16, br = 16 * bt + r16;
    const double *Ha = Hup + (size_t)min(ar, nup - 1) * ldh;
    const double *Tb = M + min(br, nup - 1);
    const bool av = ar < nup, bv = br < nup;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = tile_chain<16>(
        0, n, kq, [&](int k) { return av ? Ha[k] : 0.0; }, [&](int k) { return bv ? Tb[(size_t)hs[k] * nup] : 0.0; },
        acc);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = 16 * at + kq + 4 * q, col = 16 * bt + r16;
      if (row < nup && col < nup) Sup[(size_t)row * nup + col] = acc[q] + (row == col ? s2 : 0.0);
    }
    return;
  }
  __shared__ double Hinv[9], S3[9], PLL[9];
  if (b < nbG + nbX) {
    // initialize_invertible (k_init_invertible with N = Ni: block xb takes the cross-covariance elements
    // xb * 512 ..; the first one also the 3x3 block)
    const int xb = b - nbG, t = threadIdx.x + xb * kDiInitThreads;
    if (resout && xb == 0 && threadIdx.x < 3) resout[threadIdx.x] = H[(size_t)threadIdx.x * ldh + n];
    if (gate && *gate == 0) return;
    if (threadIdx.x == 0) inv3_cofactor(fout->HfR, Hinv);
    __syncthreads();
    if (xb == 0) {
      __shared__ double part[9][28];
      const int e = threadIdx.x / 28, j = threadIdx.x % 28;
      if (e < 9) {
        const int a = e / 3, bb = e % 3;
        double acc = 0.0;
        for (int k = j; k < n; k += 28) acc += H[(size_t)a * ldh + k] * M3[(size_t)hidx[k] * 3 + bb];
        part[e][j] = acc;
      }
      __syncthreads();
      if (threadIdx.x < 9) {
        const int a = threadIdx.x / 3, bb = threadIdx.x % 3;
        double acc = 0.0;
        for (int q = 0; q < 28; q++) acc += part[threadIdx.x][q];
        S3[threadIdx.x] = acc + (a == bb ? s2 : 0.0);
      }
      __syncthreads();
      if (threadIdx.x < 9) {
        const int a = threadIdx.x / 3, bb = threadIdx.x % 3;
        double acc = 0.0;
        for (int c = 0; c < 3; c++)
          for (int e2 = 0; e2 < 3; e2++) {
            const double sce = (c <= e2) ? S3[c * 3 + e2] : S3[e2 * 3 + c];
            acc += Hinv[a * 3 + c] * sce * Hinv[bb * 3 + e2];
          }
        PLL[threadIdx.x] = acc;
      }
    }
    if (t < Ni * 3) {
      const int i = t / 3, a = t % 3;
      double acc = 0.0;
      for (int bb = 0; bb < 3; bb++) acc += M3[(size_t)i * 3 + bb] * Hinv[a * 3 + bb];
      P[(size_t)i * ldp + Ni + a] = -acc;
      P[(size_t)(Ni + a) * ldp + i] = -acc;
    }
    if (xb == 0 && threadIdx.x < 9) {
      const int a = threadIdx.x / 3, bb = threadIdx.x % 3;
      P[(size_t)(Ni + a) * ldp + Ni + bb] = PLL[threadIdx.x];
    }
    return;
  }
  // the landmark's rows Ni .. Ni+2 of M_up: P[Ni + a][hidx[k]] as initialize_invertible writes it, then the
  // 16-row tiles of k_ekf_MS (only these three rows of the tile are stored)
  if (gate && *gate == 0) return;
  double *Pl = sh;  // 3 x n
  if (threadIdx.x == 0) inv3_cofactor(fout->HfR, Hinv);
  __syncthreads();
  for (int e = threadIdx.x; e < 3 * n; e += blockDim.x) {
    const int a = e / n, k = e - a * n, i = hidx[k];
    double acc = 0.0;
    for (int bb = 0; bb < 3; bb++) acc += M3[(size_t)i * 3 + bb] * Hinv[a * 3 + bb];
    Pl[e] = -acc;
  }
  __syncthreads();
  const int nct = (nup + 15) / 16;
  for (int t = wid; t < nct; t += kMSThreads / 64) {
    const int j0 = 16 * t, jr = j0 + r16;
    const double *Hr = Hup + (size_t)min(jr, nup - 1) * ldh;
    const bool jv = jr < nup, rv = r16 < 3;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = tile_chain<16>(
        0, n, kq, [&](int k) { return rv ? Pl[r16 * n + k] : 0.0; }, [&](int k) { return jv ? Hr[k] : 0.0; }, acc);
    const int col = j0 + r16;
    if (kq < 3 && col < nup) M[(size_t)(Ni + kq) * nup + col] = acc[0];
  }
}

void launch_di_candidate(hipStream_t s, double *P, int ldp, int Ni, const double *Hrow, int ldh, int nup, int n,
                         const int *hidx, double s2, EkfScratch &sc, const DFeatOut *fout, double *resout,
                         DClone *clones, DPoseVal *cv, int ncl, DCam *cams, DPoseVal *camv, int ncam, int calib_ext,
                         int calib_intr, double *out) {
  if (nup <= 0 || nup + 1 > kWaveMaxRows) throw std::runtime_error("delayed-init candidate rows outside 1..255");
  if (ncl + ncam > 256) throw std::runtime_error("update chain: more clones + cameras than one workgroup");
  if (!sc.M3 || !sc.chi2_gate) throw std::runtime_error("delayed-init candidate: scratch not set up");
  ensure_ekf_lds_attrs();
  static bool attrs = false;
  if (!attrs) {
    if (set_dyn_lds((const void *)k_di_M, kMaxDynLds) < kMaxDynLds ||
        set_dyn_lds((const void *)k_di_S, kMaxDynLds) < kMaxDynLds)
      throw std::runtime_error("dynamic LDS limit not granted for a delayed-init kernel");
    attrs = true;
  }
  const size_t ldsM = (size_t)16 * (n | 1) * sizeof(double);
  const size_t ldsS = std::max((size_t)n * sizeof(int), (size_t)3 * n * sizeof(double));
  if (ldsM > (size_t)kMaxDynLds || ldsS > (size_t)kMaxDynLds)
    throw std::runtime_error("delayed-init candidate with too many columns");
  const int N = Ni + 3;
  {
    hipLaunchKernelGGL(k_di_M, dim3((Ni + 15) / 16), dim3(kMSThreads), ldsM, s, P, ldp, Ni, Hrow, ldh, nup, n, hidx,
                       sc.M, sc.M3, sc.neg);
    const int nt = (nup + 15) / 16, wpb = kMSThreads / 64;
    const int nbG = (nt * (nt + 1) / 2 + wpb - 1) / wpb, nbX = (3 * Ni + kDiInitThreads - 1) / kDiInitThreads;
    double *Sup = sc.S + 2 * (size_t)nup * nup;
    hipLaunchKernelGGL(k_di_S, dim3(nbG + nbX + 1), dim3(kMSThreads), ldsS, s, P, ldp, Ni, Hrow, ldh, nup, n, hidx,
                       s2, sc.M, sc.M3, Sup, fout, sc.chi2_gate, resout, nbG, nbX);
    launch_ekf_factor(s, N, nup, Hrow + 3 * (size_t)ldh + n, ldh, sc);
    const int nb = (N + 15) / 16;
    const size_t lw = (size_t)(32 * (nup | 1) + 1024) * sizeof(double);
    hipLaunchKernelGGL(k_ekf_WP, dim3(nb * (nb + 1) / 2), dim3(256), lw, s, P, ldp, N, sc.M, nup, sc.S, sc.y, sc.dx,
                       sc.neg, sc.chi2_gate, nb);
  }
  launch_chain_apply(s, fout, sc.chi2_gate, sc.neg, sc.dx, clones, cv, ncl, cams, camv, ncam, calib_ext, calib_intr,
                     nullptr, 0, P, ldp, N, Ni, out);
}

void launch_ekf_update(hipStream_t s, double *P, int ldp, int N, const double *H, int ldh, int r, int n,
                       const int *hidx, const double *res, int res_stride, double sigma2, EkfScratch &sc) {
  launch_ekf_phaseA(s, P, ldp, N, H, ldh, r, n, hidx, sigma2, sc);
  launch_ekf_phaseB(s, P, ldp, N, r, res, res_stride, sc);
}

}  // namespace uvhp
