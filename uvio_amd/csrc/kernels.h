// Device data layouts and launch wrappers for the gfx950 kernels (kernels_*.hip).
//
// The covariance P is a dense row-major FP64 matrix resident in HBM for the whole run with a fixed
// leading dimension `ld` (capacity computed from the config, DESIGN.md "Data layout"); the active
// block is N x N in the top-left corner.  Variable ids are host-mirrored exactly like
// ov_type::Type::_id (State.cpp:28-166, StateHelper.cpp:271-391).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hp_math.h"
#include "kprof.h"

namespace uvhp {

constexpr int kMaxMeasPerFeat = 64;  // m_f <= 64 (one lane per measurement in the geometry wave)
constexpr int kMaxVarsPerFeat = 48;  // clones + per-cam calib blocks of one feature
constexpr int kMaxCams = 4;

// One clone slot (time order, State::_clones_IMU map order)
struct DClone {
  double R[9], p[3];    // R_GtoI, p_IinG (current)
  double Rf[9], pf[3];  // first estimates
  int pid;              // covariance id of the clone PoseJPL
  int canon;            // canonical H column of the clone block
  int pad[2];
};

// One camera: extrinsic (R_ItoC, p_IinC), intrinsics, covariance ids / canonical columns
struct DCam {
  double R_ItoC[9], p_IinC[3];
  CamParams cam;
  int pid_ext, pid_intr;      // -1 if not calibrated
  int canon_ext, canon_intr;  // -1 if not calibrated
};

// One measurement of a feature (uv in raw pixels, uvn normalized; float as in ov_core::Feature)
struct DMeas {
  float u, v, un, vn;
  int cam, slot;      // camera id, clone slot
  int lc_clone;       // local column of the clone block
  int lc_ext, lc_intr;  // local columns of its camera's calibration (-1 if absent)
  int pad;
};

// A local variable of a feature: covariance id, canonical column, size, local column
struct DVar {
  int pid, canon, size, loc;
};

// One feature of an update batch
struct DFeat {
  int meas_off, nmeas;  // into the measurement array (reference iteration order)
  int var_off, nvar;    // into the variable array
  int nf;               // local Jacobian columns (sum of var sizes)
  int row_off;          // first output row in H_all
  int anchor_cam, anchor_slot;  // FeatureInitializer anchor (host-computed, FeatureInitializer.cpp:35-45)
  int lc_anchor_clone, lc_anchor_ext;  // local cols of the anchor clone / anchor cam extrinsic (anchored reps)
  int rep;              // LandmarkRepresentation
  int mode;             // 0 MSCKF (triangulate+refine+nullspace), 1 SLAM update (landmark in state),
                        // 2 delayed init (triangulate+refine, all rows), 3 delayed init at a given triangulation
  double p_in[3];       // SLAM: landmark xyz (value); MSCKF: unused
  double p_in_fej[3];   // SLAM: landmark xyz (fej)
  int lm_pid, lm_loc;   // SLAM: landmark covariance id / local col
  int pad[2];
};

// Per-feature result
struct DFeatOut {
  double p_FinA[3], p_FinG[3];
  double chi2;
  double HfR[9];  // delayed init: the 3x3 upper block of H_f after the reflections (H_finit)
  int status;  // 0 accepted, 1 triangulation failed, 2 refine failed, 3 chi2 rejected
  int rows;    // rows written (accepted)
};

// Parameters shared by one update batch
struct DBatchParams {
  int nfeat;
  int n_canon;     // canonical columns n (residual column stored at index n)
  int ldh;         // leading dimension of H_all (>= n+1)
  int ldp;         // leading dimension of P
  double sigma_pix_sq;
  double chi2_mult;
  int do_fej;
  int calib_ext, calib_intr;
  // FeatureInitializerOptions
  int fi_max_runs, fi_refine, fi_tri1d;
  double fi_init_lamda, fi_max_lamda, fi_min_dx, fi_min_dcost, fi_lam_mult;
  double fi_min_dist, fi_max_dist, fi_max_baseline, fi_max_cond;
  double *dbg;         // optional per-measurement debug record (8 doubles each), nullptr in production
  long long *dbg_ts;   // optional per-feature phase timestamps (8 per feature), nullptr in production
  // device-chained updates (Engine::update_frame): mode 3 takes its triangulation from tri_in[f] (a failed
  // one fails the feature); mode 1 takes its landmark from the additive mirror xv (indexed by covariance id,
  // kept current by k_chain_apply); gate_out (one-feature batches) <- the feature's status == 0
  const DFeatOut *tri_in;
  const double *xv;
  int *gate_out;
};

// ---- launch wrappers (all asynchronous on `s`) ----
// EKFPropagation (StateHelper.cpp:36-114) for a contiguous new block [s0, s0+p) with old index list
// iold (q entries, device), Phi (p x q) and Q (p x p) in device memory.  T is N x p scratch.
void launch_cov_propagate(hipStream_t s, double *P, int ld, int N, int s0, int p, const int *iold, int q,
                          const double *Phi, const double *Q, double *T, const int *rows = nullptr);
// StateHelper::clone of imu->pose() + augment_clone time-offset term (StateHelper.cpp:341-391,579-616)
void launch_clone(hipStream_t s, double *P, int ld, int N, int src0, int dt_id, const double *dnc_dev, int do_dt);
// launch_cov_propagate (contiguous block) + launch_clone in one launch; false (nothing launched) when too large
bool launch_prop_clone(hipStream_t s, double *P, int ld, int N, int s0, int p, const int *iold, int q,
                       const double *Phi, const double *Q, double *T, int src0, int dt_id, const double *dnc_dev,
                       int do_dt);
// StateHelper::marginalize (StateHelper.cpp:271-339): Pout <- P without rows/cols [m0, m0+ms)
void launch_marginalize(hipStream_t s, const double *P, double *Pout, int ld, int N, int m0, int ms);
// Pout (Nn x Nn) <- P[src, src]: several variables marginalized at once (src: the kept indices, device)
void launch_compact(hipStream_t s, const double *P, double *Pout, int ld, int Nn, const int *src);
// several StateHelper::marginalize calls in one launch: kept indices src (ascending), Nn of them
void launch_marginalize_multi(hipStream_t s, const double *P, double *Pout, int ld, int Nn, const int *src);
// diagonal check: writes count of negative diagonal entries to *neg (device int)
void launch_check_diag(hipStream_t s, const double *P, int ld, int N, int *neg);

// MSCKF / SLAM per-feature linearization: triangulation (+LM), Jacobian, nullspace, chi2, rows to H_all
void launch_feature_linearize(hipStream_t s, const DBatchParams &bp, const DFeat *feats, const DMeas *meas,
                              const DVar *vars, const DClone *clones, const DCam *cams, const double *P,
                              const double *chi2_table, double *H_all, DFeatOut *out, int max_meas, int max_nf);
// batched chi2 gate (kernels_chi2.hip): T = H_all P[hidx, hidx], per-feature S / LDL^T / chi2;
// rejected MSCKF / SLAM features get zero rows.  T_all: like H_all.
// sbuf / sbuf_cap: the engine's buffer for the per-feature S of features too large for k_chi2's LDS staging
// (formed by k_chi2_S over many CUs, grown here on demand); nullptr: k_chi2 forms S from global memory itself
void launch_chi2_batch(hipStream_t s, const DBatchParams &bp, const DFeat *feats, const double *P, const int *hidx,
                       double *H_all, int m, double *T_all, const double *chi2_table, DFeatOut *out, int max_rows_f,
                       int *acc_count, double *pcan = nullptr,  // pcan: n^2 scratch for the gathered P_can
                       double **sbuf = nullptr, size_t *sbuf_cap = nullptr);
size_t feature_lds_bytes(int max_meas, int max_nf);

// Compression: G = A^T A over rows of A = H_all (m x (n+1), ld = ldh), partials then Cholesky ->
// R_aug ((n+1) x (n+1) upper, ld = ldr).  Rank-deficient pivots produce zero rows.
void launch_gram(hipStream_t s, const double *A, int m, int ncol, int ldh, double *partials, int *nchunks_out);
int gram_num_chunks(int m);
// Feature sharding: a rank's Gram partials summed into one (ncol x ncol) upper triangle,
// followed by [accepted features, accepted rows] of its batch, the buffer every rank all-reduces; after the
// sum the accepted-feature total becomes the P-update gate again.
void launch_shard_pack(hipStream_t s, const double *partials, int nch, int ncol, const DFeatOut *fout, int nf,
                       const int *acc, double *buf);
void launch_shard_unpack(hipStream_t s, const double *buf, int ncol, int *acc);
void launch_gram_reduce_chol(hipStream_t s, const double *partials, int nchunks, int ncol, double *R, int ldr);

// EKF update (StateHelper::EKFUpdate, StateHelper.cpp:116-197) for H (r x n, ld = ldh) whose column j
// maps to covariance index hidx[j] (device), residual res (r, device, stride res_stride), noise sigma2.
// Scratch: M (N x r), W (N x r), S (5 r x r: L^-1, -, S_up, global factor work), y (r), dx (N), neg (int).
constexpr int kMaxEkfRows = 255;        // rows of one direct (uncompressed) EKF update (+ residual <= 256)
constexpr int kMaxDynLds = 152 * 1024;  // dynamic LDS budget of the single-workgroup solvers
// S holds 5 r^2 doubles for r rows
// The ranges of one UwbData message as one device chain (Engine::uwb_update_message; UpdaterUWB::update_single,
// UpdaterUWB.cpp:53-90, per range in the message's order): the linearization state of the message's rows, moved
// by each accepted range's dx on the device with Var::update's formulas
constexpr int kUwbMaxRanges = 16;
struct DUwbState {
  double q[4], p[3];               // IMU q_GtoI, p_IinG
  double pU[3];                    // p_IinU
  double anc[kUwbMaxRanges][5];    // range j's anchor [p_AinG, const_bias, dist_bias]
  double range[kUwbMaxRanges];
  int id_imu, id_cal;              // covariance ids (id_cal < 0: p_IinU not calibrated)
  int id_anc[kUwbMaxRanges];       // < 0: fixed anchor (no columns)
  int nr;
};
// range j: apply range j-1's dx to the state if it was accepted (prev: its region, null for j = 0), then form
// the row h (n + 1 doubles, residual last) and zero the region's header
void launch_uwb_row(hipStream_t s, DUwbState *st, int j, const double *prev, double *h, double *region);
// M = P[:, hidx] h
void launch_uwb_M(hipStream_t s, const double *P, int ldp, int N, const double *h, const int *hidx, int n, double *M);
// S = h^T M[hidx] + s2, chi2 = res^2 / S against thr; accepted: P -= W W^T (W = M / sqrt S), dx = W res / sqrt S.
// region: [accepted, negative diagonals (int), chi2, S | dx (N)]
void launch_uwb_update(hipStream_t s, double *P, int ldp, int N, const double *M, const double *h, const int *hidx,
                       int n, double s2, double thr, double *region);

struct EkfScratch {
  double *M, *W, *S, *y, *dx;
  int *neg;
  double *Dinv;  // 16x16 diagonal-block inverses of a triangular factor: (rmax / 16 + 1) * 256
  const int *gate = nullptr;  // optional device count: when it is 0 the P update is skipped (no rows accepted)
  // StateHelper::initialize's chi2 test (StateHelper.cpp:458-470) on the update's own factor: when
  // chi2_gate is set, chi2 = |L^-1 r|^2 of the factored S is compared with chi2_thr right after the
  // factorization; *chi2_gate (the P-update gate) = accepted, and [chi2, accepted] go to dx[N], dx[N+1]
  int *chi2_gate = nullptr;
  double chi2_thr = 0.0;
  KProf *kp = nullptr;  // live kernel timing (kprof.h), null = off
  // optional T = H P_II (r x n rows, ld ldt) of the same H and columns, left by the batch's chi2 gate with
  // rejected rows zeroed: k_ekf_MS then forms S_up = H T^T without recomputing T
  const double *Tall = nullptr;
  int ldt = 0;
  double *M3 = nullptr;  // the delayed-init candidate's initialize_invertible M (N x 3)
};
// W (N x r, ld r) = M L^-T for lower-triangular L (r x r, ld ldl); M row-major (ldm) or, with hidx, the
// columns P[:, hidx] of P (ldm = ldp).  Dinv: scratch as in EkfScratch.
// form_dinv: k_trinv16 forms Dinv from L first (false: Dinv was written by the factorization that made L)
void launch_trsm_lt(hipStream_t s, const double *M, int ldm, const int *hidx, int N, int r, const double *L, int ldl,
                    double *Dinv, double *W, bool form_dinv = true);
void launch_ekf_update(hipStream_t s, double *P, int ldp, int N, const double *H, int ldh, int r, int n,
                       const int *hidx, const double *res, int res_stride, double sigma2, EkfScratch &sc);
// information-form update for a compressed batch (m > n): G = [H r]^T [H r] from k_gram partials;
// Gbuf holds (n+1)^2 doubles.  Same P / dx outputs as launch_ekf_update on the Givens R factor.
void launch_ekf_info(hipStream_t s, double *P, int ldp, int N, const double *partials, int nch, int n,
                     const int *hidx, double sigma2, double *Gbuf, EkfScratch &sc);
// its two halves: _pre (P_II = L L^T, V = P[:,I] L^-T; reads P and hidx only) and _post (Gram reduce, Z, X,
// P update, dx), for running the prefactor on a side stream while the Gram's rows are formed
void launch_ekf_info_pre(hipStream_t s, const double *P, int ldp, int N, int n, const int *hidx, EkfScratch &sc);
void launch_ekf_info_post(hipStream_t s, double *P, int ldp, int N, const double *partials, int nch, int n,
                          double sigma2, double *Gbuf, EkfScratch &sc);
// the same update split at the innovation covariance: phase A leaves S_up = H P H^T + s2 I (r x r) at
// sc.S + 2 r^2 (used by gated single-row updates such as UWB); phase B finishes the update.
void launch_ekf_phaseA(hipStream_t s, const double *P, int ldp, int N, const double *H, int ldh, int r, int n,
                       const int *hidx, double sigma2, EkfScratch &sc);
void launch_ekf_phaseB(hipStream_t s, double *P, int ldp, int N, int r, const double *res, int res_stride,
                       EkfScratch &sc);
// M = P[:, hidx] H^T (N x r, ld r) alone (k_ekf_MS without its S blocks); zero (optional): set to 0
void launch_ekf_M(hipStream_t s, const double *P, int ldp, int N, const double *H, int ldh, int r, int n,
                  const int *hidx, double *M, int *zero);
// StateHelper::initialize_invertible for a 3-dof variable appended at N (StateHelper.cpp:484-577)
// fout != nullptr: H_Linv = inverse of fout->HfR (formed on the device); gate: skipped when *gate == 0;
// resout != nullptr: receives the residual column of rows 0..2 (Hx[a][n]), for the host's value update
void launch_init_invertible(hipStream_t s, double *P, int ldp, int N, const double *Hx, int ldh, int n,
                            const int *hidx, const double *HLinv, double s2, EkfScratch &sc,
                            const DFeatOut *fout = nullptr, const int *gate = nullptr, double *resout = nullptr);
// the JPL pose value behind a clone / camera-extrinsic table entry (PoseJPL: q_GtoI / q_ItoC, position) and its
// covariance id, updated on the device inside a delayed-initialization chain
struct DPoseVal {
  double q[4], p[3];
  int pid, pad;
};
// One step of a device update chain (Engine::update_frame, Engine::slam_delayed_chain): the update's acceptance
// (fout's linearization status if given, the gate if given: accepted rows / the chi2 test of its factor) into
// out[0], its negative-diagonal count into out[1]; accepted with an update (dx): the clone / camera tables
// the next batch is linearized against get the update (Var::update + quat_2_Rot, the host's formulas) and the
// additive mirror xv[0, Nx) += dx; rejected with slot >= 0: the appended landmark slot's rows / columns
// (slot .. slot+2 over [0, Ntot)) are zeroed.
void launch_chain_apply(hipStream_t s, const DFeatOut *fout, const int *gate, const int *neg, const double *dx,
                        DClone *clones, DPoseVal *cv, int ncl, DCam *cams, DPoseVal *camv, int ncam, int calib_ext,
                        int calib_intr, double *xv, int Nx, double *P, int ldp, int Ntot, int slot, double *out);
// One delayed-initialization candidate (StateHelper::initialize): initialize_invertible of the landmark into the
// slot Ni (H_Linv from fout->HfR, rows Hrow[0..2]), the chi2-gated EKF update of the other nup rows (Hrow + 3,
// residual in column n; sc.chi2_gate: in = the linearization gate, out = accepted; sc.chi2_thr), and the chain
// step of launch_chain_apply (tables moved by dx, or the slot cleared; [accepted, neg] into out), as six launches.
// resout receives the residual column of the three initializing rows.
void launch_di_candidate(hipStream_t s, double *P, int ldp, int Ni, const double *Hrow, int ldh, int nup, int n,
                         const int *hidx, double s2, EkfScratch &sc, const DFeatOut *fout, double *resout,
                         DClone *clones, DPoseVal *cv, int ncl, DCam *cams, DPoseVal *camv, int ncam, int calib_ext,
                         int calib_intr, double *out);
double chi2_quantile95(int dof);

// ---- VioManager::retriangulate_active_tracks (VioManagerHelper.cpp:190-388) on the device ----
// Every observation of the frame (cameras in message order, each camera's tracks in get_last_obs order)
// updates its track's running linear triangulation system; the systems live in a featid-keyed open-
// addressing hash table (two generations: last frame's, this frame's).
struct DRetriObs {
  unsigned long long featid;
  float un, vn, u, v;  // undistorted (undistort_cv) and raw pixel coordinates
  int cam, pad;
};
struct DRetriEntry {
  double A[9], b[3];
  int cnt;
  int last_obs, last_pass;  // index of the track's last observation / last one that triangulated
  int has_uv0;              // seen by camera 0 this frame
  float u0, v0;
  double pos[3];            // p_FinG (valid when last_pass >= 0)
  double uvd[3];
  int uvd_valid;
  int first_obs;  // a track new this frame keeps its FIRST observation's system (std::map::insert)
};
struct DRetriSlam {  // SLAM landmarks: position from the state, cam0 pixel from this frame's tracks
  unsigned long long featid;
  double pos[3];
  double uvd[3];
  int has_uv0, uvd_valid;
  float u0, v0;
};
struct RetriJob {
  int nobs, nslam, cap;  // cap: hash capacity (power of two)
  const DRetriObs *obs;
  double *scratch;       // per observation: A 9, b 3, cnt, pos 3, pass
  unsigned long long *keys_old, *keys_new;
  DRetriEntry *ent_old, *ent_new;
  DRetriSlam *slam;
  double R_GtoC[kMaxCams][9], p_CinG[kMaxCams][3];  // camera poses at the current clone
  double R_ItoC0[9], p_IinC0[3], R_GtoI[9], p_IinG[3];
  int w0, h0;
  double max_cond, min_dist, max_dist;
};
constexpr unsigned long long kRetriEmpty = ~0ull;
void launch_retriangulate(hipStream_t s, const RetriJob &job);

// Raise a kernel's dynamic-LDS limit to `want` bytes, capped so static + dynamic LDS fits the CU's
// 160 KiB.  Returns the granted bytes (0 on failure); a failed call's sticky runtime error is cleared so
// it cannot surface in another library (torch) on this thread.
inline int set_dyn_lds(const void *fn, int want) {
  hipFuncAttributes a{};
  int stat = 0;
  if (hipFuncGetAttributes(&a, fn) == hipSuccess)
    stat = (int)a.sharedSizeBytes;
  else
    (void)hipGetLastError();
  int v = want < 160 * 1024 - stat ? want : 160 * 1024 - stat;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, v) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return v;
}

// ---- KLT front-end (kernels_track.hip) ----
constexpr int kMaxPyrLevels = 8;
// one image pyramid in HBM: level l image (w x h u8, packed) and Scharr derivatives (w x h x 2 int16)
struct DPyr {
  const uint8_t *img[kMaxPyrLevels];
  const int16_t *der[kMaxPyrLevels];
  int w[kMaxPyrLevels], h[kMaxPyrLevels];
  int levels;
};
// one frame's cameras at once: equalizeHist (or copy) of src[c] (row stride stride[c]) into level 0 of
// p[c], then every level's pyrDown + Scharr; hist[c]: 256 u32 scratch per camera
struct PyrJob {
  DPyr p[kMaxCams];
  const uint8_t *src[kMaxCams];
  int stride[kMaxCams];
  unsigned *hist[kMaxCams];
  int ncam, equalize;
};
void launch_pyramids(hipStream_t s, const PyrJob &job);
// algorithmic bytes of launch_pyramids: histogram read, equalized level 0 + Scharr
// written, every further level's source read, level and Scharr written
double pyramid_bytes(const PyrJob &job);
// downsample_cameras (VioManager.cpp:270-278): dst[c] (w x h) = pyrDown(src[c]) of the 2w x 2h input
// (row stride stride[c]), BORDER_REFLECT_101, (sum + 128) >> 8, all cameras in one launch
struct DecimateJob {
  const uint8_t *src[kMaxCams];
  uint8_t *dst[kMaxCams];
  int stride[kMaxCams], w[kMaxCams], h[kMaxCams];
  int ncam;
};
void launch_decimate(hipStream_t s, const DecimateJob &job);
// FAST on the grid cells of up to kMaxCams images in one launch pair: cells (x0, y0 pairs) of camera k are
// [cell_end[k-1], cell_end[k]), each sw[k] x sh[k] of image img[k] (row length w[k]); out: ncell x kmax x
// (x, y, response), out_n: per cell; score[k]: w[k] x h u8 scratch of camera k
struct FastJob {
  const uint8_t *img[kMaxCams];
  uint8_t *score[kMaxCams];
  int w[kMaxCams], sw[kMaxCams], sh[kMaxCams], cell_end[kMaxCams];
  int ncam;
};
// sort_stats (optional, device): [0] += cells whose candidates took std::sort's introsort path (> 16 candidates)
void launch_fast_multi(hipStream_t s, const FastJob &job, const int *cells, int thr, int kmax, float *out, int *out_n,
                       int *sort_stats = nullptr);
// Test probe of the Grider_GRID.h:128 std::sort emulation: per cell (responses resp[off[c] .. off[c+1]) in raster
// order) the arrangement after the introsort loop and, for kmax > 0, the top-min(n, kmax) raster indices in order
void launch_grid_order_probe(hipStream_t s, const uint8_t *resp, const int *off, int ncell, int nmax, int kmax,
                             int depth, int *arrangement, int *top);
void launch_fast_cells(hipStream_t s, const uint8_t *img, int w, int h, const int *cells, int ncell, int sw, int sh, int thr,
                       int kmax, float *out, int *out_n, uint8_t *score_map);
// cornerSubPix in place on the points (x, y) of up to kMaxCams images: points [end[k-1], end[k]) lie in img[k]
// (w[k] x h[k]); mask: (2 win + 1)^2 weights
struct SubpixJob {
  const uint8_t *img[kMaxCams];
  int w[kMaxCams], h[kMaxCams], end[kMaxCams];
  int ncam;
};
void launch_subpix_multi(hipStream_t s, const SubpixJob &job, float *pts, const float *mask, int win, int max_iters,
                         double eps2);
void launch_subpix(hipStream_t s, const uint8_t *img, int w, int h, float *pts, int n, const float *mask, int win,
                   int max_iters, double eps2);
// calcOpticalFlowPyrLK with OPTFLOW_USE_INITIAL_FLOW for up to kMaxCams point sets in one launch: slot k tracks
// n[k] points p0[k] from prev[k] into next[k]; the initial guess is p1[k] (or p0[k] when init_from_p0),
// the result goes to p1[k], the status to st[k]
struct LkSlots {
  DPyr prev[kMaxCams], next[kMaxCams];
  const float *p0[kMaxCams];
  float *p1[kMaxCams];
  uint8_t *st[kMaxCams];
  int n[kMaxCams];
  // optional: algorithmic bytes of the launch accumulated on the device (SURVEY.md §8(d) LK term:
  // 256 (5 + iterations) per point and pyramid level visited)
  unsigned long long *bytes = nullptr;
  // optional (undistort != 0): each point's p0 (camera c0) and result p1 (c1) undistorted into p0n / p1n by
  // its wavefront at the end, RANSAC's inputs (launch_ransac with undistorted = true skips its own pass)
  CamParams c0[kMaxCams], c1[kMaxCams];
  float *p0n[kMaxCams] = {}, *p1n[kMaxCams] = {};
  // optional: p1n's cam_undistort_f ambiguity flag per point (1: the host recomputes it with its libm tan)
  uint8_t *p1amb[kMaxCams] = {};
  int undistort = 0;
};
// CamBase::undistort_f of n points (uv, 2n floats) into uvn on the device, with cam_undistort_f's ambiguity
// flag per point in amb (may be null)
void launch_undistort_points(hipStream_t s, const CamParams &cam, int n, const float *uv, float *uvn, uint8_t *amb);
void launch_lk(hipStream_t s, const LkSlots &job, int nslot, int win, int max_level, int max_iters, float eps,
               bool init_from_p0);
// per slot: undistort p0 (camera c0) and p1 (c1), then findFundamentalMat(FM_RANSAC, thr) over the
// host-drawn subsets sub (max_iters x 7): hypotheses in parallel, sequential adaptive selection, inlier
// mask.  t = thr^2 (float), scratch p0n / p1n (2n), F (27 max_iters), nm (max_iters), good (3 max_iters)
struct RansacSlots {
  CamParams c0[kMaxCams], c1[kMaxCams];
  const float *p0[kMaxCams], *p1[kMaxCams];
  float *p0n[kMaxCams], *p1n[kMaxCams];
  const int *sub[kMaxCams];
  double *F[kMaxCams];
  int *nm[kMaxCams], *good[kMaxCams];
  uint8_t *mask[kMaxCams];
  float t[kMaxCams];
  int n[kMaxCams];
};
void launch_ransac(hipStream_t s, const RansacSlots &job, int nslot, int max_iters, double conf,
                   bool undistorted = false);

}  // namespace uvhp
