/*
 * uvio_hp.h — C ABI of the MI355X-native uvio/OpenVINS hot path
 * (track -> propagate -> MSCKF/SLAM/UWB update -> EKF update).
 *
 * This is the drop-in boundary.  The reference exposes C++ classes, not a C ABI
 * (SURVEY.md §8b); every entry point below names the reference interface it
 * replaces (path:line relative to the reference checkout).  All functions return
 * an int status: 0 = ok, < 0 = UVIO_HP_E_*.  They never call exit(); the
 * reference's fatal paths (std::exit on negative covariance diagonal,
 * StateHelper.cpp:112,181; propagation backwards, Propagator.cpp:39,46) become
 * UVIO_HP_E_NUMERIC / UVIO_HP_E_ORDER and leave the handle in a defined state.
 *
 * Threading (mirrors the reference, SURVEY §8b "Threading"): uvio_hp_feed_imu may be
 * called concurrently with the other feeds (IMU buffer is mutex-guarded like
 * Propagator::imu_data_mtx, Propagator.h:68); camera / sim / UWB feeds must be
 * serialized by the caller (single update thread, ROS1Visualizer.h:173).
 *
 * No torch / Eigen / OpenCV types cross this boundary: plain pointers and sizes.
 */
#ifndef UVIO_HP_H
#define UVIO_HP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UVIO_HP_OK 0
#define UVIO_HP_E_ARG (-1)      /* bad argument / size */
#define UVIO_HP_E_STATE (-2)    /* not initialized, or call not valid in this state; every state-changing call
                                   after a fatal error (E_NUMERIC / E_DEVICE / E_INTERNAL, where the reference
                                   std::exit's) returns it: the estimator is stopped, destroy the handle */
#define UVIO_HP_E_DEVICE (-3)   /* HIP runtime error or no MI355X device */
#define UVIO_HP_E_NUMERIC (-4)  /* negative covariance diagonal (ref: std::exit) */
#define UVIO_HP_E_CONFIG (-5)   /* config file missing / unparsable */
#define UVIO_HP_E_ORDER (-6)    /* measurement out of order (ref: std::exit in Propagator) */
#define UVIO_HP_E_CAPACITY (-7) /* a compile-time capacity was exceeded */
#define UVIO_HP_E_INTERNAL (-8) /* unexpected host-side error (a bug): the message names the routine */

#define UVIO_HP_MAX_CAMS 4
#define UVIO_HP_MAX_ANCHORS 16

/* ---- option structs: the keys of estimator_config.yaml / kalibr_*.yaml / uwb_*.yaml ---- */

typedef struct {
  int model;       /* 0 = radtan (pinhole-radtan, CamRadtan.h), 1 = equidistant (CamEqui.h) */
  int width, height;
  double intrinsics[8]; /* fx fy cx cy d0 d1 d2 d3 (CamBase::set_value, CamBase.h:56) */
  double q_ItoC[4];     /* JPL quaternion of R_ItoC (x y z w), from T_imu_cam (VioManagerOptions.h) */
  double p_IinC[3];
} uvio_hp_camera_t;

typedef struct {
  uint64_t id;
  int fix;
  double p_AinG[3];
  double const_bias, dist_bias;
  double cov_diag[5]; /* p p p c d (UVioManagerOptions.h:80) */
} uvio_hp_anchor_t;

typedef struct {
  /* StateOptions (ov_msckf/src/state/StateOptions.h:41-96) */
  int do_fej;
  int integration;            /* 0 discrete, 1 rk4, 2 analytical */
  int num_cameras;
  int use_stereo;
  int do_calib_camera_pose;
  int do_calib_camera_intrinsics;
  int do_calib_camera_timeoffset;
  int do_calib_imu_intrinsics;
  int do_calib_imu_g_sensitivity;
  int imu_model;              /* 0 kalibr, 1 rpng */
  int max_clone_size;
  int max_slam_features;
  int max_slam_in_update;
  int max_msckf_in_update;
  int max_aruco_features;
  int feat_rep_msckf;         /* LandmarkRepresentation (LandmarkRepresentation.h:38) */
  int feat_rep_slam;
  double dt_slam_delay;
  double gravity_mag;
  double calib_camimu_dt;
  /* UpdaterOptions (UpdaterOptions.h:33-44) */
  double msckf_sigma_pix, msckf_chi2_multipler;
  double slam_sigma_pix, slam_chi2_multipler;
  /* NoiseManager (Propagator.h:44) */
  double sigma_w, sigma_a, sigma_wb, sigma_ab;
  /* IMU intrinsics initial values (kalibr_imu_chain.yaml: Tw, Ta, Tg, R_IMUtoGYRO, R_IMUtoACC) */
  double imu_dw[6], imu_da[6], imu_tg[9];
  double q_GYROtoIMU[4], q_ACCtoIMU[4];
  /* FeatureInitializerOptions (FeatureInitializerOptions.h:33-70) */
  int fi_triangulate_1d, fi_refine_features, fi_max_runs;
  double fi_init_lamda, fi_max_lamda, fi_min_dx, fi_min_dcost, fi_lam_mult;
  double fi_min_dist, fi_max_dist, fi_max_baseline, fi_max_cond_number;
  /* cameras */
  uvio_hp_camera_t cams[UVIO_HP_MAX_CAMS];
  /* TrackKLT front-end (estimator_config.yaml: num_pts .. histogram_method) */
  int num_pts, fast_threshold, grid_x, grid_y, min_px_dist;
  int histogram_method;       /* 0 none, 1 histogram, 2 clahe */
  int downsample_cameras;     /* cams[].width/height/fx fy cx cy are the halved values (VioManagerOptions.h:251-260);
                               * camera feeds then take the raw 2 width x 2 height images */
  double track_frequency;
  /* uvio (UVioManagerOptions.h:52-90, UVioStateOptions.h:45, UVioUpdaterOptions.h:46) */
  int use_uwb;
  int do_calib_uwb_extrinsics;
  double prior_uwb_imu_cov;
  double uwb_sigma_range, uwb_chi2_multipler;
  double min_dist_to_use_uwb;
  double p_IinU[3];           /* uwb_extrinsics = -p_UinI */
  int n_anchors_to_fix;
  int n_anchors;
  uvio_hp_anchor_t anchors[UVIO_HP_MAX_ANCHORS];
  /* runtime */
  int record_timing;          /* per-frame stage timings (VioManager.cpp:631-644 schema); 1: host wall
                               * times + device event timing of the feature group, 2: also wait for the
                               * device at stage boundaries so each stage time includes its kernels */
  /* InertialInitializerOptions::init_max_features (InertialInitializerOptions.h:73): the KLT tracker
   * keeps floor(init_max_features / num_cameras) tracks per camera until an initializer succeeds
   * (VioManager.cpp:131; initialize_with_gt does not raise it to num_pts, VioManagerHelper.cpp:40) */
  int init_max_features;
  /* UpdaterZeroVelocity (VioManagerOptions.h:83-95, zupt_chi2_multipler :175) */
  int try_zupt;
  double zupt_chi2_multipler, zupt_max_velocity, zupt_noise_multiplier, zupt_max_disparity;
  int zupt_only_at_beginning;
  /* front-end selection (VioManagerOptions.h:440-452): the KLT front-end is the one implemented; use_klt = 0
   * (ORB descriptors) and use_aruco = 1 are rejected with UVIO_HP_E_CONFIG by uvio_hp_create */
  int use_klt, use_aruco;
  /* VioManagerOptions.h:98-101: per-frame timing rows in the reference CSV schema (VioManager.cpp:105-122,
   * 631-644); the file is recreated at uvio_hp_create */
  int record_timing_information;
  char record_timing_filepath[256];
  /* InertialInitializerOptions (InertialInitializerOptions.h:64-76): the static initializer's window (also
   * the IMU kept before initialization, VioManager.cpp:174-176), accelerometer excitation threshold, rest
   * disparity threshold; init_dyn_use selects the dynamic initializer, which is not built */
  double init_window_time, init_imu_thresh, init_max_disparity;
  int init_dyn_use;
} uvio_hp_options_t;

/* Per-frame stage timings in seconds, the reference CSV schema
 * "# timestamp (sec),tracking,propagation,msckf update,slam update,slam delayed,re-tri & marg,total"
 * (VioManager.cpp:117-121, rows :631-644). */
typedef struct {
  double timestamp;
  double tracking, propagation, msckf_update, slam_update, slam_delayed, marg, total;
  int n_msckf, n_slam, n_slam_delayed, n_clones, cov_dim;
  int msckf_rows;   /* stacked rows m before compression */
  int msckf_cols;   /* H columns n */
  /* device-side measurement of the per-feature linearize kernel over this frame (HIP events on the
   * library's stream, recorded only while uvio_hp_set_kernel_timing has timing on; zero otherwise):
   * launches, summed kernel seconds, and algorithmic FP64 FLOPs of those launches
   * (3 Householder reflections 12*(2m_f)*(n_f+4) + chi2 2 r n^2 + 2 r^2 n + r^3/3 per feature) */
  int k_feat_launches;
  double k_feat_s;
  double k_feat_flops;
  /* host waits on the device during this frame (tracker + estimator): count and seconds blocked */
  int device_syncs;
  double sync_wait;
  int zupt;  /* 1: this frame ended in a zero-velocity update (UpdaterZeroVelocity::try_update accepted) */
  int n_anchor_change;  /* SLAM landmarks re-anchored by UpdaterSLAM::change_anchors this frame (UpdaterSLAM.cpp:481-503) */
  /* the per-frame device update chain (MSCKF, SLAM chunks, delayed initialization enqueued back to back, DESIGN.md
   * §4): seconds of its single wait for the device plus the host replay of the results.  The chain books this
   * time in slam_delayed (the last stage); msckf_update / slam_update hold the host enqueue times of theirs */
  double chain_wait;
  /* upload staging ring this frame: restarts of the ring (each waits for the device), and 1 when
   * the update chain's state blob had to be copied out of the ring's previous epoch (engine_chain.cpp) */
  int stage_restarts;
  int chain_blob_old_epoch;
} uvio_hp_timing_t;

/* Live device timing of the kernel classes the benchmark prices against a roofline (HIP events on the
 * library stream around each launch of the class): cumulative since the timing was
 * switched on.  bound: 0 = HBM bandwidth (bytes), 1 = FP64 matrix / vector peak (flops); flops / bytes are
 * the ALGORITHMIC counts of the launches; kernels = the kernel names of the class as
 * rocprofv3 reports them (comma separated). */
typedef struct {
  char name[24];
  char kernels[192];
  int bound;
  long long launches;
  double seconds, flops, bytes;
} uvio_hp_kstat_t;

typedef struct uvio_hp uvio_hp_t;

/* ---- options ---- */
/* Defaults of the reference option structs (StateOptions.h, UpdaterOptions.h, ...). */
int uvio_hp_options_default(uvio_hp_options_t *opts);
/* Parse estimator_config.yaml (+ relative_config_imu / relative_config_imucam / config_uwb files)
 * with the reference's keys (YamlParser, opencv_yaml_parse.h:65-163; VioManagerOptions::print_and_load).
 * Only the keys present in the files are written: call uvio_hp_options_default on the struct first (as
 * the reference's option structs start from their defaults). */
int uvio_hp_options_load(const char *estimator_config_path, uvio_hp_options_t *opts);

/* ---- lifetime ---- */
/* replaces ov_msckf::VioManager::VioManager(VioManagerOptions&) (VioManager.cpp:50) and
 * uvio::UVioManager::UVioManager (uvio/src/core/UVioManager.cpp:26). device = HIP ordinal. */
int uvio_hp_create(const uvio_hp_options_t *opts, int device, uvio_hp_t **out);
int uvio_hp_destroy(uvio_hp_t *h);
/* message of the last failed call on h; with h == NULL, why the last uvio_hp_create on this thread failed */
const char *uvio_hp_last_error(const uvio_hp_t *h);

/* ---- feeds (VioManager.h:75-96, UVioManager.h:48-60) ---- */
/* VioManager::initialize_with_gt(Matrix<17,1>) (VioManagerHelper.cpp:40): x = [t, q_GtoI(4), p, v, bg, ba] */
int uvio_hp_initialize_with_gt(uvio_hp_t *h, const double x[17]);
/* VioManager::feed_measurement_imu (VioManager.cpp:166) */
int uvio_hp_feed_imu(uvio_hp_t *h, double t, const double wm[3], const double am[3]);
/* n consecutive feed_measurement_imu calls in one: t[n], wm[3n], am[3n] (a driver that receives IMU
 * samples in bursts between camera frames saves the per-call overhead) */
int uvio_hp_feed_imu_batch(uvio_hp_t *h, int n, const double *t, const double *wm, const double *am);
/* VioManager::feed_measurement_simulation (VioManager.cpp:191) — TrackSIM path.  For camera i
 * (i < ncam) there are counts[i] features; ids/uv are concatenated over cameras, uv as (u,v) pairs. */
int uvio_hp_feed_simulation(uvio_hp_t *h, double t, int ncam, const int *cam_ids, const int *counts,
                            const uint64_t *ids, const float *uv);
/* VioManager::feed_measurement_camera / UVioManager::feed_measurement_camera (UVioManager.h:48).
 * imgs[i] is a u8 W x H image with row stride strides[i]; masks may be NULL. */
int uvio_hp_feed_camera(uvio_hp_t *h, double t, int ncam, const int *cam_ids, const uint8_t *const *imgs,
                        const int *strides, const uint8_t *const *masks);
/* The same with imgs[i] in device memory (HBM-resident input, e.g. a camera DMA buffer or a torch
 * tensor); the images must be complete (their producer synchronized) before the call.  masks stay
 * host pointers. */
int uvio_hp_feed_camera_device(uvio_hp_t *h, double t, int ncam, const int *cam_ids, const uint8_t *const *imgs,
                               const int *strides, const uint8_t *const *masks);
/* UVioManager::feed_measurement_uwb (UVioManager.cpp:61): one UwbData message */
int uvio_hp_feed_uwb(uvio_hp_t *h, double t, int n, const uint64_t *anchor_ids, const double *ranges);
/* UVioManager::try_to_initialize_uwb_anchors (UVioManager.cpp:81) */
int uvio_hp_init_anchors(uvio_hp_t *h, int n, const uvio_hp_anchor_t *anchors);

/* ---- getters (VioManager.h:99-111) ---- */
int uvio_hp_initialized(const uvio_hp_t *h, int *out);
/* IMU value [q(4) p(3) v(3) bg(3) ba(3)] and the state time */
int uvio_hp_get_imu_state(uvio_hp_t *h, double *t, double out[16]);
/* covariance dimension N (State::max_covariance_size, State.h:88) */
int uvio_hp_get_cov_dim(uvio_hp_t *h, int *n);
/* dense N x N covariance into out with leading dimension ld (row-major) */
int uvio_hp_get_cov(uvio_hp_t *h, double *out, int ld);
/* the state mean in State::_variables order (each variable's value(): quat 4 + ...);
 * *len receives the number of doubles written; meta (optional, 3 ints per variable:
 * kind, covariance id, covariance size) */
int uvio_hp_get_state_vector(uvio_hp_t *h, double *out, int cap, int *len, int *meta, int meta_cap, int *nvars);
/* the first-estimate (FEJ) values, same layout as uvio_hp_get_state_vector (Type::fej(), Type.h:87) */
int uvio_hp_get_fej_vector(uvio_hp_t *h, double *out, int cap, int *len);
/* timings of the last processed frame */
int uvio_hp_get_timing(uvio_hp_t *h, uvio_hp_timing_t *out);
/* live per-class kernel timing: 0 = off (default), k > 0 = the launches of every k-th camera / simulated
 * frame are timed (each timed launch costs two event records on the host) */
int uvio_hp_set_kernel_timing(uvio_hp_t *h, int period);
/* the per-class statistics (*n receives the number of classes); flush = 1 waits for the device first so
 * every launch enqueued so far is counted */
int uvio_hp_get_kernel_stats(uvio_hp_t *h, int flush, uvio_hp_kstat_t *out, int cap, int *n);
/* VioManager::get_active_tracks (VioManager.h:114, filled by retriangulate_active_tracks,
 * VioManagerHelper.cpp:190-388): the current tracks' positions p_FinG (3 per track) and, for the tracks seen
 * by camera 0 in front of it and inside its image, (u, v, depth) (3 per track, uvd_valid 1); *t receives
 * active_tracks_time.  *n receives the number of tracks (E_CAPACITY if > cap). */
int uvio_hp_get_active_tracks(uvio_hp_t *h, double *t, uint64_t *ids, double *posinG, double *uvd, int *uvd_valid,
                              int cap, int *n);
/* number of clones and their timestamps (ascending) */
int uvio_hp_get_clone_times(uvio_hp_t *h, double *out, int cap, int *n);
/* TrackBase::get_last_obs / get_last_ids (TrackBase.h:137-148) for one camera: ids and raw (u, v) of
 * the KLT tracks after the last camera feed; *n receives the count (E_CAPACITY if > cap) */
int uvio_hp_get_tracks(uvio_hp_t *h, int cam, uint64_t *ids, float *uv, int cap, int *n);
/* the last image pyramid of one camera (TrackKLT::img_pyramid_last, TrackKLT.h:147): level size,
 * the (equalized) u8 image (w*h) and interleaved Scharr (dx, dy) int16 derivatives (w*h*2); img / der
 * may be NULL, cap = pixels available */
int uvio_hp_get_pyramid(uvio_hp_t *h, int cam, int level, int *w, int *hgt, uint8_t *img, int16_t *der, size_t cap);

/* ---- Updater-level boundary: one updater call on the handle's current state ----
 * These mirror the reference's Updater C++ surfaces for a caller that keeps its own feature database
 * (the feeds above run the whole VioManager frame instead).  Features come as flat arrays: feature i has
 * id featids[i] and the measurements meas[meas_off[i] .. meas_off[i+1]) in the order they were observed
 * (the order FeatureDatabase::update_feature appended them, FeatureDatabase.cpp:59-98); a camera's track
 * is created at its first measurement, which reproduces ov_core::Feature's per-camera map order.  The
 * results (one record per input feature) say what the reference leaves on the Feature and in
 * feature_vec.  The covariance never leaves the device; each call reads back only dx. */
typedef struct {
  int cam;          /* camera id */
  double t;         /* Feature::timestamps[cam] entry */
  float u, v;       /* Feature::uvs[cam] entry (raw pixel) */
  float un, vn;     /* Feature::uvs_norm[cam] entry (undistorted, normalized) */
} uvio_hp_feat_meas_t;

typedef struct {
  uint64_t featid;
  int status;       /* 0 used by the update (kept in feature_vec); 1 too few measurements or triangulation failed;
                     * 2 Gauss-Newton refinement failed; 3 chi2 rejected (all but 0 are erased from feature_vec) */
  int to_delete;    /* Feature::to_delete after the call */
  double p_FinG[3]; /* the triangulated position (MSCKF / delayed init; zero when not triangulated) */
  double chi2;      /* the chi2 the gate compared (0 when not gated) */
} uvio_hp_feat_result_t;

/* Overwrite the mean, the first estimates and the covariance (a state snapshot in the layout of
 * uvio_hp_get_state_vector / uvio_hp_get_fej_vector / uvio_hp_get_cov: same variables, len doubles,
 * N x N covariance with leading dimension ld).  Camera intrinsics follow the state (StateHelper.cpp:190-195). */
int uvio_hp_set_state(uvio_hp_t *h, const double *val, const double *fej, int len, const double *P, int N, int ld);
/* Propagator::propagate_and_clone (Propagator.h:110) to t with the IMU readings fed so far */
int uvio_hp_propagate_and_clone(uvio_hp_t *h, double t);
/* UpdaterMSCKF::update (UpdaterMSCKF.h:68, UpdaterMSCKF.cpp:58-295) */
int uvio_hp_msckf_update(uvio_hp_t *h, int nfeat, const uint64_t *featids, const int *meas_off,
                         const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out);
/* UpdaterSLAM::update (UpdaterSLAM.h:70, UpdaterSLAM.cpp:253-479); every feature must be a SLAM landmark of
 * the state (UVIO_HP_E_ARG otherwise); a chi2 rejection raises the landmark's fail count as in the reference */
int uvio_hp_slam_update(uvio_hp_t *h, int nfeat, const uint64_t *featids, const int *meas_off,
                        const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out);
/* UpdaterSLAM::delayed_init (UpdaterSLAM.h:77, UpdaterSLAM.cpp:61-251): accepted features (status 0) become
 * SLAM landmarks of the state in the configured feat_rep_slam */
int uvio_hp_slam_delayed_init(uvio_hp_t *h, int nfeat, const uint64_t *featids, const int *meas_off,
                              const uvio_hp_feat_meas_t *meas, uvio_hp_feat_result_t *out);
/* UpdaterSLAM::change_anchors (UpdaterSLAM.h:87, UpdaterSLAM.cpp:481-647) */
int uvio_hp_slam_change_anchors(uvio_hp_t *h);
/* StateHelper::marginalize_slam / marginalize_old_clone (StateHelper.h:230, :224) */
int uvio_hp_marginalize_slam(uvio_hp_t *h);
int uvio_hp_marginalize_old_clone(uvio_hp_t *h);
/* UpdaterUWB::update_single (UpdaterUWB.h:55, UpdaterUWB.cpp:53-90): one range to one initialized anchor on
 * the current state (t is the measurement time; the reference's Jacobian does not use it); *applied = 1
 * when the chi2 test passed and the update ran, 0 when it was gated or the anchor is unknown */
int uvio_hp_uwb_update_single(uvio_hp_t *h, double t, uint64_t anchor_id, double range, int *applied);

/* ---- feature-sharded MSCKF update across GPUs (BASELINE.json configs 4-5) ----
 * One process per GPU, each with its own handle fed the same measurement stream (the filter state is
 * replicated).  Inside UpdaterMSCKF::update (UpdaterMSCKF.cpp:58-295) the selected features are split into
 * contiguous chunks balanced by stacked rows (uvio_hp_shard_partition); each rank triangulates, linearizes,
 * nullspace-projects and chi2-gates its own chunk and forms its Gram block [H r]^T [H r]; the blocks are
 * summed across ranks (ncclAllReduce on the library's stream, or a host callback), and every rank applies
 * the same information-form update (the compressed update, UpdaterHelper.cpp:456-487 +
 * StateHelper::EKFUpdate, depends on the stacked rows only through that sum).  Updates with fewer than
 * min_features features run unsharded on every rank.  Every rank must make every feed call. */
/* In-place sum of count doubles (host memory) over all ranks; returns 0 on success. */
typedef int (*uvio_hp_allreduce_fn)(double *buf, size_t count, void *user);
/* ncclGetUniqueId: rank 0 creates it, the caller distributes the 128 bytes to every rank */
int uvio_hp_shard_unique_id(uint8_t id[128]);
/* RCCL communicator over the ranks (ncclCommInitRank: collective, every rank calls it) */
int uvio_hp_shard_init_rccl(uvio_hp_t *h, int rank, int world, const uint8_t id[128], int min_features);
/* host all-reduce callback instead of RCCL (e.g. a gloo process group; ranks may share one GPU) */
int uvio_hp_shard_init_host(uvio_hp_t *h, int rank, int world, uvio_hp_allreduce_fn fn, void *user,
                            int min_features);
/* the partition the update uses: rows[i] = stacked rows of feature i (2 m_f - 3); bounds (world + 1
 * ints) receives the contiguous ranges [bounds[r], bounds[r+1]) balanced by their row sums. */
int uvio_hp_shard_partition(const int *rows, int n, int world, int *bounds);

/* ---- inner (kernel-level) boundary used by parity tests ---- */
/* per-feature results of the last UpdaterMSCKF::update: feature id, triangulated p_FinG (3 per
 * feature), status (0 accepted, 1 triangulation/refinement failed, 3 chi2 rejected) and chi2 */
int uvio_hp_debug_last_msckf(uvio_hp_t *h, uint64_t *ids, double *pG, int *status, double *chi2, int cap, int *n);
/* per-feature results of every updater call of the last camera frame, in call order: kind (0
 * UpdaterMSCKF::update, 1 UpdaterSLAM::update, 2 UpdaterSLAM::delayed_init), feature id, p_FinG (MSCKF:
 * triangulated; delayed init: triangulated before the landmark's initialization; SLAM update: 0),
 * status (0 accepted, 1 triangulation/refinement failed or too few measurements, 3 chi2 rejected) and
 * chi2 (delayed init: StateHelper::initialize's test, StateHelper.cpp:451-470).  The lock-step tests
 * hand these to the oracle's rounding-tie witness (oracle/src/flip.h). */
int uvio_hp_debug_frame_feats(uvio_hp_t *h, int *kind, uint64_t *ids, double *pG, int *status, double *chi2, int cap,
                              int *n);
/* StateHelper::EKFUpdate (StateHelper.cpp:116) on a standalone covariance: P (N x N, row-major,
 * in/out, host memory), H (r x n, row-major) whose column j maps to covariance index H_index[j]
 * (the H_order blocks flattened), residual (r), isotropic noise sigma2.  dx_out (N) receives K*res.
 * The update runs on the device (same kernels as the manager). */
int uvio_hp_ekf_update(double *P, int N, const int *H_index, int n, const double *H, int r,
                       const double *res, double sigma2, double *dx_out);
/* UpdaterMSCKF.cpp:274-286: measurement_compress_inplace of the stacked [H | res] (m x n) followed by
 * StateHelper::EKFUpdate on the compressed rows, on a standalone covariance (same arguments as
 * uvio_hp_ekf_update).  When m > n the device runs the update in information form on H^T H, H^T res
 * (the quantities the compressed system carries); otherwise it is uvio_hp_ekf_update. */
int uvio_hp_msckf_compressed_update(double *P, int N, const int *H_index, int n, const double *H, int m,
                                    const double *res, double sigma2, double *dx_out);
/* UpdaterHelper::measurement_compress_inplace (UpdaterHelper.cpp:456) semantics: A = [H | res]
 * (m x (n+1), row-major) -> the (n+1) x (n+1) upper-triangular R factor of A (rows of the reference's
 * compressed [H|res] up to a per-row sign; the last row holds the residual norm not explained by H).
 * Computed as the Cholesky factor of the Gram matrix: intended for full-column-rank A (the manager's
 * update does not factor the Gram, see uvio_hp_msckf_compressed_update). */
int uvio_hp_compress(const double *A, int m, int n, double *R_out);
/* CamBase::undistort_f (ov_core/src/cam/CamBase.h:89; CamRadtan.h:99 cv::undistortPoints, CamEqui.h:108
 * cv::fisheye::undistortPoints): n pixel points uv (2n floats) -> normalized uvn (2n floats) for model 0
 * (radtan) or 1 (equidistant), cam = fx fy cx cy d0 d1 d2 d3.  Computed on the device; the equidistant
 * points whose float could depend on the last bit of tan are recomputed on the host (ambiguous[i] = 1,
 * may be null), so uvn equals the host libm result for every point. */
int uvio_hp_undistort(int model, const double cam[8], int n, const float *uv, float *uvn, uint8_t *ambiguous);
/* Grider_GRID.h:128 (std::sort(pts_new, Grider_FAST::compare_response)) as the device's FAST cell selection
 * runs it, on caller-given cells: cell c's responses resp[off[c] .. off[c+1]) in cv::FAST's raster order.
 * arrangement (off[ncell] ints) receives each cell's raster indices as libstdc++'s introsort loop leaves them
 * (std::sort's result is their stable order by response); for kmax in 1..64 top (ncell * kmax ints) receives the
 * first min(n, kmax) raster indices of the sorted cell (unused slots untouched).  depth < 0: the reference's
 * 2 lg n depth limit; 0 forces the heap-sort fallback (std::partial_sort(first, last, last)).  kmax 0: the whole
 * cell is arranged. */
int uvio_hp_debug_grid_order(const uint8_t *resp, const int *off, int ncell, int kmax, int depth, int *arrangement,
                             int *top);
/* the tracker's FAST cells since the handle was created and how many of them had more than 16 candidates
 * (the cells where std::sort's introsort order, not a stable one, decides the selection) */
int uvio_hp_debug_grid_stats(uvio_hp_t *h, uint64_t *cells, uint64_t *introsort_cells);

#ifdef __cplusplus
}
#endif
#endif /* UVIO_HP_H */
