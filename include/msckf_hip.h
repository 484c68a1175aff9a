/*
 * msckf_hip.h -- C-ABI of the MI355X-native MSCKF stereo-VIO EKF hot path.
 *
 * The reference (NonStopEagle137/Visual-Inertial-Odometry-MSCKF-Stereo) has no
 * FFI: its boundary is the Python class MSCKF (MSCKF/msckf.py:104-908) whose
 * dense linear algebra sits in seven numba-jitted functions
 * (MSCKF/jit_utils.py:6-187).  Each entry point below replaces one of those
 * call sites; the Python host class (msckf_amd.msckf.MSCKF) keeps the
 * reference's imu_callback / feature_callback API and calls these through
 * ctypes.
 *
 * Conventions
 *   - plain pointers and sizes; host arrays are caller-owned and copied in/out;
 *     device buffers are context-owned.
 *   - return 0 on success, >0 for a benign no-op, <0 for an error (HIP failure,
 *     bad argument, non-positive-definite innovation covariance).  Nothing
 *     throws across the ABI.  msckf_last_error() gives a message.
 *   - asynchronous calls (set_state, propagate, augment, prune, their batch
 *     forms, batch_load / batch_update / batch_triangulate, restore) enqueue
 *     work on the context's stream and return without waiting.  A kernel fault
 *     or copy error of such a call is reported by the NEXT synchronising call
 *     (get_state, readback, batch_results, triangulate, update, sync, ...),
 *     as that call's -2; its msckf_last_error() message names the last
 *     asynchronous call enqueued, so the failure is attributed correctly.
 *   - a context holds B independent filters ("filter slots") of one scalar type
 *     (4 = fp32, 8 = fp64) with a fixed cam-state capacity; a context is
 *     single-threaded (the Python wrapper serialises calls with a lock).
 *   - state layouts (all doubles at the ABI):
 *       IMU record, MSCKF_IMU_LEN doubles:
 *         [0:4] q (JPL x,y,z,w; world->IMU)  [4:7] p  [7:10] v  [10:13] bg
 *         [13:16] ba  [16:20] q_null  [20:23] p_null  [23:26] v_null
 *         [26:35] R_imu_cam0 (row-major)  [35:38] t_cam0_imu  [38:41] gravity
 *         [41] nulls_alias (0/1, quirk Q5)
 *       cam record, MSCKF_CAM_LEN doubles: [0:4] q (world->cam0)  [4:7] p
 *         [7:11] q_null   (position_null aliases p, msckf.py:400)
 *       covariance: D x D row-major, D = 21 + 6 * n_cams, error-state order
 *         [dtheta, dbg, dv, dba, dp, dtheta_ic, dp_ic, (dtheta_c, dp_c) x N].
 */
#ifndef MSCKF_HIP_H
#define MSCKF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSCKF_IMU_LEN 42
#define MSCKF_CAM_LEN 11

/* Filter parameters: the filter fields of ConfigEuRoC / OptimizationConfigEuRoC
 * (MSCKF/config.py:5-124) plus the extrinsics MSCKF.__init__ derives
 * (msckf.py:142-152). */
typedef struct msckf_config_t {
    double gyro_noise, acc_noise, gyro_bias_noise, acc_bias_noise; /* Qc, msckf.py:132-137 */
    double observation_noise;                                     /* sigma^2, msckf.py:560 */
    double R_cam0_cam1[9], t_cam0_cam1[3];                         /* T_cn_cnm1, msckf.py:148-152 */
    double huber_epsilon, estimation_precision, initial_damping;  /* feature.py:92, 234-272 */
    int32_t outer_loop_max_iteration, inner_loop_max_iteration;
} msckf_config_t;

typedef struct msckf_ctx msckf_ctx_t;

/* Replaces MSCKF.__init__ (msckf.py:105-164): allocates the device state of
 * n_filters filters of capacity n_cam_capacity cam states each
 * (1 <= n_cam_capacity <= 128). */
int msckf_create(const msckf_config_t* cfg, int hip_device, int scalar_bytes,
                 int n_filters, int n_cam_capacity, msckf_ctx_t** out);
int msckf_destroy(msckf_ctx_t* ctx);
const char* msckf_last_error(void);
int msckf_scalar_bytes(const msckf_ctx_t* ctx);
/* The HIP device the context runs on (hipGetDevice after selecting it) and
 * its PCI bus id ("dddd:bb:dd.f", hipDeviceGetPCIBusId) -- recorded by the
 * multi-GPU bench so that every replica's device is in its output.  No
 * reference counterpart (the reference has no device). */
int msckf_device_info(const msckf_ctx_t* ctx, int* device_out, char* pci_bus_id, int cap);

/* Whole-state upload / download of one filter slot (initialisation, resets,
 * publish msckf.py:888-908, keyframe selection msckf.py:691-727, tests).
 * cams / P may be NULL on get to skip them. */
int msckf_set_state(msckf_ctx_t* ctx, int filter, const double* imu, int n_cams,
                    const double* cams, const double* P);
int msckf_get_state(msckf_ctx_t* ctx, int filter, double* imu, double* cams,
                    double* P, int* n_cams);
/* Covariance diagonal entries [i0, i0+n) (online_reset, msckf.py:869-871). */
int msckf_get_cov_diag(msckf_ctx_t* ctx, int filter, int i0, int n, double* out);

/* Replaces the per-sample loop of batch_imu_processing -> process_model
 * (msckf.py:262-368) incl. _process_model, _predict_new_state and
 * _propaget_state_Covariance (jit_utils.py:6-135): n samples applied in order,
 * dt[k] = t_k - t_{k-1} (the host owns timestamps). */
int msckf_propagate(msckf_ctx_t* ctx, int filter, int n, const double* dt,
                    const double* gyro, const double* acc);

/* Replaces state_augmentation (msckf.py:385-407) + _state_augmentation
 * (jit_utils.py:137-167): appends a cam state cloned from the IMU pose and
 * grows P by 6 rows / cols. */
int msckf_augment(msckf_ctx_t* ctx, int filter);

/* Replaces Feature.initialize_position (feature.py:167-295) for nf features:
 * feature f observes cam slots obs_cam[obs_off[f]..obs_off[f+1]) with
 * measurements obs_z (4 per observation, u0 v0 u1 v1). */
int msckf_triangulate(msckf_ctx_t* ctx, int filter, int nf, const int32_t* obs_off,
                      const int32_t* obs_cam, const double* obs_z,
                      double* p_w_out, uint8_t* valid_out);

/* Replaces the stacked update of remove_lost_features (msckf.py:661-685) or
 * prune_cam_state_buffer (msckf.py:776-801): per-feature measurement_jacobian
 * + feature_jacobian (msckf.py:429-541), gating_test (606-614) with the
 * caller's per-feature chi2 thresholds, stacking in feature order with the
 * row cap (msckf.py:676-679; row_cap <= 0 = no cap) and measurement_update
 * (543-604, _fastQR / _fastSolve, jit_utils.py:173-179).
 * accepted_out[f] = 1 iff feature f's rows went into the update; gamma_out[f]
 * = its Mahalanobis distance (NaN if not evaluated).  Returns 1 (no-op) when
 * no rows are stacked, like msckf.py:544-545. */
int msckf_update(msckf_ctx_t* ctx, int filter, int nf, const int32_t* obs_off,
                 const int32_t* obs_cam, const double* obs_z, const double* p_w,
                 const double* chi2, int row_cap, uint8_t* accepted_out,
                 double* gamma_out, int32_t* rows_out);

/* Replaces the P compaction + cam-state removal loop (msckf.py:803-818):
 * removes the given cam slots (any order). */
int msckf_prune(msckf_ctx_t* ctx, int filter, int n, const int32_t* cam_slots);

/* ---- multi-filter forms (batched multi-sequence scheduling, SURVEY 8(f)
 * item 3): the per-filter calls above applied to a list of distinct filter
 * slots in ONE launch each.  The single-filter entry points are these with a
 * list of one.  A feature batch for several filters goes through
 * msckf_batch_load + msckf_batch_triangulate / msckf_batch_update.
 *
 * msckf_propagate_batch: filter filters[w] takes samples
 *   [sample_off[w], sample_off[w+1]) of dt / gyro (n x 3) / acc (n x 3)
 *   (batch_imu_processing -> process_model, msckf.py:262-368).
 * msckf_augment_batch: state_augmentation (msckf.py:385-407) of each listed filter.
 * msckf_prune_batch: P compaction + cam removal (msckf.py:803-818); filter
 *   filters[w] drops cam slots cam_slots[slot_off[w] .. slot_off[w+1]).
 * msckf_get_states_batch: IMU records (nfilt x MSCKF_IMU_LEN) and, if
 *   cams_out != NULL, cam records (nfilt x n_cam_capacity x MSCKF_CAM_LEN,
 *   zero past each filter's n_cams) and cam counts -- publish
 *   (msckf.py:888-908) and find_redundant_cam_states (msckf.py:691-727).
 * msckf_get_cov_diag_batch: out[w * n + k] = P_w[i0 + k][i0 + k]
 *   (online_reset, msckf.py:869-871).
 * msckf_batch_triangulate: Feature.initialize_position (feature.py:167-295)
 *   of every feature of the loaded batch; results via msckf_batch_results. */
int msckf_propagate_batch(msckf_ctx_t* ctx, int nfilt, const int32_t* filters, const int32_t* sample_off,
                          const double* dt, const double* gyro, const double* acc);
int msckf_augment_batch(msckf_ctx_t* ctx, int nfilt, const int32_t* filters);
int msckf_prune_batch(msckf_ctx_t* ctx, int nfilt, const int32_t* filters, const int32_t* slot_off,
                      const int32_t* cam_slots);
int msckf_get_states_batch(msckf_ctx_t* ctx, int nfilt, const int32_t* filters, double* imu_out,
                           double* cams_out, int32_t* ncams_out);
int msckf_get_cov_diag_batch(msckf_ctx_t* ctx, int nfilt, const int32_t* filters, int i0, int n, double* out);
int msckf_batch_triangulate(msckf_ctx_t* ctx);
/* A frame's sync point in ONE stream synchronisation (publish, msckf.py:888-908;
 * find_redundant_cam_states 691-727; online_reset 869-871): the listed filters'
 * IMU / cam records as msckf_get_states_batch, their covariance diagonal
 * [i0, i0+n) as msckf_get_cov_diag_batch (n = 0 or cov_out NULL: skipped),
 * and, if any of the last five pointers is non-NULL, the loaded batch's results
 * as msckf_batch_results. */
int msckf_readback(msckf_ctx_t* ctx, int nfilt, const int32_t* filters, double* imu_out, double* cams_out,
                   int32_t* ncams_out, int i0, int n, double* cov_out, uint8_t* accepted_out,
                   double* gamma_out, double* p_w_out, uint8_t* valid_out, int32_t* rows_out);

/* ---- throughput mode: B independent filters, one launch chain per step ----
 * msckf_batch_load copies features for ALL filter slots to HBM once:
 * feat_off[B+1] splits the nf features over slots.  msckf_batch_update then
 * runs triangulation (if flags & MSCKF_TRIANGULATE) + the full update chain on
 * the resident data, asynchronously; msckf_sync waits.  Triangulation covers
 * every feature when p_w is NULL, else only the features whose p_w row is not
 * finite (NaN: "not initialised"): a row given by the host is never
 * re-triangulated, so one chain serves remove_lost_features' mix of
 * initialised and new features (msckf.py:640 initialize_position, then
 * the stacked update).  A feature whose row stays non-finite (no
 * MSCKF_TRIANGULATE) or whose triangulation fails is not gated (valid = 0).
 * msckf_batch_results reads everything back with one stream synchronisation,
 * so a caller may defer it (the drop-in host does, until its next sync point).  msckf_snapshot /
 * msckf_restore copy the whole device state (P, IMU, cams) to / from a
 * shadow buffer on the device (so repeated timed steps do identical work). */
#define MSCKF_TRIANGULATE 1
int msckf_batch_load(msckf_ctx_t* ctx, const int32_t* feat_off, const int32_t* obs_off,
                     const int32_t* obs_cam, const double* obs_z, const double* p_w,
                     const double* chi2);
int msckf_batch_update(msckf_ctx_t* ctx, int row_cap, int flags);
int msckf_batch_results(msckf_ctx_t* ctx, uint8_t* accepted_out, double* gamma_out,
                        double* p_w_out, uint8_t* valid_out, int32_t* rows_out);
int msckf_snapshot(msckf_ctx_t* ctx);
int msckf_restore(msckf_ctx_t* ctx);
int msckf_sync(msckf_ctx_t* ctx);

/* Per-kernel device time (HIP events on the context stream), accumulated
 * while profiling is on.  names: NUL-separated list written to names_out. */
int msckf_set_profiling(msckf_ctx_t* ctx, int on);
/* Profiling of ONE timer stage (e.g. "gate"): every other stage records no
 * events, so the timed stream carries two event packets per step instead of
 * two per stage.  stage == NULL turns profiling off. */
int msckf_set_profiling_stage(msckf_ctx_t* ctx, const char* stage);
int msckf_kernel_times(msckf_ctx_t* ctx, int max_k, double* ms_total, int32_t* launches,
                       char* names_out, int names_cap);

#ifdef __cplusplus
}
#endif
#endif /* MSCKF_HIP_H */
