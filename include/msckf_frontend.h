/*
 * msckf_frontend.h -- C-ABI of the GPU stereo front-end (image operators of
 * MSCKF/image.py on gfx950).
 *
 * The reference front-end (class ImageProcessor, MSCKF/image.py:36-702) does
 * its image work through OpenCV calls; each entry point below replaces one of
 * them.  cv2 is absent from this image and from the GPU box: the kernels
 * restate the published OpenCV 4.x algorithms (oracle/frontend_oracle.py),
 * parity unpinned against cv2 itself.  The host side
 * (msckf_amd.frontend.ImageProcessor) keeps the reference's grid bookkeeping,
 * feature ids, pruning and publish logic in Python.
 *
 * Conventions as msckf_hip.h: plain pointers and sizes, host arrays copied
 * in / out, 0 on success and < 0 on error with mfe_last_error().  A context
 * owns NSLOT 8-bit image slots of one resolution; uploading an image into a
 * slot builds its Gaussian pyramid (levels 0..max_level) and the Scharr
 * derivatives of every level on the device.
 */
#ifndef MSCKF_FRONTEND_H
#define MSCKF_FRONTEND_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFE_RADTAN 0
#define MFE_EQUIDISTANT 1

typedef struct mfe_ctx mfe_ctx_t;

/* Replaces the image-side state of ImageProcessor.__init__ (image.py:40-93):
 * nslot image slots of width x height, pyramids of max_level + 1 levels
 * (config.py:33: pyramid_levels = 3), up to max_points points per call. */
int mfe_create(int hip_device, int width, int height, int nslot, int max_level, int max_points,
               mfe_ctx_t** out);
int mfe_destroy(mfe_ctx_t* ctx);
const char* mfe_last_error(void);

/* Replaces create_image_pyramids (image.py:149-164) and the pyramid / Scharr
 * stage of cv2.calcOpticalFlowPyrLK: upload an 8-bit image (row-major,
 * width x height) into a slot. */
int mfe_upload(mfe_ctx_t* ctx, int slot, const uint8_t* image);

/* Replaces cv2.FastFeatureDetector(threshold).detect(img, mask)
 * (image.py:50, 175, 333): FAST 9/16 with score and 3x3 non-max suppression,
 * keypoints in raster order; mask may be NULL (else width x height, 0 =
 * masked out).  Writes min(n, max_kp) keypoints (x, y) and responses; *n_out
 * = the total found. */
int mfe_fast(mfe_ctx_t* ctx, int slot, int threshold, const uint8_t* mask, int max_kp, float* xy_out,
             float* response_out, int* n_out);

/* Replaces cv2.calcOpticalFlowPyrLK(prev, next, prev_pts, next_pts,
 * winSize=(win, win), maxLevel, criteria=(EPS|COUNT, max_iter, eps),
 * flags=OPTFLOW_USE_INITIAL_FLOW) (image.py:254, 581, 585): next_pts is the
 * initial guess on entry and the tracked position on exit; status 1 =
 * tracked. */
int mfe_lk(mfe_ctx_t* ctx, int slot_prev, int slot_next, int n, const float* prev_pts, float* next_pts,
           uint8_t* status, int win, int max_level, int max_iter, double eps);

/* Replaces undistort_points (image.py:640-674: cv2.undistortPoints /
 * cv2.fisheye.undistortPoints): intrinsics [fx fy cx cy], 4 distortion
 * coefficients, rectification R (row-major 3x3, NULL = identity) and new
 * intrinsics (NULL = [1 1 0 0]). */
int mfe_undistort(mfe_ctx_t* ctx, int n, const double* pts_in, double* pts_out, const double* intrinsics,
                  int model, const double* coeffs, const double* R, const double* new_intrinsics);

/* Replaces distort_points (image.py:676-702: cv2.projectPoints with zero pose
 * / cv2.fisheye.distortPoints) of normalised points. */
int mfe_distort(mfe_ctx_t* ctx, int n, const double* pts_in, double* pts_out, const double* intrinsics,
                int model, const double* coeffs);

#ifdef __cplusplus
}
#endif
#endif /* MSCKF_FRONTEND_H */
