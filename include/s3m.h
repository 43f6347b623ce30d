/*
 * s3m.h — dense correspondence (replaces the CUDA half of the pybind module
 * `mast3r_slam_backends`: iter_proj / refine_matches,
 * splatt3r_slam/backend/src/gn.cpp:84-114 -> matching_kernels.cu).
 *
 * Shapes follow the reference exactly (matching_kernels.cu:118-315):
 *   rays_img_with_grad [b,h,w,9] f32, pts_3d_norm [b,n,3] f32,
 *   p_init [b,n,2] f32  ->  p_new [b,n,2] f32, converged [b,n] u8(bool)
 *   D11 [b,h,w,F] f16, D21 [b,n,F] f16, p1 [b,n,2] i64 -> p1_new [b,n,2] i64
 *
 * Floating-point semantics: the restatement evaluates the .cu source
 * strictly (no FMA contraction; the double-precision sub-expressions that
 * the source writes with double literals, e.g. `(1.0-du)*dv` at :157-159,
 * are evaluated in double).  refine_matches accumulates the descriptor dot
 * product exactly as c10::Half arithmetic does: every product and every
 * partial sum is rounded to fp16 (matching_kernels.cu:57-60).
 */
#ifndef S3M_H
#define S3M_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mast3r_slam_backends.iter_proj (gn.cpp:84, matching_kernels.cu:278-315). */
int s3m_iter_proj(const float* rays_img_with_grad, const float* pts_3d_norm,
                  const float* p_init, float* p_new, uint8_t* converged,
                  int b, int h, int w, int n, int max_iter, float lambda_init,
                  float cost_thresh, void* stream);

/* mast3r_slam_backends.refine_matches (gn.cpp:101, matching_kernels.cu:83-115).
 * D11/D21 are IEEE fp16 bit patterns. */
int s3m_refine_matches(const uint16_t* D11, const uint16_t* D21,
                       const int64_t* p1, int64_t* p1_new, int b, int h, int w,
                       int n, int fdim, int radius, int dilation_max,
                       void* stream);

/* Tuning hooks (not on the product path): lanes per query point of the
 * refine (1, 2, 4: per-lane kernel for radius 3 / fdim 24; 3 = default:
 * pixel-major kernel for radius 3 / fdim 24, three lanes per window pixel;
 * 8, 16, 32, 64: cooperative kernel, 16 of them also for every other
 * radius / fdim) and
 * the per-lane kernel's load distance in candidates (2, 3, 4 = default, 6);
 * results identical for every setting.  s3m_refine_set_sort: visit the
 * queries in the order of the 2^sx x 2^sy pixel tile holding their window
 * centre (mode = 16 sx + sy, sx, sy <= 6; 0 = pixel order).  An
 * out-of-range value (e.g. -1) restores the default. */
void s3m_refine_set_lanes(int lanes);
void s3m_refine_set_prefetch(int pf);
void s3m_refine_set_sort(int mode);

/* Fused prep_for_iter_proj (matching.py:25-49 + image.py:5-38):
 * rays = normalize(X11); rays_with_grad = [rays, Scharr_x(rays)/32,
 * Scharr_y(rays)/32] with reflect padding; pts = normalize(X21);
 * p_init = lin_to_pixel(idx_init) or identity when idx_init == NULL. */
int s3m_prep_iter_proj(const float* X11, const float* X21,
                       const int64_t* idx_init, float* rays_with_grad,
                       float* pts_norm, float* p_init, int b, int h, int w,
                       void* stream);

/* Occlusion test + cast (matching.py:68-76): p1 = long(p),
 * valid = converged && ||X11[p1] - X21|| < dist_thresh. */
int s3m_occlusion(const float* p, const uint8_t* converged, const float* X11,
                  const float* X21, int64_t* p1, uint8_t* valid, int b, int h,
                  int w, float dist_thresh, void* stream);

/* pixel_to_lin (matching.py:13-15): idx = u + w*v. */
int s3m_pixel_to_lin(const int64_t* p1, int64_t* idx, int64_t count, int w,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3M_H */
