/*
 * s3lie.h — Sim3 / SE3 group operations (replaces the CUDA kernels of the
 * external `lietorch` module, github.com/princeton-vl/lietorch, unpinned
 * submodule thirdparty/lietorch, .gitmodules:7-9).
 *
 * Layouts (lietorch convention, splatt3r_slam/splatt3r_utils.py:160,
 * splatt3r_slam/lietorch_utils.py:10-12):
 *   Sim3 element  = float[8]  {tx, ty, tz, qx, qy, qz, qw, s}
 *   SE3  element  = float[7]  {tx, ty, tz, qx, qy, qz, qw}
 *   Sim3 tangent  = float[7]  {tau(3), phi(3), sigma}
 *
 * Math is restated from the in-repo device code
 * splatt3r_slam/backend/src/gn_kernels.cu:177-412 (quat_comp, actSO3,
 * actSim3, expSO3, expSim3, retrSim3).  All arrays are contiguous; the
 * host wrapper broadcasts.  `n_a == 1` broadcasts a single group element
 * over `n` items where documented.
 */
#ifndef S3LIE_H
#define S3LIE_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* out[i] = a[i or 0] * b[i or 0]  (lietorch Sim3.__mul__, used at
 * tracker.py:180,212,225,264).  n_a, n_b in {1, n}. */
int s3lie_sim3_mul(const float* a, int64_t n_a, const float* b, int64_t n_b,
                   float* out, int64_t n, void* stream);

/* out[i] = a[i]^-1  (lietorch Sim3.inv, tracker.py:180). */
int s3lie_sim3_inv(const float* a, float* out, int64_t n, void* stream);

/* Y[i] = T[i or 0] . X[i] = s R X + t  (lietorch Sim3.act, geometry.py:46,
 * tracker.py:98; gn_kernels.cu:211-224 actSim3). n_T in {1, n}. */
int s3lie_sim3_act(const float* T, int64_t n_T, const float* X, float* Y,
                   int64_t n, void* stream);

/* out[i] = Exp(xi[i])  (gn_kernels.cu:319-391 expSim3). */
int s3lie_sim3_exp(const float* xi, float* out, int64_t n, void* stream);

/* xi[i] = Log(T[i])  (lietorch Sim3::Log; inverse of s3lie_sim3_exp). */
int s3lie_sim3_log(const float* T, float* xi, int64_t n, void* stream);

/* out[i] = Exp(xi[i or 0]) * T[i or 0]  (lietorch retr = left retraction,
 * tracker.py:195,247; gn_kernels.cu:393-412 retrSim3). */
int s3lie_sim3_retr(const float* T, int64_t n_T, const float* xi, int64_t n_xi,
                    float* out, int64_t n, void* stream);

/* M[i] = 4x4 row-major [sR t; 0 1] (splatt3r_utils.py:153-165 _sim3_to_4x4). */
int s3lie_sim3_matrix(const float* T, float* M, int64_t n, void* stream);

/* M[i] = 4x4 row-major [R t; 0 1] (lietorch SE3.matrix, main.py:70-71). */
int s3lie_se3_matrix(const float* T, float* M, int64_t n, void* stream);

/* In-place pose_retr_kernel (gn_kernels.cu:414-452): for k in [num_fix,N):
 * poses[k] = Exp(dx[k-num_fix]) * poses[k]. */
int s3lie_pose_retr(float* poses, const float* dx, int64_t num_poses,
                    int64_t num_fix, void* stream);

/* Host (CPU) versions of the single-pose ops used inside the host-driven
 * tracker loop (tracker.py:173-214), so that the per-iteration retraction
 * needs no device round trip.  Same math as the device functions. */
void s3lie_sim3_retr_host(const float T[8], const float xi[7], float out[8]);
void s3lie_sim3_mul_host(const float a[8], const float b[8], float out[8]);
void s3lie_sim3_inv_host(const float a[8], float out[8]);

#ifdef __cplusplus
}
#endif
#endif /* S3LIE_H */
