/*
 * s3t.h — tracker Gauss-Newton step on the GPU (the per-iteration work of
 * FrameTracker.opt_pose_ray_dist_sim3, splatt3r_slam/tracker.py:173-214,
 * and FrameTracker.solve :156-171).
 *
 * One launch per GN iteration computes, for every correspondence i,
 *   p  = T . Xf_i                          (geometry.act_Sim3, :45-52)
 *   rd = (p/|p|, |p|), drd/dp              (geometry.point_to_ray_dist, :17-34)
 *   r  = rd(Xk_i) - rd(p),  J = -drd/dp [I, -[p]x, p]
 *   w  = sqrt_info * sqrt(huber(sqrt_info * r, k))   (nonlinear_optimizer.py:28-33)
 *   A  = w J,  b = w r
 * and reduces H = sum A^T A (upper triangle, 28), g = -sum A^T b (7),
 * cost = 0.5 sum b^T b into out[36] = {H_upper(28, row-major), g(7), cost}.
 * sqrt_info = (1/sigma_ray, x3; 1/sigma_dist) * valid_i * sqrt(Q_i).
 * The pose T (Sim3, t q s) is read from device memory, so the first
 * iteration can be queued before the host knows the pose (the host loop
 * uploads later poses asynchronously, stream-ordered).
 */
#ifndef S3T_H
#define S3T_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Workspace bytes for n correspondences (block partials). */
size_t s3t_workspace_bytes(int64_t n);

int s3t_ray_dist_normal_eqs(const float* T /* device [8] */, const float* Xf, const float* Xk,
                            const float* Q, const uint8_t* valid, int64_t n,
                            float sigma_ray, float sigma_dist, float huber_k,
                            void* workspace, float* out36, void* stream);

/* Queue `iters` complete GN iterations on the stream with no host round
 * trip: normal equations at the device pose T, then a one-thread fp64
 * Cholesky solve, T <- Exp(tau) * T (lietorch retr) and the reference's
 * convergence test (rel cost decrease < rel_error or |tau| < delta_norm).
 * state (device double[4]): [0] previous cost (init +inf), [1] iterations
 * done (init 0), [2] flag (init 0; 1 converged, 2 Cholesky failed,
 * 3 max_iters reached), [3] last cost.  Once the flag is set every queued
 * kernel returns immediately, so the host queues iterations in chunks and
 * reads `state` once per chunk. */
int s3t_gn_iterations(const float* Xf, const float* Xk, const float* Q, const uint8_t* valid,
                      int64_t n, float sigma_ray, float sigma_dist, float huber_k, int iters,
                      int max_iters, float rel_error, float delta_norm, float* T /* device [8] */,
                      double* state, void* workspace, float* out36, void* stream);

/* Calibrated tracker (FrameTracker.opt_pose_calib_sim3, tracker.py:216-270;
 * residuals of geometry.project_calib :63-104).  Per keyframe pixel i
 * (n = h*w, pixel (i % w, i / w)):
 *   p = T . Xf_i,  pz = (K p).xy / (K p).z, log p.z   (log z := 0 if z <= depth_eps)
 *   meas = (i % w, i / w, log Xk_i.z), zeroed where Xk_i.z <= depth_eps
 *   r = meas - pz,  J = -dpz/dp [I, -[p]x, p]
 *   sqrt_info = (1/sigma_pixel x2, 1/sigma_depth) * valid_i * sqrt(Q_i)
 *               * [border < u < w-1-border, border < v < h-1-border,
 *                  p.z > depth_eps, Xk_i.z > depth_eps]
 * Xf is the ray-constrained frame pointmap gathered by idx_f2k, Xk the
 * keyframe pointmap (only its z is read).  K is a HOST float[9] (row-major
 * 3x3).  Output layout and the device GN loop are those of the ray variant
 * above. */
int s3t_calib_normal_eqs(const float* T /* device [8] */, const float* Xf, const float* Xk,
                         const float* Q, const uint8_t* valid, int64_t n, const float* K,
                         int h, int w, float pixel_border, float depth_eps, float sigma_pixel,
                         float sigma_depth, float huber_k, void* workspace, float* out36,
                         void* stream);

int s3t_gn_iterations_calib(const float* Xf, const float* Xk, const float* Q,
                            const uint8_t* valid, int64_t n, const float* K, int h, int w,
                            float pixel_border, float depth_eps, float sigma_pixel,
                            float sigma_depth, float huber_k, int iters, int max_iters,
                            float rel_error, float delta_norm, float* T /* device [8] */,
                            double* state, void* workspace, float* out36, void* stream);

/* The per-frame correspondence filter of FrameTracker.track (tracker.py:
 * 28-91) in one pass over the n frame pixels i (match j = idx[i] in the
 * keyframe):
 *   Xf_out[i] = Xf[j];  Q_out[i] = sqrt(Qff[j] * Qkf[i]);
 *   valid_opt[i] = vm[i] && Cf[j] > C_conf && Ck[i] > C_conf && Q_out[i] > Q_conf;
 *   counts[0] += valid_opt[i];  counts[1] += vm[i] && Q_out[i] > Q_conf;
 *   counts[2] = |{ j : some i with vm[i] has idx[i] == j }| (unique hits).
 * Xf [n,3], Cf / Ck / Qff / Qkf [n] fp32; idx int64 [n]; vm / valid_opt
 * bool bytes [n]; hit: uint32 [n + 192] scratch (zeroed here, inside the
 * stream); counts int64 [3] (written here).  Exact (same fp32 ops as the
 * reference). */
int s3t_track_prep(const int64_t* idx, const uint8_t* vm, const float* Xf, const float* Cf,
                   const float* Ck, const float* Qff, const float* Qkf, int64_t n, float C_conf,
                   float Q_conf, float* Xf_out, float* Q_out, uint8_t* valid_opt,
                   uint32_t* hit, int64_t* counts, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3T_H */
