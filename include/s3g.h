/*
 * s3g.h — backend pose-graph Gauss-Newton on rays (replaces
 * mast3r_slam_backends.gauss_newton_rays: splatt3r_slam/backend/src/gn.cpp:28-52
 * -> gn_kernels.cu:1139-1227 gauss_newton_rays_cuda, ray_align_kernel
 * :812-1137, pose_retr_kernel :414-454, SparseBlock :56-158; caller
 * splatt3r_slam/global_opt.py:121-158 FactorGraph.solve_GN_rays).
 *
 * Poses Twc [n_poses, 8] (t, q xyzw, s) are the keyframes of the graph in
 * the caller's unique-index order; ii/jj [n_edges] are LOCAL pose indices
 * (the reference's searchsorted(unique_kf_idx, ii)); the first num_fix poses
 * are held fixed (the reference hard-codes 1).  Per edge e: Xs[ii_e] /
 * Cs[ii_e] are indexed through idx_ii2jj[e, k] where valid_match[e, k],
 * against point k of Xs[jj_e].
 *
 * Everything stays on the device: per-edge residuals/Jacobians/H blocks are
 * reduced by (edge x point-slice) workgroups in a fixed order, the dense
 * 7(n_poses - num_fix) system is assembled in fp64, solved by an fp64
 * Cholesky (dx = 0 if it fails, as the reference's SimplicialLLT branch),
 * and the poses are retracted; iterations stop on the device once
 * ||dx|| < delta_thresh.  The host reads nothing until the call returns.
 */
#ifndef S3G_H
#define S3G_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device workspace bytes for one solve. */
size_t s3g_workspace_bytes(int n_poses, int n_edges, int64_t n_points, int num_fix);

/* The dense normal equations at the current poses (one iteration's linear
 * system, no solve): H [n x n] fp64 row-major, b [n] fp64, n = 7(n_poses -
 * num_fix).  b is the gradient (the reference's gs), the step is -H^-1 b. */
int s3g_ray_system(const float* Twc, int n_poses, const float* Xs, const float* Cs,
                   int64_t n_points, const int32_t* ii, const int32_t* jj, int n_edges,
                   const int64_t* idx_ii2jj, const uint8_t* valid_match, const float* Q,
                   float sigma_ray, float sigma_dist, float C_thresh, float Q_thresh,
                   int num_fix, void* workspace, double* H, double* b, void* stream);

/* The full solve: updates Twc in place, writes the last step dx
 * [n_poses - num_fix, 7] and stats[2] = {iterations run, |dx| of the last}. */
int s3g_gauss_newton_rays(float* Twc, int n_poses, const float* Xs, const float* Cs,
                          int64_t n_points, const int32_t* ii, const int32_t* jj, int n_edges,
                          const int64_t* idx_ii2jj, const uint8_t* valid_match, const float* Q,
                          float sigma_ray, float sigma_dist, float C_thresh, float Q_thresh,
                          int max_iter, float delta_thresh, int num_fix, void* workspace,
                          float* dx, float* stats, void* stream);

/* Calibrated variant (replaces mast3r_slam_backends.gauss_newton_calib:
 * gn.cpp:54-80 -> gn_kernels.cu:1545-1637 gauss_newton_calib_cuda,
 * calib_proj_kernel :1230-1542; caller global_opt.py:160-215
 * FactorGraph.solve_GN_calib).  Residuals per correspondence: projected
 * pixel (u, v) of T_ij X_j under K minus the matched pixel (idx % width,
 * idx / width), and log z_j - log z_i; valid only inside pixel_border and
 * with both depths > z_eps.  K: DEVICE pointer to the 3x3 row-major
 * intrinsics (the reference reads K[0][0], K[1][1], K[0][2], K[1][2] on the
 * device).  n_points must equal height * width.  Same workspace
 * (s3g_workspace_bytes), outputs and stop rule as the rays solve. */
int s3g_calib_system(const float* Twc, int n_poses, const float* Xs, const float* Cs,
                     int64_t n_points, const float* K, const int32_t* ii, const int32_t* jj,
                     int n_edges, const int64_t* idx_ii2jj, const uint8_t* valid_match,
                     const float* Q, int height, int width, int pixel_border, float z_eps,
                     float sigma_pixel, float sigma_depth, float C_thresh, float Q_thresh,
                     int num_fix, void* workspace, double* H, double* b, void* stream);

int s3g_gauss_newton_calib(float* Twc, int n_poses, const float* Xs, const float* Cs,
                           int64_t n_points, const float* K, const int32_t* ii, const int32_t* jj,
                           int n_edges, const int64_t* idx_ii2jj, const uint8_t* valid_match,
                           const float* Q, int height, int width, int pixel_border, float z_eps,
                           float sigma_pixel, float sigma_depth, float C_thresh, float Q_thresh,
                           int max_iter, float delta_thresh, int num_fix, void* workspace,
                           float* dx, float* stats, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3G_H */
