/*
 * s3r.h — fused splat packing for the per-frame render
 * (splatt3r_slam/splatt3r_utils.py:332-432 splatt3r_render ->
 *  decoder_splatting_cuda.py:30-83 -> cuda_splatting.py:48-128).
 *
 * One pass per view replaces: build_covariance (utils/geometry.py:52-62,
 * quaternion_to_matrix :24-49, xyzw order, two_s = 2/(|q|^2+1e-8)), the SH
 * residual sh[...,0] += RGB2SH(img) (utils/sh_utils.py:114-115,
 * C0 = 0.28209479177387814), the scale-invariant rescale (means * s,
 * cov * s^2, cuda_splatting.py:67-76) and the triu(cov) / SH rearrange
 * (cuda_splatting.py:86,121-124).
 */
#ifndef S3R_H
#define S3R_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Inputs for n splats of one view:
 *   means [n,3], scales [n,3], rotations [n,4] (xyzw), sh [n,3,d_sh]
 *   (network residual, d_sh == 1 supported), opacities [n,1],
 *   img: if img_chw_normalized, [3, n] in ImgNorm space ((x-0.5)/0.5, the
 *   frame.img layout) converted with clamp(x*0.5+0.5, 0, 1); else [n,3] in
 *   [0,1].
 * Outputs: means_out [n,3], cov6_out [n,6] (xx,xy,xz,yy,yz,zz), shs_out
 *   [n,1,3], opac_out [n,1]. */
int s3r_pack_splats(const float* means, const float* scales, const float* rotations,
                    const float* sh, const float* opacities, const float* img,
                    int64_t n, int d_sh, float scale, int img_chw_normalized,
                    float* means_out, float* cov6_out, float* shs_out,
                    float* opac_out, void* stream);

/* The pose-dependent camera of one render (decoder_splatting_cuda.py:36-55
 * + cuda_splatting.py:67-113 for a single target view), in fp64 on the
 * device in one thread instead of two 4x4 inverses and two matmuls:
 *   Mc = matrix(T_context), Mt = matrix(T_target)    (lietorch Sim3 [8])
 *   extr = Mc^-1 Mt, extr[:3,3] *= scale
 *   view = (extr^-1)^T, full = view @ proj_t, campos = extr[:3,3]
 * proj_t is the transposed projection matrix [16] (row-major, device).
 * Outputs (device, fp32, row-major): view [16], full [16], campos [3]. */
int s3r_camera(const float* T_context, const float* T_target, const float* proj_t, float scale,
               float* view, float* full, float* campos, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3R_H */
