/*
 * gsr.h — tile-binned 3D Gaussian splat rasterizer (replaces the CUDA
 * extension of the external module `diff_gaussian_rasterization`,
 * thirdparty/diff-gaussian-rasterization-modified, .gitmodules:10-12; empty
 * and unpinned in the reference snapshot).
 *
 * Python surface replaced (kept identical by splatt3r-slam_amd/
 * diff_gaussian_rasterization/__init__.py): GaussianRasterizationSettings /
 * GaussianRasterizer as called at
 *   splatt3r_core/src/pixelsplat_src/cuda_splatting.py:100-125 (per-frame render)
 *   splatt3r_slam/visualization.py:563-594               (full-map render)
 * The algorithm is the canonical graphdeco-inria 3DGS forward/backward
 * (EWA splatting, 16x16 tiles, (tile, depth) ordering, front-to-back alpha
 * blending with early termination); see DESIGN.md "Rasterizer".
 *
 * Calling sequence (all on one stream, caller-allocated buffers):
 *   gsr_geom_bytes(P)        -> geom workspace   (per Gaussian)
 *   gsr_image_bytes(H, W)    -> image workspace  (per pixel / tile)
 *   gsr_preprocess(...)      -> radii, geom; writes num_rendered to *host*
 *                               (synchronises the stream once)
 *   gsr_binning_bytes(R)     -> binning workspace (per tile-instance)
 *   gsr_render(...)          -> out_color [3,H,W]
 *   gsr_backward(...)        -> gradients (optional)
 * The three workspaces are opaque and must be kept alive from preprocess to
 * backward (the Python layer stores them as uint8 tensors, like the
 * reference's geomBuffer / binningBuffer / imgBuffer).
 */
#ifndef GSR_H
#define GSR_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int image_height;
  int image_width;
  float tanfovx;
  float tanfovy;
  float scale_modifier;
  int sh_degree;        /* D: active SH degree (0..3) */
  int prefiltered;
  int debug;
  const float* bg;          /* device [3]                                   */
  const float* viewmatrix;  /* device [16], memory of the torch [4,4] arg    */
  const float* projmatrix;  /* device [16], full projection (view @ proj)    */
  const float* campos;      /* device [3]                                    */
} gsr_settings;

size_t gsr_geom_bytes(int64_t P);
size_t gsr_image_bytes(int height, int width);
size_t gsr_binning_bytes(int64_t num_rendered);

/* Preprocess: cull, EWA 2-D covariance, conic, radius, SH->RGB (or
 * colors_precomp), tile rectangle, inclusive scan of tiles touched.
 * Exactly one of shs / colors_precomp and exactly one of
 * (scales, rotations) / cov3D_precomp must be non-NULL.  M = number of SH
 * coefficients per Gaussian (shs is [P, M, 3]). */
int gsr_preprocess(const gsr_settings* s, int64_t P, int M, const float* means3D,
                   const float* scales, const float* rotations,
                   const float* cov3D_precomp, const float* shs,
                   const float* colors_precomp, const float* opacities,
                   int32_t* radii, void* geom, int64_t* num_rendered,
                   void* stream);

/* Binning (duplicate with (tile, depth) keys, radix sort, tile ranges) and
 * front-to-back alpha blending into out_color [3, H, W]. */
int gsr_render(const gsr_settings* s, int64_t P, int64_t num_rendered,
               const int32_t* radii, void* geom, void* binning, void* image,
               float* out_color, void* stream);

/* Sync-free forward (preprocess + binning + blend with no host read):
 * the instance count and depth-key range stay on the device.  The binning
 * workspace holds gsr_binning_bytes(capacity) and the depth sort runs over
 * key_bits bits.  info (device int64[3]) receives {status, num_rendered,
 * live key bits}: status 0 = out_color is the frame (bit-identical to
 * gsr_preprocess + gsr_render); bit 0 = more instances than capacity, bit 1
 * = a depth-key range wider than key_bits -- the image is then not valid and
 * the caller re-renders with the two-call protocol (sizing the next frame
 * from info).  For callers that consume the image later than it is produced
 * (the SLAM frame loop: splatt3r_amd/slam.py), so the stream never waits on
 * the host.  No backward from this path. */
int gsr_forward_deferred(const gsr_settings* s, int64_t P, int M, const float* means3D,
                         const float* scales, const float* rotations,
                         const float* cov3D_precomp, const float* shs,
                         const float* colors_precomp, const float* opacities,
                         int32_t* radii, void* geom, void* binning, int64_t capacity,
                         int key_bits, void* image, float* out_color, int64_t* info,
                         void* stream);

/* Backward.  Outputs (caller-zeroed not required; every output is written):
 *   dL_dmeans2D [P,3] (x,y used), dL_dconic [P,4] (scratch),
 *   dL_dopacity [P,1], dL_dcolors [P,3], dL_dmeans3D [P,3],
 *   dL_dcov3D [P,6], dL_dsh [P,M,3] (may be NULL when shs == NULL),
 *   dL_dscales [P,3], dL_drotations [P,4] (may be NULL when scales == NULL). */
int gsr_backward(const gsr_settings* s, int64_t P, int M, int64_t num_rendered,
                 const float* means3D, const float* scales, const float* rotations,
                 const float* cov3D_precomp, const float* shs,
                 const float* colors_precomp, const float* opacities,
                 const int32_t* radii, const void* geom, const void* binning,
                 const void* image, const float* dL_dout_color, float* dL_dmeans2D,
                 float* dL_dconic, float* dL_dopacity, float* dL_dcolors,
                 float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                 float* dL_dscales, float* dL_drotations, void* stream);

/* GaussianRasterizer.markVisible: present[i] = (view z > 0.2). */
int gsr_mark_visible(int64_t P, const float* means3D, const float* viewmatrix,
                     const float* projmatrix, uint8_t* present, void* stream);

/* Instrumentation for bench.py: per-phase device time (ms) of the last
 * gsr_preprocess + gsr_render on the calling thread, measured with HIP
 * events on the caller's stream when enabled.  phases[0..4] =
 * preprocess, (reduce, fused: ~0), depth sort (per-tile binning: tile
 * counts + scan), binning (per-tile: fill + per-tile sort), blend. */
void gsr_set_timing(int enabled);
int gsr_last_timing(float* phases_ms, int n);

/* Forward binning (A/B hook, not on the product path): 0 = global depth
 * sort + tile sort (the default), 1 = per-tile binning (instances binned by
 * tile in Gaussian order, each tile's list depth-sorted in LDS; slower at
 * C3).  Identical output; any other value restores the default. */
void gsr_set_binning(int mode);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */
