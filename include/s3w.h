/*
 * s3w.h — camera-space Gaussian predictions -> filtered world-space records
 * (SURVEY §8 A11 / §8(f) f2).
 *
 * Replaces the torch body of gaussians_to_world
 * (splatt3r_slam/splatt3r_utils.py:180-328) for one predicted view:
 *   stride-s subsample (:259-270), RGB2SH residual on the DC band (:277-281,
 *   utils/sh_utils.py:114-115), the three splash filters (:296-312):
 *     z > depth_min, z <= quantile(z[z > depth_min], q) (torch.quantile,
 *     linear interpolation), max(scale) < max_scale, conf >= min_confidence,
 *   then means_w = M x + t, cov_w = M (R S S^T R^T) M^T (build_covariance,
 *   utils/geometry.py:24-62) packed triu (xx,xy,xz,yy,yz,zz), colour =
 *   clamp(sh0 * C0 + 0.5, 0, 1), opacity.  M = s R of the Sim3 T_WC.
 * Output records keep the reference's order (row-major over the strided
 * grid, the order of torch boolean indexing): out[k] = 13 floats
 *   {means_w[3], cov_triu[6], colour[3], opacity}.
 */
#ifndef S3W_H
#define S3W_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  const float* means;      /* [H, W, 3] camera space */
  const float* scales;     /* [H, W, 3] */
  const float* rotations;  /* [H, W, 4] xyzw */
  const float* sh;         /* [H, W, 3, d_sh] (DC = index 0) */
  const float* opacities;  /* [H, W] */
  const float* conf;       /* [H, W] or NULL (no confidence filter) */
  const float* img;        /* [3, H, W] ImgNorm-normalised frame image */
  int H, W, d_sh, stride;
} s3w_view;

/* Workspace for n = ceil(H/stride) * ceil(W/stride) Gaussians. */
size_t s3w_workspace_bytes(int64_t n);

/* T_WC: device float[16], the row-major 4x4 [s R | t; 0 0 0 1] (as
 * lietorch Sim3.matrix() returns it).  depth_max_percentile
 * >= 1 disables the quantile bound, min_confidence <= 0 the confidence
 * filter.  out: [n, 13] device; *count_dev (device int64) receives the
 * number of records written.  Stream-ordered, no host sync. */
int s3w_gaussians_to_world(const s3w_view* v, const float* T_WC, float depth_min,
                           float depth_max_percentile, float max_scale, float min_confidence,
                           void* workspace, float* out, int64_t* count_dev, void* stream);

/* Testing hook: 0 = automatic (two launches, a one-workgroup select and a
 * chip-wide emit, when n <= 30720; else sort + scan passes), 1 = always the
 * multi-pass path, 2 = the two-launch path whenever n fits.  Both paths give
 * identical records and counts. */
void s3w_set_path(int path);

/* ---- SharedGaussians map buffer (splatt3r_slam/frame.py:357-463) ----
 * Structure-of-arrays world map with a device-side count, so appends are
 * stream-ordered with no host sync.  Replaces SharedGaussians.append /
 * get_all / clear; the viz full-map render (visualization.py:467-600)
 * rasterizes means/cov_triu/colors/opacities[:n] with colors_precomp. */
typedef struct {
  float* means;       /* [cap, 3] world centres      */
  float* cov_triu;    /* [cap, 6] xx xy xz yy yz zz  */
  float* colors;      /* [cap, 3] RGB                */
  float* opacities;   /* [cap]                       */
  int32_t* kf_id;     /* [cap] source keyframe       */
  int64_t* n;         /* device: live Gaussians      */
  int64_t cap;        /* max_gaussians               */
} s3w_map;

size_t s3w_map_append_workspace_bytes(int64_t n_max);

/* SharedGaussians.append(means, cov_triu, colors, opacities, kf_idx,
 * opacity_threshold) on the world records of s3w_gaussians_to_world
 * (records [n_max, 13], *count_dev valid): keep opacity > threshold in
 * record order; if the map is full (n == cap) first move the newest half
 * to the front (FIFO eviction of the oldest half, frame.py:423-437), then
 * append min(kept, cap - n) records with kf_id = kf_idx. */
int s3w_map_append(const s3w_map* map, const float* records, const int64_t* count_dev,
                   int64_t n_max, float opacity_threshold, int32_t kf_idx, void* workspace,
                   void* stream);

/* Scale-invariant copies for the full-map render (visualization.py:534-585):
 * means_out = means * s, cov_out = cov_triu * s2 for i < *n_dev (n_max
 * bounds the launch). */
int s3w_map_scale(const float* means, const float* cov_triu, const int64_t* n_dev, int64_t n_max,
                  float s, float s2, float* means_out, float* cov_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3W_H */
