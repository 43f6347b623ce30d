/*
 * s3q.h — keyframe retrieval features and codebook quantisation (SURVEY §8(f)
 * f3), the device half of splatt3r_slam/retrieval_database.py:
 *
 *   RetrievalDatabase.prep_features  retrieval_database.py:24-41
 *     prewhiten  Whitener.forward    mast3r/retrieval/model.py:55-75 (fp64)
 *     projector  nn.Linear(1024,1024) model.py:143-156 (+ residual)
 *     attention  ||proj_feat||_2     model.py:133-134 ('l2norm')
 *     postwhiten Whitener.forward    (fp64)
 *     how_select_local top-nfeat     model.py:89-103
 *   RetrievalDatabase.quantize_custom retrieval_database.py:95-104
 *     |q|^2 + |c|^2 - 2 q c^T, topk(k, largest=False)
 *
 * The ASMK inverted file (aggregate / search, third-party `asmk`, CPU) is
 * not part of this ABI.  All pointers are device pointers; calls are async
 * on `stream`.
 */
#ifndef S3Q_H
#define S3Q_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Whitener.forward: out[M, N] (f32) = ((x - m) @ P) evaluated in fp64,
 * x [M, K] f32, m [K] f64 (NULL = no centring), P [K, N] f64 row-major. */
int s3q_whiten(const float* x, const double* m, const double* P, float* out, int M, int K, int N,
               void* stream);

/* nn.Linear (+ optional residual): out[M, N] = x @ W^T + b (+ x if
 * residual, N == K), fp32 accumulate; W [N, K] f32, b [N] f32 or NULL. */
int s3q_linear(const float* x, const float* W, const float* b, float* out, int M, int K, int N,
               int residual, void* stream);

/* how_select_local with attention = ||attn_src row||_2: per image b, the
 * nfeat tokens of largest attention (descending; equal values keep the
 * lower token index first) -> feat_out [B, nfeat, D] rows of feat,
 * attn_out [B, nfeat] f32, idx_out [B, nfeat] i64.  T <= 4096. */
int s3q_select_local(const float* attn_src, const float* feat, int B, int T, int D, int nfeat,
                     float* feat_out, float* attn_out, int64_t* idx_out, void* stream);

/* Row squared norms: out[r] = sum_k x[r, k]^2 (fp32). */
int s3q_row_sqnorm(const float* x, int R, int D, float* out, void* stream);

/* quantize_custom: for every query row, the k centroids of smallest
 * l2 = |q|^2 + |c|^2 - 2 q.c (fp32, k <= 8), ascending; ties keep the lower
 * centroid index.  q [M, D], c [C, D], c_sqnorm [C] (s3q_row_sqnorm of c),
 * idx_out [M, k] i64, dist_out [M, k] f32 (NULL = not written).
 * workspace: s3q_l2_topk_workspace_bytes(M, C, k) bytes. */
size_t s3q_l2_topk_workspace_bytes(int M, int C, int k);
int s3q_l2_topk(const float* q, const float* c, const float* c_sqnorm, int M, int C, int D, int k,
                int64_t* idx_out, float* dist_out, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3Q_H */
