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
 *   ASMK inverted file (RetrievalDatabase.update / query / add_to_ivf_custom,
 *   retrieval_database.py:43-134; the third-party `asmk` package, absent
 *   here, restated from its published algorithm: Tolias et al., ICCV'13,
 *   binary ASMK*, with Retriever's asmk_params, processor.py:84-89):
 *     aggregate  per visual word: sum of residuals (x - c_w) over the
 *                descriptors assigned to w, binarised to sign bits
 *     search     score(image) = sum over shared words of
 *                max(0, 1 - 2 hamming / D)^alpha   (alpha = 3, threshold 0)
 *
 * All pointers are device pointers; calls are async on `stream`.
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

/* ASMK aggregate_image, binary: feats [n, D] f32, words [n, k] i64 (the
 * quantize_custom indices; a descriptor is in word w's set when any of its
 * k assignments is w).  Unique words ascending -> out_words [n*k] i32
 * (first *out_count valid), out_codes [n*k, D/32] u32 with bit (d % 32) of
 * word d / 32 = (sum_x (x_d - c_wd) > 0), the sum of fp32 differences
 * accumulated in fp64.  n * k <= 4096, D % 32 == 0, D <= 4096. */
size_t s3q_asmk_aggregate_workspace_bytes(int n, int k);
int s3q_asmk_aggregate(const float* feats, const int64_t* words, const float* centroids, int n,
                       int k, int D, int32_t* out_words, uint32_t* out_codes, int32_t* out_count,
                       void* workspace, void* stream);

/* ASMK search over a flat inverted file of n_db entries (word, image, code):
 * for every entry whose word is among the query's *q_count aggregated words,
 * s = D - 2 hamming(code, q_code); when s / D >= sim_threshold, s^alpha is
 * added to scores[image] (int64, exact and order-independent; the score is
 * scores / D^alpha).  word_slot: [n_words] i32 scratch, all -1 on entry and
 * on return.  alpha in 1..3, q_max bounds *q_count. */
int s3q_asmk_search(const int32_t* q_words, const uint32_t* q_codes, const int32_t* q_count,
                    int q_max, const int32_t* db_words, const int32_t* db_images,
                    const uint32_t* db_codes, int64_t n_db, int D, int alpha,
                    float sim_threshold, int32_t* word_slot, int n_words,
                    unsigned long long* scores, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3Q_H */
