/*
 * s3n.h — MASt3RGaussians network kernels (ViT-L encoder, Base decoder,
 * DPT-Gaussian heads) for gfx950 MFMA.
 *
 * Replaces the torch/cuBLAS/cuDNN execution of
 *   splatt3r_core/src/mast3r_src/dust3r/dust3r/model.py:121-193
 *   (_encode_image, _decoder, _downstream_head),
 *   croco/models/blocks.py:58-191 (Mlp, Attention, Block, CrossAttention,
 *   DecoderBlock), croco/models/pos_embed.py:106-159 (RoPE2D) ==
 *   croco/models/curope/kernels.cu:18-82, croco/models/dpt_block.py
 *   (DPT adapter), mast3r/catmlp_dpt_head.py:140-278 (GaussianHead,
 *   gaussian_postprocess), dust3r/heads/postprocess.py:22-58.
 * The Python model object behind the reference API
 * (model.encoder._encode_image / _decoder / _downstream_head) lives in
 * splatt3r-slam_amd/splatt3r_amd/net.py and drives these entry points.
 *
 * Data types: activations entering a matrix product are fp16 (10-bit
 * mantissa, the TF32 class of the reference's matmuls); every product
 * accumulates in fp32 on MFMA; the transformer residual stream and every
 * head output are fp32.
 * "groups" batch up to 4 independent problems of identical shape with
 * different pointers in one launch (decoder branch 1/2, heads 1/2, the four
 * DPTs), i.e. a grouped GEMM.
 */
#ifndef S3N_H
#define S3N_H
#include "s3_common.h"

#ifdef __cplusplus
extern "C" {
#endif

#define S3N_MAX_GROUPS 4

enum { S3N_ACT_NONE = 0, S3N_ACT_GELU = 1, S3N_ACT_RELU = 2 };
enum { S3N_STORE_PLAIN = 0, S3N_STORE_CONVT = 1, S3N_STORE_PIXSHUF = 2 };
enum { S3N_A_DENSE = 0, S3N_A_CONV = 1 };

/* C[M,N] = epilogue( A[M,K] . B[N,K]^T ).
 * A: fp16, dense row-major (lda) or an implicit im2col of an NHWC fp16
 *    image (a_mode = S3N_A_CONV: k = (ky*ks + kx)*Cin + ci, zero padding,
 *    optional ReLU applied to the loaded input).
 * B: fp16 weights [N, K] row-major (ldb), i.e. nn.Linear layout / conv
 *    weight permuted to [Cout, ky, kx, Cin].
 * Epilogue: + bias[N] (fp32) -> act -> + R1 -> + R2 -> store C (fp32 or
 *    fp16, row-major ldc, or scattered: CONVT = ConvTranspose2d(k=s)
 *    pixel scatter into NHWC [B, sH*s, sW*s, sCout] with n = (i*s+j)*sCout+co;
 *    PIXSHUF = transpose + F.pixel_shuffle(s) into NHWC [B, sH*s, sW*s, sCout]
 *    with n = co*s*s + i*s + j) and optionally a second fp16 copy C2 (ldc2). */
typedef struct {
  int M, N, K, groups;
  const void* A[S3N_MAX_GROUPS];
  int64_t lda;
  const void* B[S3N_MAX_GROUPS];
  int64_t ldb;
  const float* bias[S3N_MAX_GROUPS];
  const void* R1[S3N_MAX_GROUPS];
  int64_t ldr1;
  int r1_f16;
  const void* R2[S3N_MAX_GROUPS];
  int64_t ldr2;
  int r2_f16;
  void* C[S3N_MAX_GROUPS];
  int64_t ldc;
  int c_f16;
  void* C2[S3N_MAX_GROUPS];
  int64_t ldc2;
  int act;
  int store_mode;
  int a_mode;
  /* implicit conv (a_mode == S3N_A_CONV): input NHWC [Bn, cH, cW, cC] */
  int cH, cW, cC, ksize, stride, pad, oH, oW, relu_in;
  /* scatter stores: token grid sH x sW, factor s, output channels sCout */
  int sH, sW, sS, sCout;
  /* split-K: split_k > 1 partitions the K tiles over split_k workgroups per
   * output tile; fp32 partials go to `workspace` (s3n_gemm_workspace_bytes)
   * and a second launch sums them in split order (deterministic) and
   * applies the epilogue.  tile: 0 = auto, 1 = 64x64, 2 = 64x128,
   * 3 = 128x128 (4 waves), 4 = 256x128 (8 waves), 5 = 128x128 (8 waves). */
  int split_k;
  int tile;
  void* workspace;
  /* RoPE2D epilogue (pos_embed.py:142-159, head_dim 64): when rope_pos[g]
   * is set, output columns [0, rope_ncols) are treated as heads of 64 and
   * rotated after the bias, with row positions rope_pos[g][row] = (y, x)
   * (int64) and tables cos/sin [rope_maxpos, 16] (dims [0,32) of a head use
   * y, [32,64) use x; d pairs with d+16 inside each half).  Requires
   * split_k <= 1, rope_ncols % 64 == 0. */
  const float* rope_cos;
  const float* rope_sin;
  int rope_maxpos;
  int rope_ncols;
  const int64_t* rope_pos[S3N_MAX_GROUPS];
  /* Fused 1x1 tail (the DPT head's last conv, dpt_block.py:323): when
   * tail_w[g] is set, every finished, activated output row (all N columns:
   * N must equal the tile width, split_k <= 1) is multiplied by tail_w
   * [tail_n, N] fp16 and offset by tail_b [tail_n] into tail_out fp32
   * [M, ld_tail] (tail_n % 8 == 0, <= 16).  C[g] may then be NULL: the
   * N-wide activation never goes to memory. */
  const void* tail_w[S3N_MAX_GROUPS];
  const float* tail_b[S3N_MAX_GROUPS];
  float* tail_out[S3N_MAX_GROUPS];
  int tail_n;
  int64_t ld_tail;
  /* Optional fragment-packed copy of each group's B for the B-direct tiles
   * (70-77): Bp[nb][ks][lane][8] fp16 with nb = n / 16 (N padded to a
   * multiple of 16 with zeros), ks = k / 32, lane = 16 * ((k % 32) / 8) +
   * n % 16, element k % 8; dense A only, K % 32 == 0.  NULL: those tiles
   * are unavailable (the other tiles never read it). */
  const void* Bp[S3N_MAX_GROUPS];
} s3n_gemm_args;

size_t s3n_gemm_workspace_bytes(const s3n_gemm_args* args);
int s3n_gemm(const s3n_gemm_args* args, void* stream);

/* Tuning hook (not on the product path): flags applied to later s3n_gemm
 * launches; 1 = skip the MFMAs, 2 = skip the operand DMA, 4 = skip the
 * epilogue, 8 = skip the K loop (results are then garbage), 16 = force the
 * per-register epilogue instead of the LDS-staged vector one (results
 * valid).  0 restores normal operation. */
void s3n_gemm_set_debug(int flags);

/* Tuning hook (not on the product path): 1 = place tiles on the 8 XCDs by
 * the band split only (no 2-D partition of the tile grid); 0 = default.
 * Results are identical either way (only the tile -> workgroup map moves). */
void s3n_gemm_set_xcd_flags(int flags);

/* Fused multi-head attention softmax(Q K^T * scale) V with 2-D RoPE
 * (pos_embed.py:142-159, base 100, F0 1) applied to Q and K on load.
 * Q rows at Q + (b*Nq + n)*q_stride + h*64, K/V likewise; O rows at
 * O + (b*Nq + n)*o_stride + h*64 (fp16).  pos: int64 [B, N, 2] (y, x);
 * NULL disables RoPE.  cos/sin tables: [maxpos, 16] fp32 computed as the
 * reference computes them. head_dim is 64. */
typedef struct {
  int B, Nq, Nk, H, groups;
  const void* Q[S3N_MAX_GROUPS];
  const void* K[S3N_MAX_GROUPS];
  const void* V[S3N_MAX_GROUPS];
  int64_t q_stride, k_stride, v_stride;
  const int64_t* qpos[S3N_MAX_GROUPS];
  const int64_t* kpos[S3N_MAX_GROUPS];
  const float* rope_cos;
  const float* rope_sin;
  int rope_maxpos;
  void* O[S3N_MAX_GROUPS];
  int64_t o_stride;
  float scale;
} s3n_attn_args;

int s3n_attention(const s3n_attn_args* args, void* stream);

/* Tuning hook (not on the product path), kernels for pre-rotated q/k:
 * 0 = transposed-score kernel with 2 key groups (default), 1 = the
 * P-through-LDS kernel, 2 = transposed-score with 1 key group, 3 = with 4;
 * -1 / -2 = the transposed-score kernels' XCD-aware workgroup order off /
 * on (default on). */
void s3n_attention_set_variant(int variant);

/* LayerNorm over the last dim C (eps), per group gamma/beta:
 * y = (x - mean) * rsqrt(var + eps) * gamma + beta.  x fp32 [rows, ldx];
 * out16 (fp16, ld16) and/or out32 (fp32, ld32) may be NULL. */
int s3n_layernorm(int rows, int C, int groups, const float* const* x, int64_t ldx,
                  const float* const* gamma, const float* const* beta, float eps,
                  void* const* out16, int64_t ld16, float* const* out32, int64_t ld32,
                  void* stream);

/* Patch embedding im2col (patch_embed.py:42-70, landscape): image
 * [B,3,H,W] fp32 -> A [B*(H/p)*(W/p), 3*p*p] fp16, k = c*p*p + ky*p + kx. */
int s3n_patch_im2col(const float* img, int B, int H, int W, int p, void* A, void* stream);

/* Bilinear x2 upsample, align_corners=True (dpt_block.py:207-212,
 * Interpolate :262-270), NHWC fp16 -> NHWC fp16, per group.  The output
 * grid is the top-left crop [oh, ow] (oh <= 2H, ow <= 2W) of the 2H x 2W
 * result (refinenet4 crop, dpt_head.py:56). */
int s3n_upsample2x(int groups, const void* const* in, void* const* out, int B, int H, int W,
                   int C, int oh, int ow, void* stream);

/* gaussian_postprocess (catmlp_dpt_head.py:140-178) + the 43-channel
 * concatenation of GaussianHead.forward (:245-278) for one view:
 * pts [n, ld_pts] (4: xyz, conf), feat [n, 25] (desc 24, desc_conf),
 * gauss [n, ld_g] (14: offset 3, scales 3, rot 4, sh 3, opacity 1) ->
 * pts3d [n,3], conf [n], desc [n,24] (+ optional fp16 copy desc16),
 * desc_conf [n], scales [n,3], rotations [n,4], sh [n,3], opacities [n],
 * means [n,3].  depth mode ('exp',-inf,inf), conf mode ('exp',1,inf). */
int s3n_gaussian_postprocess(int64_t n, const float* pts, int ld_pts, const float* feat,
                             const float* gauss, int ld_g, int use_offsets, float* pts3d,
                             float* conf, float* desc, void* desc16, float* desc_conf,
                             float* scales, float* rotations, float* sh, float* opacities,
                             float* means, void* stream);

/* Portable counter-based weights: w[i] = (2u-1)*a + c with
 * u = (splitmix64(seed + (i+1)*0x9E3779B97F4A7C15) >> 40) * 2^-24, fp32. */
int s3n_prng_fill(float* out, int64_t n, uint64_t seed, float a, float c, void* stream);

/* fp32 -> fp16 conversion (round to nearest even) of a rows x cols block
 * with row strides ld_in / ld_out (elements). */
int s3n_cast_f16(const float* in, int64_t ld_in, void* out, int64_t ld_out, int64_t rows,
                 int cols, void* stream);

/* fp16 range guard: every fp16 activation the GEMM epilogues and LayerNorm
 * write saturates at +-65504 (NaN passes through) instead of overflowing
 * to inf, and sets a device flag.  Returns how many of the two flags (GEMM,
 * LayerNorm) are set (0 = no activation left the fp16 range since the last
 * reset), -1 on a HIP error; reset != 0 clears them.  Synchronous. */
int s3n_f16_saturations(int reset);

#ifdef __cplusplus
}
#endif
#endif /* S3N_H */
