// Memory-bound network ops (include/s3n.h): LayerNorm, patch im2col,
// bilinear x2 upsample, Gaussian-head postprocess, portable PRNG fill, cast.
// All vectorised to 16 B per lane where the layout allows (guide G13).
#include <cstdlib>

#include "common.hpp"
#include "s3n.h"

namespace {

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;

// ------------------------------------------------------------ LayerNorm --
// One wave per row; C <= 1024 (multiple of 4), held in registers.
struct LnP {
  int rows, C;
  const float* x[S3N_MAX_GROUPS];
  int64_t ldx;
  const float* gamma[S3N_MAX_GROUPS];
  const float* beta[S3N_MAX_GROUPS];
  float eps;
  f16* o16[S3N_MAX_GROUPS];
  int64_t ld16;
  float* o32[S3N_MAX_GROUPS];
  int64_t ld32;
};

// fp16 range guard of the LayerNorm fp16 outputs (see net_gemm.hip sat_f16)
__device__ uint32_t g_ln_f16_sat;

__device__ __forceinline__ _Float16 ln_sat_f16(float v) {
  if (!(fabsf(v) <= 65504.0f)) {
    g_ln_f16_sat = 1u + (threadIdx.x & 63);
    if (!isnan(v)) v = copysignf(65504.0f, v);
  }
  return (_Float16)v;
}

template <int VPL>  // float4 vectors per lane
__global__ void __launch_bounds__(kThreads) k_layernorm(LnP p) {
  const int g = blockIdx.y;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= p.rows) return;
  const float* x = p.x[g] + (int64_t)row * p.ldx;
  const float* gm = p.gamma[g];
  const float* bt = p.beta[g];
  f32x4 v[VPL], gg[VPL], bb[VPL];
  float s = 0.f;
  // gamma/beta are issued with x so their latency overlaps the reductions
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (i * 64 + lane) * 4;
    const bool in = c < p.C;
    v[i] = in ? *reinterpret_cast<const f32x4*>(x + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    gg[i] = in ? *reinterpret_cast<const f32x4*>(gm + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    bb[i] = in ? *reinterpret_cast<const f32x4*>(bt + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / p.C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < p.C)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / p.C + p.eps);
  f16* o16 = p.o16[g];
  float* o32 = p.o32[g];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c >= p.C) continue;
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = (v[i][j] - mean) * rstd * gg[i][j] + bb[i][j];
    if (o32) *reinterpret_cast<f32x4*>(o32 + (int64_t)row * p.ld32 + c) = y;
    if (o16) {
      typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
      const f16x4 h = {ln_sat_f16(y[0]), ln_sat_f16(y[1]), ln_sat_f16(y[2]), ln_sat_f16(y[3])};
      *reinterpret_cast<f16x4*>(o16 + (int64_t)row * p.ld16 + c) = h;
    }
  }
}

// ------------------------------------------------------------- im2col ----
__global__ void __launch_bounds__(kThreads)
k_patch_im2col(const float* __restrict__ img, int B, int H, int W, int p, f16* __restrict__ A) {
  const int Ht = H / p, Wt = W / p, K = 3 * p * p;
  const int64_t total = (int64_t)B * Ht * Wt * K;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int k = (int)(i % K);
  const int64_t m = i / K;
  const int tx = (int)(m % Wt), ty = (int)((m / Wt) % Ht), b = (int)(m / ((int64_t)Wt * Ht));
  const int c = k / (p * p), ky = (k / p) % p, kx = k % p;
  A[i] = (f16)img[(((int64_t)b * 3 + c) * H + ty * p + ky) * W + tx * p + kx];
}

// ----------------------------------------------------------- upsample ----
// torch upsample_bilinear2d, align_corners=True: scale = (in-1)/(out-1),
// src = scale * dst, i0 = (int)src, i1 = min(i0+1, in-1), l = src - i0.
struct UpP {
  const f16* in[S3N_MAX_GROUPS];
  f16* out[S3N_MAX_GROUPS];
  int B, H, W, C, oh, ow;
};

// Idx = uint32_t when B * oh * ow * C/8 < 2^31 (every frame-loop shape):
// the per-thread index split is then 32-bit division, not the ~4x longer
// 64-bit sequences.  PX output pixels along x per thread (2: one index
// split and the row offsets for both; the same per-pixel arithmetic).
template <typename Idx, int PX>
__global__ void __launch_bounds__(kThreads) k_upsample2x(UpP p) {
  const int g = blockIdx.y;
  const int OH = 2 * p.H, OW = 2 * p.W, C8 = p.C / 8;
  const int owp = (p.ow + PX - 1) / PX;
  const Idx total = (Idx)p.B * p.oh * owp * C8;
  const Idx i = (Idx)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c8 = (int)(i % (Idx)C8);
  Idx t = i / (Idx)C8;
  const int ox0 = (int)(t % (Idx)owp) * PX;
  t /= (Idx)owp;
  const int oy = (int)(t % (Idx)p.oh);
  const int b = (int)(t / (Idx)p.oh);
  const float sh = OH > 1 ? (float)(p.H - 1) / (float)(OH - 1) : 0.f;
  const float sw = OW > 1 ? (float)(p.W - 1) / (float)(OW - 1) : 0.f;
  const float fy = sh * oy;
  const int y0 = (int)fy;
  const int y1 = min(y0 + 1, p.H - 1);
  const float ly = fy - y0;
  const float hy = 1.f - ly;
  const f16* src = p.in[g] + (int64_t)b * p.H * p.W * p.C + c8 * 8;
  const f16* r0 = src + (int64_t)y0 * p.W * p.C;
  const f16* r1 = src + (int64_t)y1 * p.W * p.C;
  f16* dst = p.out[g] + (((int64_t)b * p.oh + oy) * p.ow) * p.C + c8 * 8;
#pragma unroll
  for (int k = 0; k < PX; ++k) {
    const int ox = ox0 + k;
    if (PX > 1 && ox >= p.ow) break;
    const float fx = sw * ox;
    const int x0 = (int)fx;
    const int x1 = min(x0 + 1, p.W - 1);
    const float lx = fx - x0;
    const float hx = 1.f - lx;
    const f16x8 a = *reinterpret_cast<const f16x8*>(r0 + (int64_t)x0 * p.C);
    const f16x8 bq = *reinterpret_cast<const f16x8*>(r0 + (int64_t)x1 * p.C);
    const f16x8 cq = *reinterpret_cast<const f16x8*>(r1 + (int64_t)x0 * p.C);
    const f16x8 d = *reinterpret_cast<const f16x8*>(r1 + (int64_t)x1 * p.C);
    f16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = (f16)(hy * (hx * (float)a[j] + lx * (float)bq[j]) + ly * (hx * (float)cq[j] + lx * (float)d[j]));
    *reinterpret_cast<f16x8*>(dst + (int64_t)ox * p.C) = o;
  }
}

// ------------------------------------------------------ postprocess -------
// pts3d / conf, desc_conf and the Gaussian parameters of row i (the
// descriptor normalisation is the caller's: in registers or through LDS)
__device__ __forceinline__ void gauss_post_row(int64_t i, const float* __restrict__ pts, int ldp,
                                               float f24, const float* __restrict__ gs, int ldg,
                                               int use_offsets, float* pts3d, float* conf,
                                               float* desc_conf, float* scales, float* rot,
                                               float* sh, float* opac, float* means) {
  const float* P = pts + i * ldp;
  // reg_dense_depth, mode exp: xyz / clip(|xyz|, 1e-8) * expm1(|xyz|)
  const float x = P[0], y = P[1], z = P[2];
  const float d = sqrtf(x * x + y * y + z * z);
  const float dc = fmaxf(d, 1e-8f);
  const float e = expm1f(d);
  const float px = x / dc * e, py = y / dc * e, pz = z / dc * e;
  pts3d[i * 3 + 0] = px; pts3d[i * 3 + 1] = py; pts3d[i * 3 + 2] = pz;
  conf[i] = 1.0f + expf(P[3]);  // reg_dense_conf exp: vmin + exp(x).clip(max=inf)
  desc_conf[i] = 1.0f + expf(f24);
  const float* G = gs + i * ldg;
  // reg_dense_offsets(shift 6): xyz/clip(d,1e-8) * (exp(d-6) - exp(-6))
  const float ox = G[0], oy = G[1], oz = G[2];
  const float od = sqrtf(ox * ox + oy * oy + oz * oz);
  const float odc = fmaxf(od, 1e-8f);
  const float of = expf(od - 6.0f) - expf(-6.0f);
  scales[i * 3 + 0] = expf(G[3]); scales[i * 3 + 1] = expf(G[4]); scales[i * 3 + 2] = expf(G[5]);
  const float r0 = G[6], r1 = G[7], r2 = G[8], r3 = G[9];
  const float rn = sqrtf(r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3) + 1e-8f;
  rot[i * 4 + 0] = r0 / rn; rot[i * 4 + 1] = r1 / rn; rot[i * 4 + 2] = r2 / rn; rot[i * 4 + 3] = r3 / rn;
  sh[i * 3 + 0] = G[10]; sh[i * 3 + 1] = G[11]; sh[i * 3 + 2] = G[12];
  opac[i] = 1.0f / (1.0f + expf(-G[13]));
  if (use_offsets) {
    means[i * 3 + 0] = px + ox / odc * of;
    means[i * 3 + 1] = py + oy / odc * of;
    means[i * 3 + 2] = pz + oz / odc * of;
  } else {
    means[i * 3 + 0] = px; means[i * 3 + 1] = py; means[i * 3 + 2] = pz;
  }
}

// One row per thread, the workgroup's 256 descriptor rows (25 floats: 24 +
// desc_conf logit) moved through LDS: read as one coalesced range,
// normalised in registers from the thread's own row (LDS stride 25 is
// conflict-free), written back into the slot and stored as coalesced desc /
// desc16 ranges.  A row per lane straight from memory (96-100 B stride)
// touches ~50 cache lines per load / store instruction.
__global__ void __launch_bounds__(kThreads)
k_gauss_post(int64_t n, const float* __restrict__ pts, int ldp, const float* __restrict__ feat,
             const float* __restrict__ gs, int ldg, int use_offsets, float* pts3d, float* conf,
             float* desc, f16* desc16, float* desc_conf, float* scales, float* rot, float* sh,
             float* opac, float* means) {
  __shared__ float s_f[kThreads * 25];
  const int64_t r0 = (int64_t)blockIdx.x * kThreads;
  const int rows = (int)min((int64_t)kThreads, n - r0);
  const int t = threadIdx.x;
  for (int e = t; e < rows * 25; e += kThreads) s_f[e] = feat[r0 * 25 + e];
  __syncthreads();
  float F[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) F[k] = t < rows ? s_f[t * 25 + k] : 1.0f;
  __syncthreads();
  if (t < rows) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 24; ++k) s += F[k] * F[k];
    const float inv = 1.0f / sqrtf(s);
#pragma unroll
    for (int k = 0; k < 24; ++k) s_f[t * 25 + k] = F[k] * inv;
    gauss_post_row(r0 + t, pts, ldp, F[24], gs, ldg, use_offsets, pts3d, conf, desc_conf,
                   scales, rot, sh, opac, means);
  }
  __syncthreads();
  for (int e = t; e < rows * 24; e += kThreads) {
    const float v = s_f[(e / 24) * 25 + e % 24];
    desc[r0 * 24 + e] = v;
    if (desc16) desc16[r0 * 24 + e] = (f16)v;
  }
}

// ------------------------------------------------------------- PRNG ------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(kThreads)
k_prng(float* __restrict__ out, int64_t n, uint64_t seed, float a, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t z = mix64(seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
  const float u = (float)(uint32_t)(z >> 40) * 5.9604644775390625e-08f;
  const float t = u * 2.0f;
  const float w = t - 1.0f;
  const float y = w * a;
  out[i] = y + c;
}

__global__ void __launch_bounds__(kThreads)
k_cast(const float* __restrict__ in, int64_t ldi, f16* __restrict__ out, int64_t ldo,
       int64_t rows, int cols) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols, c = i % cols;
  out[r * ldo + c] = (f16)in[r * ldi + c];
}

}  // namespace

extern "C" {

int s3n_layernorm(int rows, int C, int groups, const float* const* x, int64_t ldx,
                  const float* const* gamma, const float* const* beta, float eps,
                  void* const* out16, int64_t ld16, float* const* out32, int64_t ld32,
                  void* stream) {
  S3_REQUIRE(rows >= 0 && C > 0 && C % 4 == 0 && C <= 2048, "s3n_layernorm: C must be 4..2048, %%4");
  S3_REQUIRE(groups >= 1 && groups <= S3N_MAX_GROUPS, "s3n_layernorm: groups 1..4");
  S3_REQUIRE(ldx % 4 == 0 && (!out32 || ld32 % 4 == 0) && (!out16 || ld16 % 4 == 0),
             "s3n_layernorm: strides must be multiples of 4");
  if (rows == 0) return S3_OK;
  LnP p;
  p.rows = rows; p.C = C; p.ldx = ldx; p.eps = eps; p.ld16 = ld16; p.ld32 = ld32;
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    const bool on = g < groups;
    p.x[g] = on ? x[g] : nullptr;
    p.gamma[g] = on ? gamma[g] : nullptr;
    p.beta[g] = on ? beta[g] : nullptr;
    p.o16[g] = (on && out16) ? (f16*)out16[g] : nullptr;
    p.o32[g] = (on && out32) ? out32[g] : nullptr;
  }
  dim3 grid((unsigned)s3::cdiv(rows, 4), (unsigned)groups);
  hipStream_t st = s3::as_stream(stream);
  const int vpl = (int)s3::cdiv(C, 256);
  if (vpl <= 1) k_layernorm<1><<<grid, kThreads, 0, st>>>(p);
  else if (vpl <= 2) k_layernorm<2><<<grid, kThreads, 0, st>>>(p);
  else if (vpl <= 3) k_layernorm<3><<<grid, kThreads, 0, st>>>(p);
  else if (vpl <= 4) k_layernorm<4><<<grid, kThreads, 0, st>>>(p);
  else k_layernorm<8><<<grid, kThreads, 0, st>>>(p);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3n_patch_im2col(const float* img, int B, int H, int W, int p, void* A, void* stream) {
  S3_REQUIRE(B > 0 && p > 0 && H % p == 0 && W % p == 0, "s3n_patch_im2col: bad sizes");
  const int64_t total = (int64_t)B * (H / p) * (W / p) * 3 * p * p;
  k_patch_im2col<<<(unsigned)s3::cdiv(total, kThreads), kThreads, 0, s3::as_stream(stream)>>>(
      img, B, H, W, p, (f16*)A);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3n_upsample2x(int groups, const void* const* in, void* const* out, int B, int H, int W,
                   int C, int oh, int ow, void* stream) {
  S3_REQUIRE(groups >= 1 && groups <= S3N_MAX_GROUPS && B > 0 && H > 0 && W > 0 && C % 8 == 0,
             "s3n_upsample2x: bad sizes");
  S3_REQUIRE(oh > 0 && ow > 0 && oh <= 2 * H && ow <= 2 * W, "s3n_upsample2x: bad crop");
  UpP p;
  p.B = B; p.H = H; p.W = W; p.C = C; p.oh = oh; p.ow = ow;
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    p.in[g] = g < groups ? (const f16*)in[g] : nullptr;
    p.out[g] = g < groups ? (f16*)out[g] : nullptr;
  }
  // S3_UPSAMPLE_PX=1 / 4: output pixels per thread (A/B)
  static const int px = [] {
    const char* e = std::getenv("S3_UPSAMPLE_PX");
    return e && e[0] == '1' ? 1 : (e && e[0] == '4' ? 4 : 2);
  }();
  const int64_t total = (int64_t)B * oh * ((ow + px - 1) / px) * (C / 8);
  dim3 grid((unsigned)s3::cdiv(total, kThreads), (unsigned)groups);
  hipStream_t st = s3::as_stream(stream);
  const bool small = (int64_t)B * oh * ow * (C / 8) < ((int64_t)1 << 31);
  if (px == 4 && small) k_upsample2x<uint32_t, 4><<<grid, kThreads, 0, st>>>(p);
  else if (px == 4) k_upsample2x<int64_t, 4><<<grid, kThreads, 0, st>>>(p);
  else if (px == 2 && small) k_upsample2x<uint32_t, 2><<<grid, kThreads, 0, st>>>(p);
  else if (px == 2) k_upsample2x<int64_t, 2><<<grid, kThreads, 0, st>>>(p);
  else if (small) k_upsample2x<uint32_t, 1><<<grid, kThreads, 0, st>>>(p);
  else k_upsample2x<int64_t, 1><<<grid, kThreads, 0, st>>>(p);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3n_gaussian_postprocess(int64_t n, const float* pts, int ld_pts, const float* feat,
                             const float* gauss, int ld_g, int use_offsets, float* pts3d,
                             float* conf, float* desc, void* desc16, float* desc_conf,
                             float* scales, float* rotations, float* sh, float* opacities,
                             float* means, void* stream) {
  S3_REQUIRE(n >= 0 && ld_pts >= 4 && ld_g >= 14, "s3n_gaussian_postprocess: bad sizes");
  if (n == 0) return S3_OK;
  k_gauss_post<<<(unsigned)s3::cdiv(n, kThreads), kThreads, 0, s3::as_stream(stream)>>>(
      n, pts, ld_pts, feat, gauss, ld_g, use_offsets, pts3d, conf, desc, (f16*)desc16,
      desc_conf, scales, rotations, sh, opacities, means);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3n_prng_fill(float* out, int64_t n, uint64_t seed, float a, float c, void* stream) {
  S3_REQUIRE(n >= 0, "s3n_prng_fill: n < 0");
  if (n == 0) return S3_OK;
  k_prng<<<(unsigned)s3::cdiv(n, kThreads), kThreads, 0, s3::as_stream(stream)>>>(out, n, seed, a, c);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3n_cast_f16(const float* in, int64_t ld_in, void* out, int64_t ld_out, int64_t rows,
                 int cols, void* stream) {
  S3_REQUIRE(rows >= 0 && cols >= 0, "s3n_cast_f16: bad sizes");
  const int64_t n = rows * cols;
  if (n == 0) return S3_OK;
  k_cast<<<(unsigned)s3::cdiv(n, kThreads), kThreads, 0, s3::as_stream(stream)>>>(
      in, ld_in, (f16*)out, ld_out, rows, cols);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

}  // extern "C"

int s3n_ln_f16_saturations(int reset) {
  uint32_t v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ln_f16_sat), sizeof(v)) != hipSuccess) return -1;
  if (reset && v) {
    const uint32_t z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ln_f16_sat), &z, sizeof(z)) != hipSuccess) return -1;
  }
  return v ? 1 : 0;
}
