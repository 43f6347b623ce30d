// Grouped fp16 MFMA GEMM with fused epilogues and an implicit-im2col
// convolution A path (include/s3n.h s3n_gemm).
//
// Tile: BM x BN x 64 per 256-lane workgroup (4 waves as 2x2), each wave a
// (BM/2)x(BN/2) block of v_mfma_f32_32x32x16_f16 accumulators.  Operands are
// staged global -> registers -> LDS (double buffer, one barrier per K tile,
// next tile's global loads issued before the current tile's MFMAs).  LDS
// rows are 128 B (64 fp16); 16-B chunks are XOR-swizzled with (row>>1)&7 so
// every ds_read_b128 lane group of the A/B fragment reads hits 16 distinct
// 16-B slots of the 256-B bank row (conflict-free, guide §2/T2).  The tile
// grid is remapped so that each XCD gets a contiguous run of tiles.
//
// In-workgroup split-K (KG > 1): a workgroup holds KG groups of NWM x NWN
// waves on the same output tile; group kg consumes the K tiles
// kt = kg, kg + KG, ... through its own LDS ring, all groups step together
// (one barrier per K step), and the KG partial tiles are summed through LDS
// in group order before one epilogue.  At M = 768 (one image) the tile grid
// alone leaves one 4-wave workgroup per CU waiting on its DMA; KG groups give
// each SIMD KG waves to overlap load latency with MFMA without the fp32
// workspace round trip of a split-K launch.
#include <algorithm>

#pragma once
#include "common.hpp"
#include "s3n.h"

// Shared by the GEMM translation units (net_gemm*.hip): the kernel template
// is instantiated per tile family in its own file so the families compile in
// parallel; the argument struct and the host tuning flags are common.
namespace s3gemm {
typedef _Float16 f16;
struct GemmP;
extern int g_xcd_flags;   // tuning hook s3n_gemm_set_xcd_flags: 1 = band split only
// launch the tile family of one translation unit; -1000 = tile not in it
int launch_t1(int tile, const GemmP& p, hipStream_t st);
int launch_t2(int tile, const GemmP& p, hipStream_t st);
int launch_t3(int tile, const GemmP& p, hipStream_t st);
int launch_t4(int tile, const GemmP& p, hipStream_t st);
int launch_t5(int tile, const GemmP& p, hipStream_t st);
int launch_t6(int tile, const GemmP& p, hipStream_t st);
int launch_t7(int tile, const GemmP& p, hipStream_t st);
int launch_t8(int tile, const GemmP& p, hipStream_t st);
int launch_t9(int tile, const GemmP& p, hipStream_t st);
// read (and optionally reset) one translation unit's fp16 saturation flag
int sat_t1(int reset);
int sat_t2(int reset);
int sat_t3(int reset);
int sat_t4(int reset);
int sat_t5(int reset);
int sat_t6(int reset);
int sat_t7(int reset);
int sat_t8(int reset);
int sat_t9(int reset);
constexpr int kNotMine = -1000;
}  // namespace s3gemm

namespace s3gemm {

struct GemmP {
  int M, N, K, groups;
  const f16* A[S3N_MAX_GROUPS];
  int64_t lda;
  const f16* B[S3N_MAX_GROUPS];
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
  f16* C2[S3N_MAX_GROUPS];
  int64_t ldc2;
  int act, store_mode, a_mode;
  int cH, cW, cC, ks, st, pad, oH, oW, relu_in;
  int sH, sW, sS, sCout;
  int tiles_m, tiles_n;
  int split_k, kt_per_split;
  float* ws;
  int debug;       // s3n_gemm_set_debug flags (tuning only)
  int vec_epi;     // LDS-staged epilogue with 8-column vector accesses (host-checked)
  const f16* tail_w[S3N_MAX_GROUPS];   // fused 1x1 tail (s3n.h), tail_n % 8 == 0
  const float* tail_b[S3N_MAX_GROUPS];
  float* tail_out[S3N_MAX_GROUPS];
  int tail_n;
  int64_t ld_tail;
  int col_major;   // tile order: 1 = M fastest (each XCD owns a band of N)
  int xcd_px;      // > 0: each XCD owns a (tiles_m / xcd_px) x (tiles_n * xcd_px / 8) block
  const float* rope_cos;
  const float* rope_sin;
  int rope_ncols;
  const int64_t* rope_pos[S3N_MAX_GROUPS];
  const f16* Bp[S3N_MAX_GROUPS];   // fragment-packed B (net_gemm_t9.hip), or null
};
}  // namespace s3gemm

namespace {
using s3gemm::GemmP;
using s3gemm::g_xcd_flags;
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kThreads = 256;

// XOR swizzle of the 16-B chunks of one LDS tile row (BK fp16 = 128 or
// 256 B): every 16-lane group of a ds_read_b128 fragment read (rows of one
// 32-row block at one logical chunk) then hits 16 distinct 16-B bank slots.
template <int BK>
__device__ __forceinline__ int swz(int row, int kc) {
  if constexpr (BK == 64) return kc ^ ((row >> 1) & 7);   // 2 rows per 256-B bank row
  else return kc ^ (row & 15);                            // 1 row per 256-B bank row
}

// fp16 range guard: activations stored as fp16 saturate at +-65504 instead
// of becoming inf (real checkpoints may produce larger activations than the
// portable-PRNG weights), and the event is recorded for the host
// (s3n_f16_saturations).  The flag store carries a lane-dependent value.
__device__ uint32_t g_f16_sat;

__device__ __forceinline__ f16 sat_f16(float v) {
  if (!(fabsf(v) <= 65504.0f)) {
    g_f16_sat = 1u + (threadIdx.x & 63);
    if (!isnan(v)) v = copysignf(65504.0f, v);
  }
  return (f16)v;
}

// erf by Abramowitz & Stegun 7.1.26: 1 - (a1 t + .. + a5 t^5) e^{-x^2},
// t = 1 / (1 + p |x|), on the bare v_rcp_f32 / v_exp_f32.  |error| <= 4.7e-7
// in fp32 over the whole line (tests/test_net_ops.py
// test_gemm_gelu_erf_accuracy), against the library erff's ~40 instructions
// over two divergent branches: the GELU epilogue of the fc1 GEMMs costs a
// third of the VALU.  The GELU output is stored in fp16 (quantum >= 6e-8 x
// its magnitude); an absolute erf error e moves it by 0.5 |x| e.
__device__ __forceinline__ float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  q *= t;
  const float e = __builtin_amdgcn_exp2f(-(a * a) * 1.4426950408889634f);
  return copysignf(1.0f - q * e, x);
}

__device__ __forceinline__ float gelu(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, k = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// A operand modes of the kernel template (AMODE): dense rows, implicit-im2col
// conv, implicit-im2col conv with ReLU applied to the A fragments.
constexpr int kDense = 0, kConv = 1, kConvRelu = 2;

// 16-B LDS-DMA through a raw buffer resource: voffset per lane (bytes),
// soffset uniform (bytes); offsets at or past num_records read as zero,
// which implements every M/N/K tail and conv padding tap.
#define S3_BLDS(rsrc, lptr, voff, soff)                                               \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(                                          \
      (rsrc), (__attribute__((address_space(3))) void*)(lptr), 16, (int)(voff), (int)(soff), 0, 0)

constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const int64_t lim = bytes < 0x7fffffff ? bytes : 0x7fffffff;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)lim,
                                           0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until <= min(after, MAXA) * PERW loads remain (after: tiles issued
// behind the one being waited for; wave-uniform)
template <int PERW, int MAXA>
__device__ __forceinline__ void wait_tiles(int after) {
  if constexpr (MAXA <= 0) {
    wait_vmcnt<0>();
  } else {
    if (after >= MAXA) wait_vmcnt<PERW * MAXA>();
    else wait_tiles<PERW, MAXA - 1>(after);
  }
}

// Store of one finished element (plain / ConvT / pixel-shuffle scatter) and
// its optional fp16 copy.
__device__ __forceinline__ int64_t out_offset(const GemmP& p, int row, int col) {
  int64_t off;
  if (p.store_mode == S3N_STORE_PLAIN) {
    off = (int64_t)row * p.ldc + col;
  } else {
    // row = token (b, ty, tx) on an sH x sW grid; col -> (i, j, co)
    const int tx = row % p.sW, t = row / p.sW, ty = t % p.sH, b = t / p.sH;
    int i, j, co;
    if (p.store_mode == S3N_STORE_CONVT) {
      co = col % p.sCout;
      const int ij = col / p.sCout;
      i = ij / p.sS;
      j = ij % p.sS;
    } else {
      co = col / (p.sS * p.sS);
      const int ij = col % (p.sS * p.sS);
      i = ij / p.sS;
      j = ij % p.sS;
    }
    const int64_t oy = (int64_t)ty * p.sS + i, ox = (int64_t)tx * p.sS + j;
    off = (((int64_t)b * p.sH * p.sS + oy) * ((int64_t)p.sW * p.sS) + ox) * p.sCout + co;
  }
  return off;
}

__device__ __forceinline__ void store_out(const GemmP& p, int g, int row, int col, float v) {
  void* C = p.C[g];
  f16* C2 = p.C2[g];
  const int64_t off = out_offset(p, row, col);
  if (p.c_f16) reinterpret_cast<f16*>(C)[off] = sat_f16(v);
  else reinterpret_cast<float*>(C)[off] = v;
  if (C2) C2[(int64_t)row * p.ldc2 + col] = sat_f16(v);
}

__device__ __forceinline__ float act_fn(const GemmP& p, float v) {
  if (p.act == S3N_ACT_GELU) return gelu(v);
  if (p.act == S3N_ACT_RELU) return fmaxf(v, 0.0f);
  return v;
}

__device__ __forceinline__ float load_res(const void* R, int r_f16, int64_t o) {
  return r_f16 ? (float)reinterpret_cast<const f16*>(R)[o] : reinterpret_cast<const float*>(R)[o];
}

// bias -> act -> + R1 -> + R2 -> store, for one element (split-K combine).
template <bool kBias = true>
__device__ __forceinline__ void epilogue(const GemmP& p, int g, int row, int col, float v) {
  const float* __restrict__ bias = p.bias[g];
  if (kBias && bias) v += bias[col];
  v = act_fn(p, v);
  if (p.R1[g]) v += load_res(p.R1[g], p.r1_f16, (int64_t)row * p.ldr1 + col);
  if (p.R2[g]) v += load_res(p.R2[g], p.r2_f16, (int64_t)row * p.ldr2 + col);
  store_out(p, g, row, col, v);
}

// Row of accumulator register r of a 32x32 MFMA block, relative to the
// block row of this lane half (lane >> 5 adds 4).
__device__ __forceinline__ int acc_row(int r) { return (r & 3) + 8 * (r >> 2); }

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Accumulator block of one MFMA shape: v_mfma_f32_32x32x16_f16 (16 fp32
// per lane, column lane & 31, rows acc_row(r) + 4 (lane >> 5)) or
// v_mfma_f32_16x16x32_f16 (4 fp32 per lane, column lane & 15, rows
// 4 (lane >> 4) + r).  The 16x16x32 form holds the chip's clock higher
// under load (MI355X_MICROARCH.md "DVFS give-back" item 7) and lets a wave
// tile be any multiple of 16 (e.g. 32 x 80), so a 4-wave workgroup can own
// the large tiles whose operand reuse keeps the LDS reads per MFMA low.
template <int MF>
struct AccT;
template <>
struct AccT<32> {
  typedef f32x16 T;
  static constexpr int R = 16;
  static constexpr int KS = 16;   // K per MFMA
  __device__ static __forceinline__ int row(int r, int lane) { return acc_row(r) + 4 * (lane >> 5); }
  __device__ static __forceinline__ int col(int lane) { return lane & 31; }
  __device__ static __forceinline__ int frag_row(int lane) { return lane & 31; }
  __device__ static __forceinline__ int frag_chunk(int ks, int lane) { return 2 * ks + (lane >> 5); }
  __device__ static __forceinline__ T mfma(f16x8 a, f16x8 b, T c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <>
struct AccT<16> {
  typedef f32x4 T;
  static constexpr int R = 4;
  static constexpr int KS = 32;
  __device__ static __forceinline__ int row(int r, int lane) { return 4 * (lane >> 4) + r; }
  __device__ static __forceinline__ int col(int lane) { return lane & 15; }
  __device__ static __forceinline__ int frag_row(int lane) { return lane & 15; }
  __device__ static __forceinline__ int frag_chunk(int ks, int lane) { return 4 * ks + (lane >> 4); }
  __device__ static __forceinline__ T mfma(f16x8 a, f16x8 b, T c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

// The same epilogue for the 16 elements one lane holds of a 32x32 block
// (rows row0 + acc_row(r), one column).  Every operand load is issued before
// the first store: R1 may be the output itself (in-place residual add), so
// a load placed after a store could not be hoisted and each of the 16 would
// pay a full memory latency on its own.
template <bool kBias = true>
__device__ __forceinline__ void epilogue_block(const GemmP& p, int g, int row0, int col,
                                               const float (&v)[16]) {
  if (col >= p.N) return;
  const float* __restrict__ bias = p.bias[g];
  const void* R1 = p.R1[g];
  const void* R2 = p.R2[g];
  const float bv = (kBias && bias) ? bias[col] : 0.0f;
  // rows past M only occur in the last row tile: clamp the loads there
  // (their values are dropped), so the load batch stays branch-free
  const int rmax = p.M - 1 - row0;
  float r1[16], r2[16];
  if (R1) {
    const int64_t o = (int64_t)row0 * p.ldr1 + col;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      r1[r] = load_res(R1, p.r1_f16, o + (int64_t)min(acc_row(r), rmax) * p.ldr1);
  }
  if (R2) {
    const int64_t o = (int64_t)row0 * p.ldr2 + col;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      r2[r] = load_res(R2, p.r2_f16, o + (int64_t)min(acc_row(r), rmax) * p.ldr2);
  }
  float x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float t = v[r];
    if (kBias && bias) t += bv;
    t = act_fn(p, t);
    if (R1) t += r1[r];
    if (R2) t += r2[r];
    x[r] = t;
  }
  if (p.store_mode == S3N_STORE_PLAIN) {
    const int64_t o = (int64_t)row0 * p.ldc + col;
    f16* C2 = p.C2[g];
    const int64_t o2 = (int64_t)row0 * p.ldc2 + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (acc_row(r) > rmax) continue;
      const int64_t e = o + (int64_t)acc_row(r) * p.ldc;
      if (p.c_f16) reinterpret_cast<f16*>(p.C[g])[e] = sat_f16(x[r]);
      else reinterpret_cast<float*>(p.C[g])[e] = x[r];
      if (C2) C2[o2 + (int64_t)acc_row(r) * p.ldc2] = sat_f16(x[r]);
    }
  } else {
    for (int r = 0; r < 16; ++r)
      if (acc_row(r) <= rmax) store_out(p, g, row0 + acc_row(r), col, x[r]);
  }
}

// NWM x NWN waves, each owning a (BM/NWM) x (BN/NWN) block of 32x32
// accumulators.
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load8(const float* q, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(q);
  const f32x4 b = *reinterpret_cast<const f32x4*>(q + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
}

__device__ __forceinline__ void load8_res(const void* R, int f16in, int64_t o, float (&v)[8]) {
  if (f16in) {
    const f16x8 h = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(R) + o);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)h[e];
  } else {
    load8(reinterpret_cast<const float*>(R) + o, v);
  }
}

__device__ __forceinline__ void store8_f32(float* q, const float (&v)[8]) {
  *reinterpret_cast<f32x4*>(q) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(q + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

__device__ __forceinline__ void store8_f16(f16* q, const float (&v)[8]) {
  f16x8 h;
#pragma unroll
  for (int e = 0; e < 8; ++e) h[e] = sat_f16(v[e]);
  *reinterpret_cast<f16x8*>(q) = h;
}

// The accumulator tile goes through LDS (row-major fp32, the staging ring
// is free once the K loop is done) and comes back as 8-column row chunks,
// so that bias / residual / RoPE-table loads and the stores are 16/32-B
// vector accesses along rows (fully coalesced) instead of one 2-4 B access
// per accumulator register.  The host enables it when every row stride and
// base is 16-B aligned and 8-column chunks stay contiguous in the output.
template <int BM, int BN, int NWM, int NWN, int FM, int FN, int LDT, int RING_BYTES, int KG = 1,
          int MF = 32>
__device__ __forceinline__ void epilogue_vec(const GemmP& p, int g, int m0, int n0,
                                             typename AccT<MF>::T (&acc)[FM][FN], float* stage) {
  typedef AccT<MF> AT;
  constexpr int WM = BM / NWM, WN = BN / NWN, NT = 64 * NWM * NWN * KG;
  constexpr int CPR = BN / 8;                 // 8-column chunks per tile row
  constexpr int NCH = (BM * CPR + NT - 1) / NT;   // chunks per thread
  constexpr int SLICE = BM * LDT;             // one K-group's partial tile (floats)
  // small tiles: the chunk operands (bias, fp32 residual, RoPE position) are
  // loaded before the LDS staging so their latency overlaps it
  constexpr bool kPre = NCH <= 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = wave / (NWM * NWN), wq = wave % (NWM * NWN);
  const int wm = wq / NWN, wn = wq % NWN;
  const float* __restrict__ bias = p.bias[g];
  const void* R1 = p.R1[g];
  const void* R2 = p.R2[g];
  const int64_t* __restrict__ pos = p.rope_pos[g];
  f16* C2 = p.C2[g];
  const bool split = p.split_k > 1;
  const f16* __restrict__ tw = p.tail_w[g];
  float pb[kPre ? NCH : 1][8], pr[kPre ? NCH : 1][8];
  int64_t pps[kPre ? NCH : 1];
  if constexpr (kPre) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = min(tid + k * NT, BM * CPR - 1), rl = c / CPR, cl = (c % CPR) * 8;
      const int row = min(m0 + rl, p.M - 1), col = min(n0 + cl, p.N - 8);
      if (bias && !split) load8(bias + col, pb[k]);
      if (R1 && !split) load8_res(R1, p.r1_f16, (int64_t)row * p.ldr1 + col, pr[k]);
      pps[k] = (pos && col < p.rope_ncols) ? pos[(int64_t)row * 2 + ((col & 63) >> 5)] : 0;
    }
  }
  __syncthreads();   // every wave is done with the K loop's LDS reads
  // each K-group stages its partial tile in its own slice
  float* mine = stage + kg * SLICE;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
      for (int r = 0; r < AT::R; ++r)
        mine[(wm * WM + fm * MF + AT::row(r, lane)) * LDT + wn * WN + fn * MF + AT::col(lane)] =
            acc[fm][fn][r];
  __syncthreads();
  if constexpr (KG > 1) {
    // sum the K-groups' partials in group order into slice 0 (fixed order:
    // the result does not depend on scheduling)
    for (int c = tid; c < BM * CPR; c += NT) {
      const int rl = c / CPR, cl = (c % CPR) * 8;
      float v[8], t[8];
      load8(stage + rl * LDT + cl, v);
#pragma unroll
      for (int q = 1; q < KG; ++q) {
        load8(stage + q * SLICE + rl * LDT + cl, t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      store8_f32(stage + rl * LDT + cl, v);
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = tid + k * NT;
    if (c >= BM * CPR) continue;
    const int rl = c / CPR, cl = (c % CPR) * 8;
    const int row = m0 + rl, col = n0 + cl;
    if (row >= p.M || col >= p.N) continue;
    float v[8];
    load8(stage + rl * LDT + cl, v);
    if (split) {
      store8_f32(p.ws + (((int64_t)g * p.split_k + blockIdx.y) * p.M + row) * p.N + col, v);
      continue;
    }
    if (bias) {
      float bl[8];
      if constexpr (kPre) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bl[e] = pb[k][e];
      } else {
        load8(bias + col, bl);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bl[e];
    }
    if (pos && col < p.rope_ncols) {
      // partner columns col ^ 16 of the same 64-wide head: same row of the tile
      float xp[8], bp[8], cs[8], sn[8];
      load8(stage + rl * LDT + (cl ^ 16), xp);
      if (bias) {
        load8(bias + (col ^ 16), bp);
#pragma unroll
        for (int e = 0; e < 8; ++e) xp[e] += bp[e];
      }
      int64_t ps;
      if constexpr (kPre) ps = pps[k];
      else ps = pos[(int64_t)row * 2 + ((col & 63) >> 5)];
      load8(p.rope_cos + ps * 16 + (col & 15), cs);
      load8(p.rope_sin + ps * 16 + (col & 15), sn);
      const bool lo = (col & 31) < 16;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = lo ? v[e] * cs[e] - xp[e] * sn[e] : v[e] * cs[e] + xp[e] * sn[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = act_fn(p, v[e]);
    if (R1) {
      float t[8];
      if constexpr (kPre) {
#pragma unroll
        for (int e = 0; e < 8; ++e) t[e] = pr[k][e];
      } else {
        load8_res(R1, p.r1_f16, (int64_t)row * p.ldr1 + col, t);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    if (R2) {
      float t[8];
      load8_res(R2, p.r2_f16, (int64_t)row * p.ldr2 + col, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    if (p.C[g]) {
      const int64_t off = out_offset(p, row, col);
      if (p.c_f16) store8_f16(reinterpret_cast<f16*>(p.C[g]) + off, v);
      else store8_f32(reinterpret_cast<float*>(p.C[g]) + off, v);
    }
    if (C2) store8_f16(C2 + (int64_t)row * p.ldc2 + col, v);
    if (tw) store8_f32(stage + rl * LDT + cl, v);   // the tail reads the finished row
  }
  if (tw) {
    // fused 1x1 tail: out[row, o] = sum_k v[row, k] w[o, k] + b[o] (fp32
    // activations, fp16 weights, fp32 accumulation), 8 outputs per thread.
    // The tail weights sit behind the staged tile in LDS when they fit.
    // (converted to fp32 once, so the product loop has no conversions:
    // (float)w is exact, the same fma chain)
    constexpr int kWOff = BM * LDT * 4;
    constexpr bool kWLds32 = kWOff + 16 * BN * 4 <= RING_BYTES;
    constexpr bool kWLds = !kWLds32 && kWOff + 16 * BN * 2 <= RING_BYTES;
    const f16* wsrc = tw;
    float* wl32 = reinterpret_cast<float*>(reinterpret_cast<char*>(stage) + kWOff);
    if constexpr (kWLds32) {
      for (int i = tid * 8; i < p.tail_n * BN; i += NT * 8) {
        const f16x8 w8 = *reinterpret_cast<const f16x8*>(tw + i);
        float w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = (float)w8[j];
        store8_f32(wl32 + i, w);
      }
    } else if constexpr (kWLds) {
      f16* wl = reinterpret_cast<f16*>(reinterpret_cast<char*>(stage) + kWOff);
      for (int i = tid * 8; i < p.tail_n * BN; i += NT * 8)
        *reinterpret_cast<f16x8*>(wl + i) = *reinterpret_cast<const f16x8*>(tw + i);
      wsrc = wl;
    }
    __syncthreads();
    const int TC = p.tail_n / 8;
    const float* __restrict__ tb = p.tail_b[g];
    for (int c = tid; c < BM * TC; c += NT) {
      const int rl = c / TC, oc = (c % TC) * 8;
      const int row = m0 + rl;
      if (row >= p.M) continue;
      float a[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = 0.f;
      for (int k = 0; k < BN; k += 8) {
        float x[8];
        load8(stage + rl * LDT + k, x);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if constexpr (kWLds32) {
            float w[8];
            load8(wl32 + (oc + e) * BN + k, w);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[e] += x[j] * w[j];
          } else {
            const f16x8 w8 = *reinterpret_cast<const f16x8*>(wsrc + (oc + e) * BN + k);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[e] += x[j] * (float)w8[j];
          }
        }
      }
      if (tb) {
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += tb[oc + e];
      }
      store8_f32(p.tail_out[g] + (int64_t)row * p.ld_tail + oc, a);
    }
  }
}

// Per-register epilogue (scatter stores, unaligned operands, split-K
// partial planes, RoPE via lane shuffles) of a BM x BN tile of NWM x NWN
// waves, each holding FM x FN 32x32 accumulators.
template <int BM, int BN, int NWM, int NWN, int FM, int FN>
__device__ __forceinline__ void epilogue_regs(const GemmP& p, int g, int m0, int n0,
                                              f32x16 (&acc)[FM][FN]) {
  constexpr int WM = BM / NWM, WN = BN / NWN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  const int M = p.M, N = p.N;
  const int s_idx = blockIdx.y;
  if (p.rope_pos[g]) {
    // bias, then RoPE: the partner column (col ^ 16, same rows) sits in lane
    // ^ 16 of the same 32x32 accumulator, so one xor-shuffle fetches it.
    // Positions, then the cos/sin rows, are loaded for all 16 rows at once.
    const int64_t* __restrict__ pos = p.rope_pos[g];
    const float* __restrict__ bias = p.bias[g];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int col = n0 + wn * WN + fn * 32 + (lane & 31);
        const int row0 = m0 + wm * WM + fm * 32 + 4 * (lane >> 5);
        const float bv = (bias && col < N) ? bias[col] : 0.0f;
        const int d = col & 63, j = col & 15;
        const bool lo = (col & 31) < 16, rot = col < p.rope_ncols;
        float x[16], xp[16];
        int64_t ps[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          x[r] = acc[fm][fn][r] + bv;
          xp[r] = __shfl_xor(x[r], 16, 64);
          const int row = row0 + acc_row(r);
          ps[r] = (rot && row < M) ? pos[(int64_t)row * 2 + (d >> 5)] : 0;
        }
        if (rot) {
          float cs[16], sn[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            cs[r] = p.rope_cos[ps[r] * 16 + j];
            sn[r] = p.rope_sin[ps[r] * 16 + j];
          }
#pragma unroll
          for (int r = 0; r < 16; ++r)
            x[r] = lo ? x[r] * cs[r] - xp[r] * sn[r] : x[r] * cs[r] + xp[r] * sn[r];
        }
        epilogue_block<false>(p, g, row0, col, x);
      }
    return;
  }
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int col = n0 + wn * WN + fn * 32 + (lane & 31);
      const int row0 = m0 + wm * WM + fm * 32 + 4 * (lane >> 5);
      if (col >= N) continue;
      if (p.split_k > 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = row0 + acc_row(r);
          if (row < M) p.ws[(((int64_t)g * p.split_k + s_idx) * M + row) * N + col] = acc[fm][fn][r];
        }
      } else {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[fm][fn][r];
        epilogue_block(p, g, row0, col, v);
      }
    }
}

// Waves per SIMD the LDS footprint allows (the register budget the
// compiler may use without costing occupancy).
constexpr int lds_waves_per_simd(int BM, int BN, int NW, int S, int BK) {
  const int wg = (160 * 1024) / (S * (BM + BN) * BK * 2);
  const int w = (wg > 8 ? 8 : wg) * NW / 4;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

template <int BM, int BN, int NWM, int NWN, int AMODE, int kStages, int BK, int KG = 1, int MF = 32>
__global__ void __launch_bounds__(64 * NWM * NWN * KG,
                                  lds_waves_per_simd(BM, BN, NWM * NWN * KG, kStages * KG, BK))
k_gemm(GemmP p) {
  typedef AccT<MF> AT;
  constexpr int NW = NWM * NWN;   // waves of one K-group
  constexpr int WM = BM / NWM, WN = BN / NWN;
  constexpr int FM = WM / MF, FN = WN / MF;
  // One LDS-DMA wave instruction moves 64 lanes x 16 B = RPI tile rows of
  // BK fp16.  Each wave issues AW + BW per K tile.
  static_assert(BK == 64 || BK == 128, "K tile");
  constexpr int CPR = BK / 8;          // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;        // rows per DMA instruction
  constexpr int AW = BM / RPI / NW, BW = BN / RPI / NW;
  static_assert(AW * RPI * NW == BM && BW * RPI * NW == BN, "LDS-DMA rows must split over waves");
  static_assert(WM % MF == 0 && WN % MF == 0, "whole MFMA accumulator blocks per wave");
  constexpr int PERW = AW + BW;
  constexpr int STAGE = (BM + BN) * BK;
  __shared__ __attribute__((aligned(1024))) f16 smem[KG * kStages * STAGE];

  const int g = blockIdx.z;
  const int nwg = p.tiles_m * p.tiles_n;
  int tm, tn;
  if (p.xcd_px > 0) {
    // 2-D XCD partition (host-checked divisibility, nwg % 8 == 0): XCD x
    // (= blockIdx.x % 8 under round-robin dispatch) owns one block of the
    // tile grid, so it reads 1/xcd_px of A and xcd_px/8 of B instead of all
    // of one operand -- the L2-miss traffic of the operand that a band
    // split leaves whole on every XCD
    const int px = p.xcd_px, py = 8 / px;
    const int xcd = blockIdx.x % 8, k = blockIdx.x / 8;
    const int rm = p.tiles_m / px, rn = p.tiles_n / py;
    tm = (xcd / py) * rm + k % rm;
    tn = (xcd % py) * rn + k / rm;
  } else {
    const int tile = xcd_remap(blockIdx.x, nwg);
    // xcd_remap gives each XCD a contiguous run of tile ids; the order makes
    // that run share the larger operand (its slice stays in the XCD's L2).
    tm = p.col_major ? tile % p.tiles_m : tile / p.tiles_n;
    tn = p.col_major ? tile / p.tiles_m : tile % p.tiles_n;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wave_all / NW;            // K-group of this wave
  const int wave = wave_all % NW;          // wave within its K-group
  const int wm = wave / NWN, wn = wave % NWN;
  const int M = p.M, N = p.N, K = p.K;
  const f16* __restrict__ A = p.A[g];
  const f16* __restrict__ B = p.B[g];
  const int KT_all = (K + BK - 1) / BK;
  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int kt_end = min(KT_all, kt_begin + p.kt_per_split);

  // Lane -> (row within its 8-row group, LDS chunk); the global k chunk is
  // pre-swizzled so the LDS image is the XOR-swizzled layout the fragment
  // reads expect (swz is an involution).
  const int lrow = lane / CPR, lchunk = lane % CPR;
  uint32_t a_off[AW];   // dense: byte offset of the lane's row chunk at k = 0
  int64_t a_img[AW];    // conv: element offset of the lane's image
  int a_iy0[AW], a_ix0[AW];
  bool a_ok[AW];
  int a_kc[AW];
  // conv: per-row (tap, ci, ky, kx) of the lane's current k, advanced by BK
  // per issued tile (no integer division in the K loop)
  int c_ci[AW], c_ky[AW], c_kx[AW];
#pragma unroll
  for (int j = 0; j < AW; ++j) {
    const int r = (wave * AW + j) * RPI + lrow;
    a_kc[j] = swz<BK>(r, lchunk);
    const int m = m0 + r;
    a_ok[j] = m < M;
    const int mm = a_ok[j] ? m : 0;
    if constexpr (AMODE == kDense) {
      a_off[j] = a_ok[j] ? (uint32_t)(((int64_t)mm * p.lda + a_kc[j] * 8) * 2) : kOOB;
      a_iy0[j] = a_ix0[j] = 0;
      a_img[j] = 0;
    } else {
      const int ox = mm % p.oW, t = mm / p.oW, oy = t % p.oH, b = t / p.oH;
      a_off[j] = 0;
      a_img[j] = (int64_t)b * p.cH * p.cW * p.cC;
      a_iy0[j] = oy * p.st - p.pad;
      a_ix0[j] = ox * p.st - p.pad;
      const int k = (kt_begin + kg) * BK + a_kc[j] * 8, tap = k / p.cC;
      c_ci[j] = k - tap * p.cC;
      c_ky[j] = tap / p.ks;
      c_kx[j] = tap - c_ky[j] * p.ks;
    }
  }
  uint32_t b_off[BW];
  bool b_ok[BW];
  int b_kc[BW];
#pragma unroll
  for (int j = 0; j < BW; ++j) {
    const int r = (wave * BW + j) * RPI + lrow;
    b_kc[j] = swz<BK>(r, lchunk);
    b_ok[j] = (n0 + r) < N;
    b_off[j] = b_ok[j] ? (uint32_t)(((int64_t)(n0 + r) * p.ldb + b_kc[j] * 8) * 2) : kOOB;
  }

  // Buffer resources: operand extents bound the reads (tails read zero).
  const int Bn = AMODE == kDense ? 0 : M / (p.oH * p.oW);
  const __amdgpu_buffer_rsrc_t ra =
      AMODE == kDense ? make_rsrc(A, ((int64_t)(M - 1) * p.lda + K) * 2)
                      : make_rsrc(A, (int64_t)Bn * p.cH * p.cW * p.cC * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, ((int64_t)(N - 1) * p.ldb + K) * 2);
  const bool k_tail = (K % BK) != 0;

  // Issue the LDS-DMA loads of K tile kt into stage st (tiles are issued in
  // order kt = 0, 1, 2, ...: the conv state advances one tile per call).
  f16* const ring = smem + kg * kStages * STAGE;   // this K-group's stages
  auto issue = [&](int kt, int st) {
    f16* As = ring + st * STAGE;
    f16* Bs = As + BM * BK;
    const int k0 = kt * BK;
    const bool tail = k_tail && (k0 + BK > K);   // wave-uniform
#pragma unroll
    for (int j = 0; j < AW; ++j) {
      uint32_t off;
      if constexpr (AMODE == kDense) {
        off = a_off[j];
        if (tail && k0 + a_kc[j] * 8 >= K) off = kOOB;
        if (!(p.debug & 2)) S3_BLDS(ra, As + (wave * AW + j) * 512, off, k0 * 2);
      } else {
        off = kOOB;
        const int iy = a_iy0[j] + c_ky[j], ix = a_ix0[j] + c_kx[j];
        if (a_ok[j] && !(tail && k0 + a_kc[j] * 8 >= K) && iy >= 0 && iy < p.cH && ix >= 0 &&
            ix < p.cW)
          off = (uint32_t)((a_img[j] + ((int64_t)iy * p.cW + ix) * p.cC + c_ci[j]) * 2);
        c_ci[j] += BK * KG;
        while (c_ci[j] >= p.cC) {
          c_ci[j] -= p.cC;
          if (++c_kx[j] == p.ks) { c_kx[j] = 0; ++c_ky[j]; }
        }
        if (!(p.debug & 2)) S3_BLDS(ra, As + (wave * AW + j) * 512, off, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BW; ++j) {
      uint32_t off = b_off[j];
      if (tail && k0 + b_kc[j] * 8 >= K) off = kOOB;
      if (!(p.debug & 2)) S3_BLDS(rb, Bs + (wave * BW + j) * 512, off, k0 * 2);
    }
  };

  typename AT::T acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < AT::R; ++r) acc[i][j][r] = 0.0f;

  // kStages-deep ring per K-group: tiles kt+1 .. kt+kStages-2 stay in
  // flight while tile kt is consumed; one raw barrier per K step.  K-group
  // kg owns the workgroup's K tiles kg, kg + KG, ...; every group runs IT
  // steps (the largest count) so the barriers pair up.
  constexpr int AHEAD = kStages - 1;
  const int KT_wg = (p.debug & 8) ? 0 : kt_end - kt_begin;   // this workgroup's K tiles
  const int KT = KT_wg > kg ? (KT_wg - kg + KG - 1) / KG : 0;  // this K-group's
  const int IT = (KT_wg + KG - 1) / KG;
#pragma unroll
  for (int i = 0; i < AHEAD; ++i)
    if (i < KT) issue(kt_begin + kg + i * KG, i);
  for (int kt = 0; kt < IT; ++kt) {
    // Tile kt has landed once at most (tiles issued after it) x PERW DMA
    // instructions of this wave are still outstanding.
    if (kt < KT) wait_tiles<PERW, AHEAD - 1>(KT - 1 - kt);
    // Everyone's DMA for tile kt is visible, and everyone finished reading
    // the stage that tile kt+AHEAD overwrites (read during iteration kt-1).
    s3::ring_barrier();
    if (kt >= KT) continue;
    const f16* As = ring + (kt % kStages) * STAGE;
    const f16* Bs = As + BM * BK;
    // All fragments of this K tile first (their LDS latency overlaps the
    // next tile's DMA issue below), then the MFMA chain.
    constexpr int NKS = BK / AT::KS;
    f16x8 af[NKS][FM], bf[NKS][FN];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int kc = AT::frag_chunk(ks, lane);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int row = wm * WM + fm * MF + AT::frag_row(lane);
        af[ks][fm] = *reinterpret_cast<const f16x8*>(As + row * BK + swz<BK>(row, kc) * 8);
      }
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int row = wn * WN + fn * MF + AT::frag_row(lane);
        bf[ks][fn] = *reinterpret_cast<const f16x8*>(Bs + row * BK + swz<BK>(row, kc) * 8);
      }
    }
    if (kt + AHEAD < KT) issue(kt_begin + kg + (kt + AHEAD) * KG, (kt + AHEAD) % kStages);
    if (p.debug & 1) continue;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if constexpr (AMODE == kConvRelu) {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            af[ks][fm][e] = af[ks][fm][e] > (f16)0 ? af[ks][fm][e] : (f16)0;
      }
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = AT::mfma(af[ks][fm], bf[ks][fn], acc[fm][fn]);
    }
  }

  // ---- epilogue ----
  if (p.debug & 4) return;
  // the LDS-staged vector epilogue where the fp32 tile fits the ring (one
  // partial-tile slice per K-group, summed in group order inside)
  constexpr bool kVecFits = BM * BN * 4 <= kStages * STAGE * 2;
  if constexpr (kVecFits) {
    if (p.vec_epi) {
      // row pitch BN + 4 floats where it fits (rows 16 B apart in the banks)
      constexpr int LDT = BM * (BN + 4) * 4 <= kStages * STAGE * 2 ? BN + 4 : BN;
      epilogue_vec<BM, BN, NWM, NWN, FM, FN, LDT, KG * kStages * STAGE * 2, KG, MF>(
          p, g, m0, n0, acc, reinterpret_cast<float*>(smem));
      return;
    }
  }
  if constexpr (MF != 32) {
    return;   // host-checked: the 16x16 tiles always take the vector epilogue
  } else {
  if constexpr (KG > 1) {
    // register epilogue: groups 1.. hand their accumulators to group 0
    // through LDS (lane-contiguous), group 0 adds them in group order
    static_assert((KG - 1) * BM * BN * 4 <= KG * kStages * STAGE * 2, "K-group partials in LDS");
    float* part = reinterpret_cast<float*>(smem);
    __syncthreads();
    if (kg > 0) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            part[((((kg - 1) * NW + wave) * FM + fm) * FN + fn) * 1024 + r * 64 + lane] =
                acc[fm][fn][r];
    }
    __syncthreads();
    if (kg > 0) return;
#pragma unroll
    for (int q = 1; q < KG; ++q)
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            acc[fm][fn][r] += part[((((q - 1) * NW + wave) * FM + fm) * FN + fn) * 1024 +
                                   r * 64 + lane];
  }
  epilogue_regs<BM, BN, NWM, NWN, FM, FN>(p, g, m0, n0, acc);
  }
}

// Split-K combine: sum the partial planes in split order, then the epilogue.
// V consecutive columns of one row per thread (16-B plane loads when V = 4,
// host-checked N % 4 == 0); the sum order per element is unchanged.
template <int V>
__global__ void __launch_bounds__(kThreads) k_splitk_reduce(GemmP p) {
  const int g = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * V;
  const int64_t MN = (int64_t)p.M * p.N;
  if (i >= MN) return;
  const float* w = p.ws + (int64_t)g * p.split_k * MN + i;
  if constexpr (V == 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(w);
    for (int s = 1; s < p.split_k; ++s) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(w + s * MN);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += t[j];
    }
    const int row = (int)(i / p.N), col = (int)(i % p.N);
#pragma unroll
    for (int j = 0; j < 4; ++j) epilogue(p, g, row, col + j, v[j]);
  } else {
    float v = w[0];
    for (int s = 1; s < p.split_k; ++s) v += w[s * MN];
    epilogue(p, g, (int)(i / p.N), (int)(i % p.N), v);
  }
}

// Launch geometry shared by the kernel templates: tile counts, split-K
// ranges (no empty splits), tile order and the 2-D XCD partition.
__attribute__((unused)) static GemmP plan_grid(const GemmP& p, int BM, int BN, int BK) {
  GemmP q = p;
  q.tiles_m = (p.M + BM - 1) / BM;
  q.tiles_n = (p.N + BN - 1) / BN;
  const int KT = (p.K + BK - 1) / BK;
  q.split_k = p.split_k > 1 ? p.split_k : 1;
  q.kt_per_split = (KT + q.split_k - 1) / q.split_k;
  q.split_k = (KT + q.kt_per_split - 1) / q.kt_per_split;   // no empty splits
  const int64_t a_bytes = p.a_mode == S3N_A_DENSE ? (int64_t)p.M * p.K
                                                  : (int64_t)p.M / (p.oH * p.oW) * p.cH * p.cW * p.cC;
  q.col_major = (int64_t)p.N * p.K > a_bytes;
  // 2-D XCD partition for dense A: the split px x (8 / px) of the tile grid
  // that minimises the per-XCD operand reads 8 (A / px + B px / 8)
  q.xcd_px = 0;
  if (p.a_mode == S3N_A_DENSE && !(g_xcd_flags & 1)) {
    const double A = (double)p.M * p.K, Bw = (double)p.N * p.K;
    double best = A * 8 + Bw;   // the band split the fallback does (either way)
    best = std::min(best, A + Bw * 8);
    for (int px = 1; px <= 8; px *= 2) {
      const int py = 8 / px;
      if (q.tiles_m % px || q.tiles_n % py) continue;
      const double c = 8.0 * (A / px + Bw / py);
      if (c < best) { best = c; q.xcd_px = px; }
    }
  }
  return q;
}

// The split-K combine launch after a split kernel.
__attribute__((unused)) static int launch_splitk_reduce(const GemmP& q, hipStream_t st) {
  if (q.split_k > 1) {
    if (q.N % 4 == 0) {
      dim3 rg((unsigned)s3::cdiv((int64_t)q.M * q.N / 4, kThreads), q.groups);
      k_splitk_reduce<4><<<rg, kThreads, 0, st>>>(q);
    } else {
      dim3 rg((unsigned)s3::cdiv((int64_t)q.M * q.N, kThreads), q.groups);
      k_splitk_reduce<1><<<rg, kThreads, 0, st>>>(q);
    }
    S3_LAUNCH_CHECK();
  }
  return S3_OK;
}

template <int BM, int BN, int S, int NWM = 2, int NWN = 2, int BK = 64, int KG = 1, int MF = 32>
int launch(const GemmP& p, hipStream_t st) {
  S3_REQUIRE(MF == 32 || p.vec_epi, "s3n_gemm: 16x16 MFMA tiles need the vector epilogue");
  static_assert(MF == 32 || BM * BN * 4 <= S * (BM + BN) * BK * 2,
                "16x16 MFMA tiles stage their fp32 tile in the LDS ring");
  S3_REQUIRE(!p.tail_w[0] || p.N == BN,
             "s3n_gemm: the fused tail needs N == the tile width (%d, N = %d)", BN, p.N);
  S3_REQUIRE(!p.tail_w[0] || BM * BN * 4 <= S * (BM + BN) * BK * 2,
             "s3n_gemm: the fused tail needs a tile whose fp32 image fits its LDS ring");
  S3_REQUIRE(KG == 1 || !p.tail_w[0], "s3n_gemm: the fused tail runs with one K-group");
  constexpr int NT = 64 * NWM * NWN * KG;
  const GemmP q = plan_grid(p, BM, BN, BK);
  dim3 grid(q.tiles_m * q.tiles_n, q.split_k, p.groups);
  if (p.a_mode == S3N_A_DENSE)
    k_gemm<BM, BN, NWM, NWN, kDense, S, BK, KG, MF><<<grid, NT, 0, st>>>(q);
  else if (p.relu_in)
    k_gemm<BM, BN, NWM, NWN, kConvRelu, S, BK, KG, MF><<<grid, NT, 0, st>>>(q);
  else
    k_gemm<BM, BN, NWM, NWN, kConv, S, BK, KG, MF><<<grid, NT, 0, st>>>(q);
  S3_LAUNCH_CHECK();
  return launch_splitk_reduce(q, st);
}



// this translation unit's fp16 saturation flag (g_f16_sat is per code object)
__attribute__((unused)) int read_sat(int reset) {
  uint32_t v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_f16_sat), sizeof(v)) != hipSuccess) return -1;
  if (reset && v) {
    const uint32_t z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_f16_sat), &z, sizeof(z)) != hipSuccess) return -1;
  }
  return v ? 1 : 0;
}

}  // namespace
