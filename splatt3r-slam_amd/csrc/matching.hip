// Dense correspondence kernels behind include/s3m.h.
//
// Restates splatt3r_slam/backend/src/matching_kernels.cu (iter_proj
// :118-274, refine_matches :24-80) and the torch glue of
// splatt3r_slam/matching.py:25-90 / image.py:5-38 as wave64 kernels:
// 256-thread blocks (4 waves) instead of the reference's 16-thread blocks
// (a quarter wave), one query point per lane.  This file is compiled with
// -ffp-contract=off so that the arithmetic is the strict evaluation of the
// reference source text (see s3m.h).
#include "common.hpp"
#include "device_util.hpp"
#include "s3m.h"

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float clampf(float x, float lo, float hi) {
  return fminf(fmaxf(x, lo), hi);
}

// Bilinear sample of channels [c0, c0+3) of the 9-channel ray image at
// (u, v); weights exactly as matching_kernels.cu:150-180 ("pixels are
// opposite the area calc").
struct Taps {
  const float* r11;  // (v11+1, u11+1)
  const float* r12;  // (v11+1, u11)
  const float* r21;  // (v11,   u11+1)
  const float* r22;  // (v11,   u11)
  float w11, w12, w21, w22;
};

__device__ __forceinline__ Taps make_taps(const float* img, int w, float u, float v) {
  Taps t;
  int u11 = (int)floorf(u);
  int v11 = (int)floorf(v);
  float du = u - (float)u11;
  float dv = v - (float)v11;
  t.w11 = du * dv;
  t.w12 = (float)((1.0 - (double)du) * (double)dv);
  t.w21 = (float)((double)du * (1.0 - (double)dv));
  t.w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
  t.r11 = img + ((int64_t)(v11 + 1) * w + (u11 + 1)) * 9;
  t.r12 = img + ((int64_t)(v11 + 1) * w + u11) * 9;
  t.r21 = img + ((int64_t)v11 * w + (u11 + 1)) * 9;
  t.r22 = img + ((int64_t)v11 * w + u11) * 9;
  return t;
}

__device__ __forceinline__ float lerp_ch(const Taps& t, int c) {
  return t.w11 * t.r11[c] + t.w12 * t.r12[c] + t.w21 * t.r21[c] + t.w22 * t.r22[c];
}

__global__ void __launch_bounds__(kBlock)
k_iter_proj(const float* __restrict__ rays_img, const float* __restrict__ pts,
            const float* __restrict__ p_init, float* __restrict__ p_new,
            uint8_t* __restrict__ converged_out, int h, int w, int n,
            int max_iter, float lambda_init, float cost_thresh) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= n) return;
  const float* img = rays_img + b * (int64_t)h * w * 9;
  const int64_t pi = b * (int64_t)n + i;
  float u = clampf(p_init[pi * 2 + 0], 1.0f, (float)(w - 2));
  float v = clampf(p_init[pi * 2 + 1], 1.0f, (float)(h - 2));
  const float p0 = pts[pi * 3 + 0], p1 = pts[pi * 3 + 1], p2 = pts[pi * 3 + 2];

  float lambda = lambda_init;
  bool converged = false;
  for (int it = 0; it < max_iter; ++it) {
    Taps t = make_taps(img, w, u, v);
    float r0 = lerp_ch(t, 0), r1 = lerp_ch(t, 1), r2 = lerp_ch(t, 2);
    float gx0 = lerp_ch(t, 3), gx1 = lerp_ch(t, 4), gx2 = lerp_ch(t, 5);
    float gy0 = lerp_ch(t, 6), gy1 = lerp_ch(t, 7), gy2 = lerp_ch(t, 8);
    float r_norm = sqrtf(r0 * r0 + r1 * r1 + r2 * r2);
    float r_norm_inv = (float)(1.0 / (double)r_norm);
    r0 *= r_norm_inv; r1 *= r_norm_inv; r2 *= r_norm_inv;
    float e0 = r0 - p0, e1 = r1 - p1, e2 = r2 - p2;
    float cost = e0 * e0 + e1 * e1 + e2 * e2;

    float A00 = gx0 * gx0 + gx1 * gx1 + gx2 * gx2;
    float A01 = gx0 * gy0 + gx1 * gy1 + gx2 * gy2;
    float A11 = gy0 * gy0 + gy1 * gy1 + gy2 * gy2;
    float b0 = -(e0 * gx0 + e1 * gx1 + e2 * gx2);
    float b1 = -(e0 * gy0 + e1 * gy1 + e2 * gy2);
    A00 += lambda;
    A11 += lambda;
    float det_inv = (float)(1.0 / (double)(A00 * A11 - A01 * A01));
    float delta_u = det_inv * (A11 * b0 - A01 * b1);
    float delta_v = det_inv * (-A01 * b0 + A00 * b1);

    float u_new = clampf(u + delta_u, 1.0f, (float)(w - 2));
    float v_new = clampf(v + delta_v, 1.0f, (float)(h - 2));

    Taps t2 = make_taps(img, w, u_new, v_new);
    float q0 = lerp_ch(t2, 0), q1 = lerp_ch(t2, 1), q2 = lerp_ch(t2, 2);
    float q_norm = sqrtf(q0 * q0 + q1 * q1 + q2 * q2);
    float q_norm_inv = (float)(1.0 / (double)q_norm);
    q0 *= q_norm_inv; q1 *= q_norm_inv; q2 *= q_norm_inv;
    float f0 = q0 - p0, f1 = q1 - p1, f2 = q2 - p2;
    float new_cost = f0 * f0 + f1 * f1 + f2 * f2;

    if (new_cost < cost) {
      u = u_new;
      v = v_new;
      lambda = (float)((double)lambda * 0.1);
      converged = new_cost < cost_thresh;
    } else {
      lambda = (float)((double)lambda * 10.0);
      converged = cost < cost_thresh;
    }
  }
  p_new[pi * 2 + 0] = u;
  p_new[pi * 2 + 1] = v;
  converged_out[pi] = converged ? 1 : 0;
}

// c10::Half dot product: every product and partial sum rounded to fp16.
// Initial best score: cuda::std::numeric_limits<c10::Half>::min() in the
// reference (:46).  c10::Half has no cuda::std specialisation, so the
// primary template returns Half() == 0; see DESIGN.md "refine_matches".
template <int F>
__global__ void __launch_bounds__(kBlock)
k_refine(const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
         const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h,
         int w, int n, int fdim_rt, int radius, int dilation_max) {
  const int fdim = F > 0 ? F : fdim_rt;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= n) return;
  const int64_t pi = b * (int64_t)n + i;
  const _Float16* d21 = D21 + pi * fdim;
  const _Float16* d11 = D11 + b * (int64_t)h * w * fdim;

  float q[F > 0 ? F : 1];
  if constexpr (F > 0) {
#pragma unroll
    for (int k = 0; k < F; ++k) q[k] = (float)d21[k];
  }

  int64_t u0 = p1[pi * 2 + 0];
  int64_t v0 = p1[pi * 2 + 1];
  _Float16 max_score = (_Float16)0.0f;
  int64_t u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; --d) {
    const int rd = radius * d;
    const int diam = 2 * rd + 1;
    for (int ii = 0; ii < diam; ii += d) {
      for (int jj = 0; jj < diam; jj += d) {
        const int64_t u = u0 - rd + ii;
        const int64_t v = v0 - rd + jj;
        if (v >= 0 && v < h && u >= 0 && u < w) {
          const _Float16* row = d11 + (v * w + u) * fdim;
          _Float16 score = (_Float16)0.0f;
          if constexpr (F > 0) {
#pragma unroll
            for (int k = 0; k < F; ++k) {
              _Float16 prod = (_Float16)(q[k] * (float)row[k]);
              score = (_Float16)((float)score + (float)prod);
            }
          } else {
            for (int k = 0; k < fdim; ++k) {
              _Float16 prod = (_Float16)((float)d21[k] * (float)row[k]);
              score = (_Float16)((float)score + (float)prod);
            }
          }
          if ((float)score > (float)max_score) {
            max_score = score;
            u_new = u;
            v_new = v;
          }
        }
      }
    }
    u0 = u_new;
    v0 = v_new;
  }
  p1_new[pi * 2 + 0] = u_new;
  p1_new[pi * 2 + 1] = v_new;
}

// Cooperative refine: 16 lanes per query point (4 queries per wave).  At
// each dilation level the (2r+1)^2 window candidates are dealt round-robin
// over the 16 lanes in image-row order, every lane issues the descriptor loads of all its
// candidates before any arithmetic (up to 4 x 3 16-B loads in flight per
// lane, instead of one dependent candidate at a time), and a 16-lane
// butterfly picks the level's winner.  Same result as the sequential scan
// of matching_kernels.cu:50-72: the sequential loop keeps the FIRST
// candidate (in (i, j) order) that strictly beats the running maximum, which
// is the smallest-index candidate holding the level's maximum score if that
// score beats the maximum carried in from the previous levels.  The fp16
// dot product keeps the reference's rounding of every product and partial
// sum (v_mul_f16 / v_add_f16, no contraction in this file).
// kRefLanes lanes per query point, kRefMaxPer = 64 / kRefLanes candidate
// slots each -> (2r+1)^2 <= 64, r <= 3.  The result does not depend on the
// split (ties resolve to the smallest candidate index).
template <int F, int kRefLanes = 16>
__global__ void __launch_bounds__(kBlock)
k_refine_coop(const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
              const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h, int w,
              int n, int radius, int dilation_max, const int* __restrict__ perm) {
  constexpr int kRefMaxPer = 64 / kRefLanes;
  static_assert(F % 8 == 0, "16-B descriptor chunks");
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  constexpr int NC = F / 8;
  const int lane = threadIdx.x & (kRefLanes - 1);
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kRefLanes;
  const int64_t b = blockIdx.y;
  const bool live = i < n;                 // dead groups still join the shuffles
  // perm (may be null): visiting order of the queries, see k_refine_bin
  const int64_t pi = b * (int64_t)n + (live ? (perm ? perm[b * (int64_t)n + i] : i) : 0);
  const h8* q8 = reinterpret_cast<const h8*>(D21 + pi * F);
  h8 q[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) q[c] = q8[c];
  const _Float16* d11 = D11 + b * (int64_t)h * w * F;

  const int side = 2 * radius + 1, ncand = side * side;
  int64_t u0 = p1[pi * 2 + 0], v0 = p1[pi * 2 + 1];
  float max_score = 0.0f;                  // Half() == 0, see k_refine
  int64_t u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; --d) {
    const int rd = radius * d;
    h8 row[kRefMaxPer][NC];
    bool ok[kRefMaxPer];
    int cidx[kRefMaxPer];
#pragma unroll
    for (int t = 0; t < kRefMaxPer; ++t) {
      // slot s walks the window row by row (u fastest), so the lanes of a
      // query read neighbouring pixels of one image row; c is the
      // candidate's index in the reference's (i = u outer, j = v inner) scan
      const int s = lane + t * kRefLanes;
      const int jj = s / side, ii = s - jj * side;
      cidx[t] = ii * side + jj;
      const int64_t u = u0 - rd + (int64_t)ii * d, v = v0 - rd + (int64_t)jj * d;
      ok[t] = live && s < ncand && v >= 0 && v < h && u >= 0 && u < w;
      // empty slots (past the window, outside the image) issue no loads
      if (ok[t]) {
        const h8* r8 = reinterpret_cast<const h8*>(d11 + (v * w + u) * F);
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) row[t][cc] = r8[cc];
      } else {
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) row[t][cc] = h8{};
      }
    }
    float best = -INFINITY;
    int best_c = 1 << 30;
#pragma unroll
    for (int t = 0; t < kRefMaxPer; ++t) {
      _Float16 score = (_Float16)0.0f;
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) {
        const h8 prod = q[cc] * row[t][cc];
#pragma unroll
        for (int e = 0; e < 8; ++e) score = score + prod[e];
      }
      const float sc = (float)score;
      if (ok[t] && (sc > best || (sc == best && cidx[t] < best_c))) { best = sc; best_c = cidx[t]; }
    }
#pragma unroll
    for (int m = kRefLanes / 2; m > 0; m >>= 1) {
      const float ob = __shfl_xor(best, m, kRefLanes);
      const int oc = __shfl_xor(best_c, m, kRefLanes);
      if (ob > best || (ob == best && oc < best_c)) { best = ob; best_c = oc; }
    }
    if (best > max_score) {
      max_score = best;
      const int ii = best_c / side, jj = best_c - ii * side;
      u_new = u0 - rd + (int64_t)ii * d;
      v_new = v0 - rd + (int64_t)jj * d;
    }
    u0 = u_new;
    v0 = v_new;
  }
  if (live && lane == 0) {
    p1_new[pi * 2 + 0] = u_new;
    p1_new[pi * 2 + 1] = v_new;
  }
}

// Radius 3 (a 7 x 7 window per dilation level), F = 24, LPQ lanes per query
// point (1, 2 or 4).  Candidate c = i * 7 + j is pixel (u0 - 3d + i d,
// v0 - 3d + j d) (matching_kernels.cu:50-72: i outer, j inner; the first
// candidate that strictly beats the running maximum wins).  Lane s of a
// query takes the window rows j in [s RPL, s RPL + RPL) (RPL = 7, 4, 2) and
// scores its candidates against the maximum carried in from the
// previous levels (rows outer, columns inner: L1 reuse along a row) and
// keeps its subset's largest score and, of those, the smallest c; a
// log2(LPQ)-step butterfly keeps (larger score, then smaller c) -- the
// sequential scan's choice.  Every candidate is loaded with three
// 16-B buffer loads PF candidates ahead of the one being scored, from
// per-level column / row byte-offset tables: an off-image candidate loads an
// in-image pixel (its off-image coordinate's offset is 0) and is masked out
// of the compare, so the loop has no branches.  The fp16 dot product keeps
// the reference's rounding of every product and partial sum (packed
// v_pk_mul_f16 products, then 24 dependent v_add_f16).
template <int LPQ, int PF>
__global__ void __launch_bounds__(kBlock)
k_refine_lane(const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
              const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h, int w,
              int n, int dilation_max, const int* __restrict__ perm) {
  constexpr int F = 24, CH = F / 8, R = 3, SIDE = 2 * R + 1;
  constexpr int RPL = (SIDE + LPQ - 1) / LPQ;   // window rows per lane
  constexpr int PER = SIDE * RPL;               // candidate slots per lane
  static_assert(LPQ == 1 || LPQ == 2 || LPQ == 4, "1, 2 or 4 lanes per query");
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef int i4 __attribute__((ext_vector_type(4)));
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t / LPQ;
  const int sub = (int)(threadIdx.x & (LPQ - 1));
  const int64_t b = blockIdx.y;
  if (LPQ == 1 && i >= n) return;
  const bool live = i < n;                  // dead lanes still join the butterfly
  // perm (may be null): visiting order of the queries, see k_refine_bin
  const int64_t pi = b * (int64_t)n + (live ? (perm ? perm[b * (int64_t)n + i] : i) : 0);
  h2 q[F / 2];
  {
    const i4* q4 = reinterpret_cast<const i4*>(D21 + pi * F);
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const i4 x = q4[k];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // through a scalar: this clang bit-casts a vector-element lvalue
        // from element 0 whatever the index
        const int xe = x[e];
        q[k * 4 + e] = __builtin_bit_cast(h2, xe);
      }
    }
  }
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<_Float16*>(D11 + b * (int64_t)h * w * F), (short)0, (int)((int64_t)h * w * F * 2),
      0x00020000);
  constexpr uint32_t PIX = F * 2;           // bytes per pixel
  const uint32_t rowb = (uint32_t)w * PIX;
  int64_t u0 = p1[pi * 2 + 0], v0 = p1[pi * 2 + 1];
  _Float16 max_score = (_Float16)0.0f;      // Half() == 0, see k_refine
  int64_t u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; --d) {
    const int64_t ub = u0 - R * d, vb = v0 - R * d;
    // column offsets of the whole window, row offsets of this lane's rows
    uint32_t coff[SIDE], roff[RPL], cm = 0, rm = 0;
#pragma unroll
    for (int k = 0; k < SIDE; ++k) {
      const int64_t u = ub + (int64_t)k * d;
      const bool oc = u >= 0 && u < w;
      coff[k] = oc ? (uint32_t)u * PIX : 0u;
      cm |= (uint32_t)oc << k;
    }
#pragma unroll
    for (int x = 0; x < RPL; ++x) {
      const int j = sub * RPL + x;
      const int64_t v = vb + (int64_t)j * d;
      const bool orr = j < SIDE && v >= 0 && v < h;
      roff[x] = orr ? (uint32_t)v * rowb : 0u;
      rm |= (uint32_t)orr << x;
    }
    // slot k = x * SIDE + ii walks this lane's rows outer and the window
    // columns inner: the 7 candidates of one row read one image row at
    // shifts of d pixels, so a wave's loads of a row overlap in the vector
    // L1 (~4.5 KiB of lines per row instead of 7 x 3 KiB from L2); the
    // scan order changes, so ties are resolved on the candidate index
    uint64_t okl = 0;                       // bit k: slot inside the image
#pragma unroll
    for (int x = 0; x < RPL; ++x) okl |= ((rm >> x) & 1u) ? (uint64_t)cm << (x * SIDE) : 0ull;
    i4 rows[PF + 1][CH];
    auto load = [&](int k, i4 (&r)[CH]) {
      const uint32_t off = coff[k % SIDE] + roff[k / SIDE];
#pragma unroll
      for (int kk = 0; kk < CH; ++kk)
        r[kk] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * kk, 0, 0);
    };
#pragma unroll
    for (int p = 0; p < PF; ++p)
      if (p < PER) load(p, rows[p]);
    _Float16 best = max_score;
    int best_c = -1;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (k + PF < PER) load(k + PF, rows[(k + PF) % (PF + 1)]);
      const i4 (&cur)[CH] = rows[k % (PF + 1)];
      // the 12 packed products first (a packed result read by the next
      // instruction costs a wait state), then the dependent sum
      h2 prod[F / 2];
#pragma unroll
      for (int kk = 0; kk < CH; ++kk)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int re = cur[kk][e];
          prod[kk * 4 + e] = q[kk * 4 + e] * __builtin_bit_cast(h2, re);
        }
      _Float16 score = (_Float16)0.0f;
#pragma unroll
      for (int e = 0; e < F / 2; ++e) {
        score = score + prod[e][0];
        score = score + prod[e][1];
      }
      const bool ok = (okl >> k) & 1ull;
      const int c = (k % SIDE) * SIDE + sub * RPL + k / SIDE;
      // best_c == -1 (the carried maximum) is never displaced by a tie
      if (ok && (score > best || (score == best && c < best_c))) {
        best = score;
        best_c = c;
      }
    }
#pragma unroll
    for (int m = 1; m < LPQ; m <<= 1) {
      const _Float16 ob = __builtin_bit_cast(
          _Float16, (short)__shfl_xor((int)__builtin_bit_cast(short, best), m, LPQ));
      const int oc = __shfl_xor(best_c, m, LPQ);
      // best_c == -1 only at the carried maximum, which no improving lane ties
      if (ob > best || (ob == best && oc < best_c)) {
        best = ob;
        best_c = oc;
      }
    }
    if (best_c >= 0) {
      max_score = best;
      const int ii = best_c / SIDE, jj = best_c - ii * SIDE;
      u_new = ub + (int64_t)ii * d;
      v_new = vb + (int64_t)jj * d;
    }
    u0 = u_new;
    v0 = v_new;
  }
  if (live && sub == 0) {
    p1_new[pi * 2 + 0] = u_new;
    p1_new[pi * 2 + 1] = v_new;
  }
}

// Pixel-major refine: 3 lanes per candidate pixel, one 16-B chunk (8 of the
// 24 fp16 descriptor values) each.  Radius 3, F = 24.  A query's 21 lanes
// are 7 triplets, triplet t owning window column i = t (u = ub + t d); 3
// queries per wave (lane 63 idles).  Per dilation level the wave moves the
// window into LDS by LDS-DMA one window row at a time: row j's instruction
// has triplet t read pixel (u_t, v_j) as 48 contiguous bytes, so a query's
// row is 7 x 48 B of one image row (contiguous at d = 1) -- about a third of
// the 64-B segments per load of the candidate-per-lane kernels, which the
// texture addresser bounds (profiles/r05j_refine_counters.txt).
//
// The reference's strict fp16 chain (matching_kernels.cu:55-64: every
// product and every partial sum rounded to fp16, elements 0..23 in order)
// runs systolically over the triplet: at step s member c scores chunk c of
// window row j = s - c, starting from the partial sum member c - 1 produced
// for the same pixel one step earlier (handed over by a wave_shr:1 DPP move;
// member 0 starts from 0).  Member 2 finishes row s - 2 and keeps its
// column's first strictly larger score (rows in scan order); the 7 columns
// are then merged keeping the larger score and, on a tie, the smaller
// column -- the sequential scan's first maximum (c = i 7 + j, i outer).
// Same rule against the maximum carried in from the coarser levels.
__global__ void __launch_bounds__(kBlock)
k_refine_px(const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
            const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h, int w, int n,
            int dilation_max, const int* __restrict__ perm) {
  constexpr int F = 24, R = 3, SIDE = 2 * R + 1, QPW = 3, LPQ = 3 * SIDE;
  constexpr int WAVES = kBlock / 64;
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef int i4 __attribute__((ext_vector_type(4)));
  // window rows of every wave: [wave][row j][lane] 16 B (the LDS-DMA image)
  __shared__ __attribute__((aligned(1024))) i4 win[WAVES][SIDE][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int qw = lane / LPQ;               // query of the wave (3: the idle lane)
  const int r = lane - qw * LPQ;
  const int base = qw * LPQ;               // the query's first lane
  const int t = r / 3, c = r - 3 * (r / 3);
  const int64_t i = ((int64_t)blockIdx.x * WAVES + wave) * QPW + qw;
  const int64_t b = blockIdx.y;
  const bool live = qw < QPW && i < n;
  const int64_t pi = b * (int64_t)n + (live ? (perm ? perm[b * (int64_t)n + i] : i) : 0);
  // this member's 8 query values
  h2 q[4];
  {
    const i4 x = *reinterpret_cast<const i4*>(D21 + pi * F + c * 8);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int xe = x[e];
      q[e] = __builtin_bit_cast(h2, xe);
    }
  }
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<_Float16*>(D11 + b * (int64_t)h * w * F), (short)0, (int)((int64_t)h * w * F * 2),
      0x00020000);
  constexpr int PIX = F * 2;
  constexpr uint32_t kOff = 0x80000000u;   // out of range: the DMA writes zeros
  // image coordinates fit 32 bits (refine_lane_ok: h w F 2 < 2^31)
  int u0 = (int)p1[pi * 2 + 0], v0 = (int)p1[pi * 2 + 1];
  _Float16 max_score = (_Float16)0.0f;      // Half() == 0, see k_refine
  int u_new = u0, v_new = v0;
  // this lane's slot of window row 0 (row j is 64 slots further)
  i4* const wl = &win[wave][0][lane];
  for (int d = dilation_max; d > 0; --d) {
    const int ub = u0 - R * d, vb = v0 - R * d;
    const int u = ub + t * d;
    const bool ou = live && (unsigned)u < (unsigned)w;
    const int row_step = d * w * PIX;
    int off = (vb * w + u) * PIX + 16 * c;  // pixel (u, v_0), chunk c (used when in range)
    uint32_t okr = 0;                       // bit j: pixel (u, v_j) inside the image
#pragma unroll
    for (int j = 0; j < SIDE; ++j) {
      const bool ok = ou && (unsigned)(vb + j * d) < (unsigned)h;
      okr |= (uint32_t)ok << j;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)&win[wave][j][0], 16,
          ok ? off : (int)kOff, 0, 0, 0);
      off += row_step;
    }
    // bit s: member 2 compares at step s (its row s - 2 is inside the image)
    const uint32_t cmpm = c == 2 ? okr << 2 : 0u;
    _Float16 best = max_score;
    int best_j = -1;
    _Float16 carry = (_Float16)0.0f;
#pragma unroll
    for (int s = 0; s < SIDE + 2; ++s) {
      // step s reads window rows <= s: this wave's DMA of row s has landed
      // once at most 6 - s of its row instructions are outstanding (in order)
      if (s == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (s == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if (s == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (s == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (s == 4) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (s == 5) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else if (s == 6) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int j = s - c;                  // this member's window row
      const int jc = j < 0 ? 0 : (j >= SIDE ? SIDE - 1 : j);
      const i4 x = wl[jc * 64];
      _Float16 sc = c == 0 ? (_Float16)0.0f : carry;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int xe = x[e];
        const h2 prod = q[e] * __builtin_bit_cast(h2, xe);
        sc = sc + prod[0];
        sc = sc + prod[1];
      }
      if (s >= 2 && ((cmpm >> s) & 1u) && sc > best) {
        best = sc;
        best_j = s - 2;
      }
      if (s + 1 < SIDE + 2) {
        // hand the partial sum to the next member (lane + 1)
        const int scb = (int)__builtin_bit_cast(unsigned short, sc);
        const int nb = __builtin_amdgcn_update_dpp(0, scb, 0x138, 0xf, 0xf, false);   // wave_shr:1
        carry = __builtin_bit_cast(_Float16, (unsigned short)nb);
      }
    }
    // merge the 7 columns (member-2 lanes, 3 apart): larger score, the
    // smaller column on a tie (a column with best_j >= 0 beat the carried
    // maximum); a tree over columns t, t+1 | t+2 | t+4, then lane t = 0's
    // result to the query's 21 lanes.  key = score bits << 16 | j << 8 | t
    int key = ((int)__builtin_bit_cast(unsigned short, best) << 16) | ((best_j & 0xff) << 8) | t;
#pragma unroll
    for (int k = 1; k < SIDE; k <<= 1) {
      const int o = __shfl_down(key, 3 * k, 64);
      const int oj = (int)(signed char)((o >> 8) & 0xff);
      const int kj = (int)(signed char)((key >> 8) & 0xff);
      const _Float16 os = __builtin_bit_cast(_Float16, (unsigned short)((o >> 16) & 0xffff));
      const _Float16 ks = __builtin_bit_cast(_Float16, (unsigned short)((key >> 16) & 0xffff));
      if (t + k < SIDE && oj >= 0 && (kj < 0 || os > ks)) key = o;
    }
    key = __shfl(key, base + 2, 64);
    const int lj = (int)(signed char)((key >> 8) & 0xff);
    if (lj >= 0) {
      max_score = __builtin_bit_cast(_Float16, (unsigned short)((key >> 16) & 0xffff));
      u_new = ub + (key & 0xff) * d;
      v_new = vb + lj * d;
    }
    u0 = u_new;
    v0 = v_new;
  }
  if (live && r == 0) {
    p1_new[pi * 2 + 0] = u_new;
    p1_new[pi * 2 + 1] = v_new;
  }
}

// Window-centre binning ahead of the refine.  On the
// tracking loop the queries' window centres scatter (pixel order puts 64
// queries of one frame row on 64 columns and several rows of the keyframe),
// so the lanes of a wave each pull their own cache lines.  Visiting the
// queries in the order of the 2^sx x 2^sy pixel tile that holds their p1
// makes a wave's windows overlap: candidate k of every lane falls in one
// tile-sized patch, shifted by the candidate offset, and the loads of the
// wave share lines in the vector L1.  Counting sort in three launches: bin
// (tile count + arrival rank), scan (tile offsets; re-zeroes the counts for
// the next call), scatter (perm[offset + rank] = query).  Batch b's tiles
// follow batch b-1's, so batch b's queries occupy perm[b n, (b+1) n).  The
// order inside a tile is the atomic arrival order: a query's result depends
// on its own inputs only, so every order gives the same bits.
__device__ __forceinline__ int refine_tile(const int64_t* __restrict__ p1, int64_t pi, int h,
                                           int w, int sx, int sy, int tiles_x) {
  const int64_t u = p1[pi * 2 + 0], v = p1[pi * 2 + 1];
  const int uc = (int)(u < 0 ? 0 : (u >= w ? w - 1 : u));
  const int vc = (int)(v < 0 ? 0 : (v >= h ? h - 1 : v));
  return (vc >> sy) * tiles_x + (uc >> sx);
}

__global__ void __launch_bounds__(kBlock)
k_refine_bin(const int64_t* __restrict__ p1, int* __restrict__ cnt, int* __restrict__ rank, int h,
             int w, int n, int sx, int sy, int tiles_x, int tiles) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= n) return;
  const int64_t pi = b * (int64_t)n + i;
  rank[pi] = atomicAdd(&cnt[b * tiles + refine_tile(p1, pi, h, w, sx, sy, tiles_x)], 1);
}

constexpr int kScanBlock = 1024;

// exclusive scan of the tile counts of every batch (one workgroup; a
// contiguous run of tiles per thread), counts reset to zero
__global__ void __launch_bounds__(kScanBlock)
k_refine_scan(int* __restrict__ cnt, int* __restrict__ off, int total) {
  __shared__ int wsum[kScanBlock / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int per = (total + kScanBlock - 1) / kScanBlock;
  const int lo = t * per, hi = min(lo + per, total);
  int s = 0;
  for (int k = lo; k < hi; ++k) s += cnt[k];
  int x = s;                                  // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  int run = x - s;
  for (int k = 0; k < wv; ++k) run += wsum[k];
  for (int k = lo; k < hi; ++k) {
    const int c = cnt[k];
    off[k] = run;
    run += c;
    cnt[k] = 0;
  }
}

__global__ void __launch_bounds__(kBlock)
k_refine_scatter(const int64_t* __restrict__ p1, const int* __restrict__ rank,
                 const int* __restrict__ off, int* __restrict__ perm, int h, int w, int n, int sx,
                 int sy, int tiles_x, int tiles) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= n) return;
  const int64_t pi = b * (int64_t)n + i;
  perm[off[b * tiles + refine_tile(p1, pi, h, w, sx, sy, tiles_x)] + rank[pi]] = (int)i;
}

// |x| / max(||x||, 1e-12) (F.normalize), strict order ((x0^2+x1^2)+x2^2).
__device__ __forceinline__ void normalize3(const float* x, float* o) {
  float nrm = sqrtf(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  float d = fmaxf(nrm, 1e-12f);
  o[0] = x[0] / d; o[1] = x[1] / d; o[2] = x[2] / d;
}

__device__ __forceinline__ int reflect(int i, int n) {
  return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

// prep_for_iter_proj: one thread per pixel of X11 / X21.
__global__ void __launch_bounds__(kBlock)
k_prep(const float* __restrict__ X11, const float* __restrict__ X21,
       const int64_t* __restrict__ idx_init, float* __restrict__ rays_out,
       float* __restrict__ pts_out, float* __restrict__ p_init, int h, int w) {
  const int64_t hw = (int64_t)h * w;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= hw) return;
  const int y = (int)(i / w), x = (int)(i % w);
  const float* X = X11 + b * hw * 3;
  float r[3][3][3];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      int yy = reflect(y + dy - 1, h), xx = reflect(x + dx - 1, w);
      normalize3(X + ((int64_t)yy * w + xx) * 3, r[dy][dx]);
    }
  float* o = rays_out + (b * hw + i) * 9;
  const float k3 = 3.0f / 32.0f, k10 = 10.0f / 32.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    o[c] = r[1][1][c];
    // Scharr x: [[-3,0,3],[-10,0,10],[-3,0,3]]/32, row-major tap order.
    float gx = -k3 * r[0][0][c] + k3 * r[0][2][c] - k10 * r[1][0][c] +
               k10 * r[1][2][c] - k3 * r[2][0][c] + k3 * r[2][2][c];
    // Scharr y: [[-3,-10,-3],[0,0,0],[3,10,3]]/32.
    float gy = -k3 * r[0][0][c] - k10 * r[0][1][c] - k3 * r[0][2][c] +
               k3 * r[2][0][c] + k10 * r[2][1][c] + k3 * r[2][2][c];
    o[3 + c] = gx;
    o[6 + c] = gy;
  }
  float pn[3];
  normalize3(X21 + (b * hw + i) * 3, pn);
  pts_out[(b * hw + i) * 3 + 0] = pn[0];
  pts_out[(b * hw + i) * 3 + 1] = pn[1];
  pts_out[(b * hw + i) * 3 + 2] = pn[2];
  int64_t lin = idx_init ? idx_init[b * hw + i] : i;
  p_init[(b * hw + i) * 2 + 0] = (float)(lin % w);
  p_init[(b * hw + i) * 2 + 1] = (float)(lin / w);
}

__global__ void __launch_bounds__(kBlock)
k_occlusion(const float* __restrict__ p, const uint8_t* __restrict__ conv,
            const float* __restrict__ X11, const float* __restrict__ X21,
            int64_t* __restrict__ p1, uint8_t* __restrict__ valid, int h, int w,
            float dist_thresh) {
  const int64_t hw = (int64_t)h * w;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= hw) return;
  const int64_t pi = b * hw + i;
  int64_t u = (int64_t)p[pi * 2 + 0];
  int64_t v = (int64_t)p[pi * 2 + 1];
  p1[pi * 2 + 0] = u;
  p1[pi * 2 + 1] = v;
  const float* a = X11 + (b * hw + v * w + u) * 3;
  const float* c = X21 + pi * 3;
  float d0 = a[0] - c[0], d1 = a[1] - c[1], d2 = a[2] - c[2];
  float dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
  valid[pi] = (conv[pi] && dist < dist_thresh) ? 1 : 0;
}

__global__ void k_pixel_to_lin(const int64_t* __restrict__ p1, int64_t* __restrict__ idx,
                               int64_t count, int w) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  idx[i] = p1[i * 2 + 0] + (int64_t)w * p1[i * 2 + 1];
}

}  // namespace

extern "C" {

int s3m_iter_proj(const float* rays_img_with_grad, const float* pts_3d_norm,
                  const float* p_init, float* p_new, uint8_t* converged, int b,
                  int h, int w, int n, int max_iter, float lambda_init,
                  float cost_thresh, void* stream) {
  S3_REQUIRE(b >= 0 && n >= 0 && h >= 3 && w >= 3 && max_iter >= 0,
             "s3m_iter_proj: bad shape b=%d h=%d w=%d n=%d", b, h, w, n);
  if (b == 0 || n == 0) return S3_OK;
  dim3 grid((unsigned)s3::cdiv(n, kBlock), (unsigned)b);
  k_iter_proj<<<grid, kBlock, 0, s3::as_stream(stream)>>>(
      rays_img_with_grad, pts_3d_norm, p_init, p_new, converged, h, w, n,
      max_iter, lambda_init, cost_thresh);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

// lanes per query point of the refine: 1, 2 or 4 (k_refine_lane, radius 3,
// F = 24), 3 (k_refine_px, radius 3, F = 24: 3 lanes per window pixel, the
// default) or 8 / 16 / 32 / 64 (k_refine_coop), and the
// lane kernel's load distance in candidates (2, 3, 4 or 6); tuning hooks for
// A/B runs.  The per-lane kernel wins when neighbouring query points have
// neighbouring windows (129 vs 173 us at C2 on a clean 2-px shift,
// tools/bench_match.py); on the tracking loop's matches, whose window
// centres scatter (median row spread 3-6 px per 64 queries, 46-68 px on
// every other call: tools/refine_stats.py), its lanes touch one cache line
// each and the 16-lane kernel is faster (185 vs 208 us per call,
// profiles/r04g_summary.txt)
// round 6: the pixel-major kernel (3 lanes per pixel, k_refine_px) is the
// default: 161-180 vs 176-197 us on the tracking loop's inputs
// (profiles/r06e_refine_px.log)
constexpr int kRefineLanesDefault = 3;
// window-centre binning: 0 = off (pixel order), else 16 sx + sy for
// 2^sx x 2^sy pixel tiles (k_refine_bin)
constexpr int kRefineSortDefault = 0;
static int g_refine_lanes = kRefineLanesDefault;
static int g_refine_pf = 4;
static int g_refine_sort = kRefineSortDefault;
// (any other value, e.g. -1: the default)
extern "C" void s3m_refine_set_lanes(int lanes) {
  g_refine_lanes = (lanes == 1 || lanes == 2 || lanes == 3 || lanes == 4 || lanes == 8 ||
                    lanes == 16 || lanes == 32 || lanes == 64)
                       ? lanes : kRefineLanesDefault;
}
extern "C" void s3m_refine_set_prefetch(int pf) {
  g_refine_pf = (pf == 2 || pf == 3 || pf == 6) ? pf : 4;
}
extern "C" void s3m_refine_set_sort(int mode) {
  const int sx = mode >> 4, sy = mode & 15;
  g_refine_sort = mode == 0 ? 0 : (mode > 0 && sx <= 6 && sy <= 6) ? mode : kRefineSortDefault;
}

}  // extern "C"

// Device scratch of the binning, one per (device, stream): tile counts
// (kept zero between calls: the scan resets them), tile offsets, arrival
// ranks and the visiting order.  Grown (to the next power of two), never
// shrunk.  Growing is refused while the stream is being captured (an
// allocation is not capturable); otherwise the stream is drained first, so
// the outgrown buffers, which only work queued on this stream reads, are
// freed, not leaked.  The first call at the largest batch size should come
// before any capture (the binning is off by default, s3m_refine_set_sort).
struct RefineScratch {
  int* cnt = nullptr;
  int* off = nullptr;
  int* rank = nullptr;
  int* perm = nullptr;
  int64_t queries = 0, tiles = 0;
};
static std::mutex g_scratch_mu;
static std::map<std::pair<int, hipStream_t>, RefineScratch> g_scratch;

static int refine_scratch(hipStream_t st, int64_t queries, int64_t tiles, RefineScratch* out) {
  int dev = 0;
  S3_HIP(s3::stream_device(st, &dev));
  s3::DeviceGuard guard(dev);   // allocations on the stream's device
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  RefineScratch& s = g_scratch[{dev, st}];
  if (s.tiles < tiles || s.queries < queries) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    S3_HIP(hipStreamIsCapturing(st, &cs));
    S3_REQUIRE(cs == hipStreamCaptureStatusNone,
               "s3m_refine_matches: the binning scratch must grow (%lld queries, %lld tiles) "
               "while the stream is being captured; run one call at this size first",
               (long long)queries, (long long)tiles);
    S3_HIP(hipStreamSynchronize(st));   // queued reads of the old buffers are done
  }
  if (s.tiles < tiles) {
    int64_t t = 4096;
    while (t < tiles) t *= 2;
    if (s.cnt) S3_HIP(hipFree(s.cnt));
    if (s.off) S3_HIP(hipFree(s.off));
    s.cnt = s.off = nullptr;
    s.tiles = 0;
    S3_HIP(hipMalloc(&s.cnt, t * sizeof(int)));
    S3_HIP(hipMalloc(&s.off, t * sizeof(int)));
    S3_HIP(hipMemsetAsync(s.cnt, 0, t * sizeof(int), st));
    s.tiles = t;
  }
  if (s.queries < queries) {
    int64_t q = 1 << 16;
    while (q < queries) q *= 2;
    if (s.rank) S3_HIP(hipFree(s.rank));
    if (s.perm) S3_HIP(hipFree(s.perm));
    s.rank = s.perm = nullptr;
    s.queries = 0;
    S3_HIP(hipMalloc(&s.rank, q * sizeof(int)));
    S3_HIP(hipMalloc(&s.perm, q * sizeof(int)));
    s.queries = q;
  }
  *out = s;
  return S3_OK;
}

// the visiting order of the b x n queries (k_refine_bin), or null when
// binning is off or the batch is too small to gain from it
static int refine_order(const int64_t* p1, int b, int h, int w, int n, hipStream_t st,
                        const int** perm) {
  *perm = nullptr;
  if (g_refine_sort == 0 || (int64_t)b * n < 2048) return S3_OK;
  const int sx = g_refine_sort >> 4, sy = g_refine_sort & 15;
  const int tiles_x = (int)s3::cdiv(w, 1 << sx), tiles = tiles_x * (int)s3::cdiv(h, 1 << sy);
  const int64_t total = (int64_t)b * tiles;
  S3_REQUIRE(total < (1 << 26) && (int64_t)b * n < 0x7fffffff, "s3m_refine_matches: batch too large to bin");
  RefineScratch s;
  const int rc = refine_scratch(st, (int64_t)b * n, total, &s);
  if (rc != S3_OK) return rc;
  dim3 grid((unsigned)s3::cdiv(n, kBlock), (unsigned)b);
  k_refine_bin<<<grid, kBlock, 0, st>>>(p1, s.cnt, s.rank, h, w, n, sx, sy, tiles_x, tiles);
  k_refine_scan<<<1, kScanBlock, 0, st>>>(s.cnt, s.off, (int)total);
  k_refine_scatter<<<grid, kBlock, 0, st>>>(p1, s.rank, s.off, s.perm, h, w, n, sx, sy, tiles_x,
                                            tiles);
  S3_LAUNCH_CHECK();
  *perm = s.perm;
  return S3_OK;
}

template <int LPQ>
static void launch_refine_lane(const _Float16* d11, const _Float16* d21, const int64_t* p1,
                               int64_t* p1_new, int b, int h, int w, int n, int dilation_max,
                               const int* perm, hipStream_t st) {
  dim3 grid((unsigned)s3::cdiv((int64_t)n * LPQ, kBlock), (unsigned)b);
  switch (g_refine_pf) {
    case 2: k_refine_lane<LPQ, 2><<<grid, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, dilation_max, perm); break;
    case 4: k_refine_lane<LPQ, 4><<<grid, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, dilation_max, perm); break;
    case 6: k_refine_lane<LPQ, 6><<<grid, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, dilation_max, perm); break;
    default: k_refine_lane<LPQ, 3><<<grid, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, dilation_max, perm); break;
  }
}

static void refine_lane(const _Float16* d11, const _Float16* d21, const int64_t* p1,
                        int64_t* p1_new, int b, int h, int w, int n, int dilation_max,
                        const int* perm, hipStream_t st) {
  if (g_refine_lanes == 4)
    launch_refine_lane<4>(d11, d21, p1, p1_new, b, h, w, n, dilation_max, perm, st);
  else if (g_refine_lanes == 2)
    launch_refine_lane<2>(d11, d21, p1, p1_new, b, h, w, n, dilation_max, perm, st);
  else
    launch_refine_lane<1>(d11, d21, p1, p1_new, b, h, w, n, dilation_max, perm, st);
}

// the per-lane kernel: radius 3, fdim 24, one image of D11 addressable
// with 32-bit buffer offsets
static bool refine_lane_ok(int h, int w, int fdim, int radius) {
  return radius == 3 && fdim == 24 && (int64_t)h * w * fdim * 2 < 0x7fffffff;
}

extern "C" {

int s3m_refine_matches(const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                       int64_t* p1_new, int b, int h, int w, int n, int fdim,
                       int radius, int dilation_max, void* stream) {
  S3_REQUIRE(b >= 0 && n >= 0 && h > 0 && w > 0 && fdim > 0 && radius >= 0 &&
                 dilation_max >= 0,
             "s3m_refine_matches: bad shape");
  if (b == 0 || n == 0) return S3_OK;
  dim3 grid((unsigned)s3::cdiv(n, kBlock), (unsigned)b);
  auto d11 = reinterpret_cast<const _Float16*>(D11);
  auto d21 = reinterpret_cast<const _Float16*>(D21);
  auto st = s3::as_stream(stream);
  const int side = 2 * radius + 1;
  const bool px_k = g_refine_lanes == 3 && refine_lane_ok(h, w, fdim, radius);
  const bool lane_k = !px_k && g_refine_lanes <= 4 && refine_lane_ok(h, w, fdim, radius);
  const bool coop_k = side * side <= 64 && (fdim == 24 || fdim == 16 || fdim == 32);
  const int* perm = nullptr;
  if (px_k || lane_k || coop_k) {
    const int rc = refine_order(p1, b, h, w, n, st, &perm);
    if (rc != S3_OK) return rc;
  }
  if (px_k) {
    // 3 queries per wave, 4 waves per workgroup
    dim3 pg((unsigned)s3::cdiv(n, 3 * (kBlock / 64)), (unsigned)b);
    k_refine_px<<<pg, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, dilation_max, perm);
  } else if (lane_k) {
    refine_lane(d11, d21, p1, p1_new, b, h, w, n, dilation_max, perm, st);
  } else if (coop_k) {
    const int lanes = g_refine_lanes <= 4 ? 16 : g_refine_lanes;   // other radius / fdim
    dim3 cg((unsigned)s3::cdiv((int64_t)n * lanes, kBlock), (unsigned)b);
    auto go = [&](auto tag) {
      constexpr int F = decltype(tag)::value;
      if (lanes == 8)
        k_refine_coop<F, 8><<<cg, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, radius, dilation_max, perm);
      else if (lanes == 32)
        k_refine_coop<F, 32><<<cg, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, radius, dilation_max, perm);
      else if (lanes == 64)
        k_refine_coop<F, 64><<<cg, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, radius, dilation_max, perm);
      else
        k_refine_coop<F, 16><<<cg, kBlock, 0, st>>>(d11, d21, p1, p1_new, h, w, n, radius, dilation_max, perm);
    };
    if (fdim == 24) go(std::integral_constant<int, 24>{});
    else if (fdim == 16) go(std::integral_constant<int, 16>{});
    else go(std::integral_constant<int, 32>{});
  } else if (fdim == 24)
    k_refine<24><<<grid, kBlock, 0, s3::as_stream(stream)>>>(
        d11, d21, p1, p1_new, h, w, n, fdim, radius, dilation_max);
  else
    k_refine<0><<<grid, kBlock, 0, s3::as_stream(stream)>>>(
        d11, d21, p1, p1_new, h, w, n, fdim, radius, dilation_max);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3m_prep_iter_proj(const float* X11, const float* X21, const int64_t* idx_init,
                       float* rays_with_grad, float* pts_norm, float* p_init,
                       int b, int h, int w, void* stream) {
  S3_REQUIRE(b >= 0 && h >= 2 && w >= 2, "s3m_prep_iter_proj: bad shape");
  if (b == 0) return S3_OK;
  dim3 grid((unsigned)s3::cdiv((int64_t)h * w, kBlock), (unsigned)b);
  k_prep<<<grid, kBlock, 0, s3::as_stream(stream)>>>(X11, X21, idx_init, rays_with_grad,
                                                    pts_norm, p_init, h, w);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3m_occlusion(const float* p, const uint8_t* converged, const float* X11,
                  const float* X21, int64_t* p1, uint8_t* valid, int b, int h,
                  int w, float dist_thresh, void* stream) {
  S3_REQUIRE(b >= 0 && h > 0 && w > 0, "s3m_occlusion: bad shape");
  if (b == 0) return S3_OK;
  dim3 grid((unsigned)s3::cdiv((int64_t)h * w, kBlock), (unsigned)b);
  k_occlusion<<<grid, kBlock, 0, s3::as_stream(stream)>>>(p, converged, X11, X21, p1, valid,
                                                         h, w, dist_thresh);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3m_pixel_to_lin(const int64_t* p1, int64_t* idx, int64_t count, int w, void* stream) {
  S3_REQUIRE(count >= 0 && w > 0, "s3m_pixel_to_lin: bad shape");
  if (count == 0) return S3_OK;
  k_pixel_to_lin<<<(unsigned)s3::cdiv(count, kBlock), kBlock, 0, s3::as_stream(stream)>>>(
      p1, idx, count, w);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

}  // extern "C"
