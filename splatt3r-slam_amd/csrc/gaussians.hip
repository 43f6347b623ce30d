// gaussians_to_world for one predicted view (include/s3w.h).
//
// Multi-pass path (n > kSelMax: the stride-1 views, 196,608 Gaussians at
// 512x384), hand-written, no library sort or scan:
// k_prep       strided gather of z -> order-preserving uint32 keys
//              ("z > depth_min", 0xffffffff otherwise) and the valid count
// k_sel_hist / k_sel_pick
//              the two order statistics torch.quantile (linear) needs, by a
//              radix select: 4 passes of 8-bit digits, per-block LDS
//              histograms of the keys still matching each rank's prefix,
//              one workgroup picks the digit (integer counts: exact)
// k_flags      quantile bound + scale / confidence filters, per-block kept
//              counts
// k_scan_blocks  exclusive scan of the block counts (one workgroup) and
//              the total
// k_emit       block-local scan of the flags + the block's offset (stable
//              compaction order): world transform, covariance, colour,
//              opacity -> 13-float records
// All stream-ordered; the only host-visible result is *count_dev.
//
// Map buffer (SharedGaussians, frame.py:357-463):
// k_map_flags  opacity > threshold over the valid records, block counts
// k_scan_blocks  (record-order compaction)
// k_map_evict  if full: newest half -> front (one grid-stride copy), and the
//              post-eviction count for the append
// k_map_emit   scatter kept records into the SoA map, update the count
#include <algorithm>

#include "common.hpp"
#include "s3w.h"

namespace {

constexpr int kThreads = 256;
constexpr float kC0 = 0.28209479177387814f;

struct Ws {
  uint32_t* keys;     // fkey(z) / 0xffffffff, per Gaussian
  uint32_t* flags;    // kept, per Gaussian
  uint32_t* bsum;     // per-block kept counts -> exclusive block offsets; [nblk] = total
  uint32_t* hist;     // [2][256] select histograms
  uint32_t* sel;      // [0..3] (prefix, remaining rank) of the two ranks, [4] n0
};

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

int64_t nblocks(int64_t n) { return (n + kThreads - 1) / kThreads; }

size_t ws_bytes(int64_t n) {
  return 2 * align256(sizeof(uint32_t) * n) + align256(sizeof(uint32_t) * (nblocks(n) + 1)) +
         align256(sizeof(uint32_t) * 512) + 256;
}

Ws carve(void* base, int64_t n) {
  char* p = static_cast<char*>(base);
  Ws w;
  w.keys = (uint32_t*)p;  p += align256(sizeof(uint32_t) * n);
  w.flags = (uint32_t*)p; p += align256(sizeof(uint32_t) * n);
  w.bsum = (uint32_t*)p;  p += align256(sizeof(uint32_t) * (nblocks(n) + 1));
  w.hist = (uint32_t*)p;  p += align256(sizeof(uint32_t) * 512);
  w.sel = (uint32_t*)p;
  return w;
}

struct Grid {
  int H, W, s, ws;
  __device__ int64_t pix(int64_t i) const {
    const int64_t y = (i / ws) * s, x = (i % ws) * s;
    return y * W + x;
  }
};

// The three splash filters of one Gaussian (splatt3r_utils.py:296-312).
__device__ __forceinline__ bool keep(int64_t p, const float* __restrict__ means,
                                     const float* __restrict__ scales,
                                     const float* __restrict__ conf, float depth_min, bool use_q,
                                     float zq, float max_scale, float min_conf) {
  const float z = means[p * 3 + 2];
  bool v = z > depth_min;
  if (use_q) v = v && (z <= zq);
  // torch max propagates NaN
  float m = scales[p * 3 + 0];
  const float s1 = scales[p * 3 + 1], s2 = scales[p * 3 + 2];
  if (!(s1 <= m) && !isnan(m)) m = s1;
  if (!(s2 <= m) && !isnan(m)) m = s2;
  v = v && (m < max_scale);
  if (conf && min_conf > 0.0f) v = v && (conf[p] >= min_conf);
  return v;
}

// One world record (13 floats) of the Gaussian at pixel p: world transform,
// covariance, colour, opacity (shared by both paths, so they agree bit for
// bit).
__device__ __forceinline__ void emit_record(const s3w_view& v, const Grid& g,
                                            const float* __restrict__ T44, int64_t p,
                                            float* __restrict__ o) {
  // T44: row-major [4,4] (s R | t); M[0..8] = s R, M[9..11] = t
  float M[12];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) M[r * 3 + c] = T44[r * 4 + c];
    M[9 + r] = T44[r * 4 + 3];
  }
  const float x = v.means[p * 3 + 0], y = v.means[p * 3 + 1], z = v.means[p * 3 + 2];
  for (int r = 0; r < 3; ++r) o[r] = (M[r * 3 + 0] * x + M[r * 3 + 1] * y + M[r * 3 + 2] * z) + M[9 + r];
  // quaternion_to_matrix (xyzw, two_s = 2 / (|q|^2 + 1e-8)), utils/geometry.py:24-49
  const float qi = v.rotations[p * 4 + 0], qj = v.rotations[p * 4 + 1];
  const float qk = v.rotations[p * 4 + 2], qr = v.rotations[p * 4 + 3];
  const float two_s = 2.0f / ((qi * qi + qj * qj + qk * qk + qr * qr) + 1e-8f);
  const float R[9] = {1 - two_s * (qj * qj + qk * qk), two_s * (qi * qj - qk * qr),
                      two_s * (qi * qk + qj * qr),     two_s * (qi * qj + qk * qr),
                      1 - two_s * (qi * qi + qk * qk), two_s * (qj * qk - qi * qr),
                      two_s * (qi * qk - qj * qr),     two_s * (qj * qk + qi * qr),
                      1 - two_s * (qi * qi + qj * qj)};
  const float s[3] = {v.scales[p * 3 + 0], v.scales[p * 3 + 1], v.scales[p * 3 + 2]};
  float RS[9], C[9], MC[9], W[9];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) RS[a * 3 + b] = (R[a * 3 + b] * s[b]) * s[b];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b)
      C[a * 3 + b] = RS[a * 3 + 0] * R[b * 3 + 0] + RS[a * 3 + 1] * R[b * 3 + 1] + RS[a * 3 + 2] * R[b * 3 + 2];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b)
      MC[a * 3 + b] = M[a * 3 + 0] * C[0 * 3 + b] + M[a * 3 + 1] * C[1 * 3 + b] + M[a * 3 + 2] * C[2 * 3 + b];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b)
      W[a * 3 + b] = MC[a * 3 + 0] * M[b * 3 + 0] + MC[a * 3 + 1] * M[b * 3 + 1] + MC[a * 3 + 2] * M[b * 3 + 2];
  o[3] = W[0]; o[4] = W[1]; o[5] = W[2]; o[6] = W[4]; o[7] = W[5]; o[8] = W[8];
  // colour: SH2RGB(sh0 + RGB2SH(clamp(img*0.5+0.5)))  (:277-281, :315-318)
  const int64_t hw = (int64_t)g.H * g.W;
  for (int c = 0; c < 3; ++c) {
    float rgb = v.img[c * hw + p] * 0.5f + 0.5f;
    rgb = fminf(fmaxf(rgb, 0.0f), 1.0f);
    const float sh0 = v.sh[(p * 3 + c) * v.d_sh] + (rgb - 0.5f) / kC0;
    o[9 + c] = fminf(fmaxf(sh0 * kC0 + 0.5f, 0.0f), 1.0f);
  }
  o[12] = v.opacities[p];
}

// ---- two-launch path (n <= kSelMax): k_g2w_select, one workgroup, holds
// the depth keys in LDS and finds the two order statistics the quantile
// needs (ranks floor / ceil of q (n0 - 1)) by a 4-pass MSB radix select
// (8-bit digits, LDS histograms, one wave per rank); it then evaluates the
// filters into an LDS flag array and scans it (stable compaction order),
// writing each kept Gaussian's record slot (0xffffffff = dropped) and the
// count.  k_g2w_emit writes the records on the whole chip.  Same values as
// sort -> k_flags -> scan -> k_emit, bit for bit, in 2 launches instead of
// ~10 (memset, prep, the radix sort's passes, flags, the scan's passes, emit).
constexpr int kSelThreads = 1024;
constexpr int kSelMax = 30720;   // keys (4 B) + flags (1 B) per Gaussian in 160 KiB of LDS
int g_g2w_path = 0;   // s3w_set_path: 0 auto, 1 multi-pass only, 2 two-launch whenever n fits

// order-preserving float <-> uint32 (the radix-sort key transform)
__device__ __forceinline__ uint32_t fkey(float z) {
  const uint32_t u = __float_as_uint(z);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

__global__ void __launch_bounds__(kSelThreads)
k_g2w_select(int n, Grid g, const float* __restrict__ means, const float* __restrict__ scales,
             const float* __restrict__ conf, float depth_min, float q, float max_scale,
             float min_conf, uint32_t* __restrict__ slot, int64_t* __restrict__ count) {
  __shared__ uint32_t keys[kSelMax];
  __shared__ uint8_t kept[kSelMax];
  __shared__ uint32_t hist[2][256];
  __shared__ uint32_t wpart[kSelThreads / 64];
  __shared__ uint32_t sel[2][2];   // [rank][prefix, remaining rank]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kSelThreads / 64;
  // depth keys (+ the count n0 of z > depth_min); consecutive threads take
  // consecutive Gaussians, 4 loads in flight per thread
  uint32_t cnt = 0;
#pragma unroll 4
  for (int i = tid; i < n; i += kSelThreads) {
    const float z = means[g.pix(i) * 3 + 2];
    const bool ok = z > depth_min;
    keys[i] = ok ? fkey(z) : 0xFFFFFFFFu;
    cnt += ok ? 1u : 0u;
  }
  cnt = wave_incl_scan(cnt, lane);
  if (lane == 63) wpart[wave] = cnt;
  __syncthreads();
  uint32_t n0 = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) n0 += wpart[w];
  const bool use_q = n0 > 0 && q < 1.0f;
  float zq = 0.0f;
  if (use_q) {
    // torch.quantile linear: ranks = q (n0 - 1), below / above order statistics
    const float ranks = q * (float)(n0 - 1);
    const uint32_t lo = (uint32_t)(int64_t)ranks, hi = (uint32_t)(int64_t)ceilf(ranks);
    if (tid < 2) {
      sel[tid][0] = 0u;
      sel[tid][1] = tid == 0 ? lo : hi;
    }
    uint32_t mask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int b = tid; b < 512; b += kSelThreads) (&hist[0][0])[b] = 0u;
      __syncthreads();
      const uint32_t p0 = sel[0][0], p1 = sel[1][0];
      for (int i = tid; i < n; i += kSelThreads) {
        const uint32_t k = keys[i];
        const uint32_t d = (k >> shift) & 255u;
        if ((k & mask) == p0) atomicAdd(&hist[0][d], 1u);
        if ((k & mask) == p1) atomicAdd(&hist[1][d], 1u);
      }
      __syncthreads();
      if (wave < 2) {
        // wave t finds the digit holding its remaining rank: 4 bins per lane
        const uint32_t rem = sel[wave][1];
        uint32_t h[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { h[j] = hist[wave][4 * lane + j]; sum += h[j]; }
        const uint32_t incl = wave_incl_scan(sum, lane);
        const uint64_t hit = __ballot(rem < incl);
        const int L = __ffsll((unsigned long long)hit) - 1;
        if (lane == L) {
          uint32_t c = incl - sum;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (rem < c + h[j]) {
              sel[wave][0] |= (uint32_t)(4 * lane + j) << shift;
              sel[wave][1] = rem - c;
              break;
            }
            c += h[j];
          }
        }
      }
      mask |= 255u << shift;
      __syncthreads();
    }
    const float a = fval(sel[0][0]), b = fval(sel[1][0]);
    const float w = ranks - (float)(int64_t)ranks;
    zq = fabsf(w) < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
  }
  // the filters, coalesced over Gaussians, into LDS flags
#pragma unroll 4
  for (int i = tid; i < n; i += kSelThreads)
    kept[i] = keep(g.pix(i), means, scales, conf, depth_min, use_q, zq, max_scale, min_conf);
  __syncthreads();
  // stable compaction: thread t scans the contiguous chunk t of the flags
  const int chunk = (n + kSelThreads - 1) / kSelThreads;
  const int c0 = min(n, tid * chunk), c1 = min(n, c0 + chunk);
  uint32_t mine = 0;
  for (int i = c0; i < c1; ++i) mine += kept[i];
  const uint32_t incl = wave_incl_scan(mine, lane);
  if (lane == 63) wpart[wave] = incl;   // (the n0 reads of wpart are behind a barrier)
  __syncthreads();
  uint32_t base = incl - mine, total = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wave) base += wpart[w];
    total += wpart[w];
  }
  if (tid == 0) *count = (int64_t)total;
  for (int i = c0; i < c1; ++i) {
    const bool k = kept[i];
    slot[i] = k ? base : 0xFFFFFFFFu;
    base += k ? 1u : 0u;
  }
}

__global__ void __launch_bounds__(kThreads)
k_g2w_emit(int64_t n, Grid g, s3w_view v, const float* __restrict__ T44,
           const uint32_t* __restrict__ slot, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t o = slot[i];
  if (o == 0xFFFFFFFFu) return;
  emit_record(v, g, T44, g.pix(i), out + (int64_t)o * 13);
}

// ---- multi-pass path (n > kSelMax) ---------------------------------------

// block-wide exclusive scan of one value per thread (kThreads threads)
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NW = kThreads / 64;
  const uint32_t incl = wave_incl_scan(x, lane);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wave) base += s_w[w];
    tot += s_w[w];
  }
  __syncthreads();
  if (total) *total = tot;
  return base + incl - x;
}

__global__ void __launch_bounds__(kThreads)
k_prep(int64_t n, Grid g, const float* __restrict__ means, float depth_min,
       uint32_t* __restrict__ keys, uint32_t* __restrict__ sel) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  bool ok = false;
  if (i < n) {
    const float z = means[g.pix(i) * 3 + 2];
    ok = z > depth_min;
    keys[i] = ok ? fkey(z) : 0xFFFFFFFFu;
  }
  uint32_t tot = 0;
  block_excl_scan(ok ? 1u : 0u, s_w, &tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&sel[4], tot);   // n0 (integer: order-free)
}

// one select pass: histograms of digit (key >> shift) & 255 over the keys
// whose higher digits equal each rank's prefix so far
__global__ void __launch_bounds__(kThreads)
k_sel_hist(int64_t n, const uint32_t* __restrict__ keys, const uint32_t* __restrict__ sel,
           uint32_t mask, int shift, uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[2][256];
  for (int b = threadIdx.x; b < 512; b += kThreads) (&lh[0][0])[b] = 0u;
  __syncthreads();
  const uint32_t p0 = sel[0], p1 = sel[2];
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads) {
    const uint32_t k = keys[i], d = (k >> shift) & 255u;
    if ((k & mask) == p0) atomicAdd(&lh[0][d], 1u);
    if ((k & mask) == p1) atomicAdd(&lh[1][d], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < 512; b += kThreads)
    if ((&lh[0][0])[b]) atomicAdd(&hist[b], (&lh[0][0])[b]);
}

// one workgroup of two waves: wave t finds the digit holding its rank's
// remaining rank (ranks floor / ceil of q (n0 - 1), set on the first pass),
// then the histograms are cleared for the next pass
__global__ void __launch_bounds__(128)
k_sel_pick(uint32_t* __restrict__ hist, uint32_t* __restrict__ sel, int shift, float q) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n0 = sel[4];
  if (shift == 24 && threadIdx.x < 2) {
    const float ranks = q * (float)(n0 > 0 ? n0 - 1 : 0);
    sel[2 * threadIdx.x + 1] = threadIdx.x == 0 ? (uint32_t)(int64_t)ranks
                                                : (uint32_t)(int64_t)ceilf(ranks);
  }
  __syncthreads();
  const uint32_t rem = sel[2 * wave + 1];
  uint32_t h[4], sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { h[j] = hist[wave * 256 + 4 * lane + j]; sum += h[j]; }
  const uint32_t incl = wave_incl_scan(sum, lane);
  const uint64_t hit = __ballot(rem < incl);
  const int L = hit ? __ffsll((unsigned long long)hit) - 1 : -1;
  if (lane == L) {
    uint32_t c = incl - sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (rem < c + h[j]) {
        sel[2 * wave] |= (uint32_t)(4 * lane + j) << shift;
        sel[2 * wave + 1] = rem - c;
        break;
      }
      c += h[j];
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < 512; b += 128) hist[b] = 0u;
}

__global__ void __launch_bounds__(kThreads)
k_flags(int64_t n, Grid g, const float* __restrict__ means, const float* __restrict__ scales,
        const float* __restrict__ conf, float depth_min, float q, float max_scale, float min_conf,
        const uint32_t* __restrict__ sel, uint32_t* __restrict__ flags,
        uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint32_t n0 = sel[4];
  const bool use_q = n0 > 0 && q < 1.0f;
  float zq = 0.0f;
  if (use_q) {
    // torch.quantile linear between the two order statistics (as k_g2w_select)
    const float ranks = q * (float)(n0 - 1);
    const float a = fval(sel[0]), b = fval(sel[2]);
    const float w = ranks - (float)(int64_t)ranks;
    zq = fabsf(w) < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
  }
  uint32_t f = 0;
  if (i < n) {
    f = keep(g.pix(i), means, scales, conf, depth_min, use_q, zq, max_scale, min_conf) ? 1u : 0u;
    flags[i] = f;
  }
  uint32_t tot = 0;
  block_excl_scan(f, s_w, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// exclusive scan of the nblk block counts in place, total in bsum[nblk]
// (and, when given, in *count)
__global__ void __launch_bounds__(1024)
k_scan_blocks(uint32_t* __restrict__ bsum, int64_t nblk, int64_t* __restrict__ count) {
  __shared__ uint32_t s_w[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t c0 = 0; c0 < nblk; c0 += 1024) {
    const int64_t c = c0 + threadIdx.x;
    const uint32_t v = c < nblk ? bsum[c] : 0u;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      if (w < wave) base += s_w[w];
      tot += s_w[w];
    }
    if (c < nblk) bsum[c] = carry + base + incl - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    bsum[nblk] = carry;
    if (count) *count = (int64_t)carry;
  }
}

__global__ void __launch_bounds__(kThreads)
k_emit(int64_t n, Grid g, s3w_view v, const float* __restrict__ T44,
       const uint32_t* __restrict__ flags, const uint32_t* __restrict__ bsum,
       float* __restrict__ out) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint32_t f = i < n ? flags[i] : 0u;
  const uint32_t off = bsum[blockIdx.x] + block_excl_scan(f, s_w, nullptr);
  if (f) emit_record(v, g, T44, g.pix(i), out + (int64_t)off * 13);
}

int64_t count_for(const s3w_view* v) {
  return s3::cdiv(v->H, v->stride) * s3::cdiv(v->W, v->stride);
}

}  // namespace

extern "C" void s3w_set_path(int path) { g_g2w_path = path; }

extern "C" size_t s3w_workspace_bytes(int64_t n) {
  if (n <= 0) return 256;
  return ws_bytes(n);   // >= the two-launch path's slot array (n x 4 B)
}

extern "C" int s3w_gaussians_to_world(const s3w_view* v, const float* T_WC, float depth_min,
                                      float depth_max_percentile, float max_scale,
                                      float min_confidence, void* workspace, float* out,
                                      int64_t* count_dev, void* stream) {
  S3_REQUIRE(v && T_WC && workspace && out && count_dev, "s3w_gaussians_to_world: null argument");
  S3_REQUIRE(v->H > 0 && v->W > 0 && v->stride >= 1 && v->d_sh >= 1,
             "s3w_gaussians_to_world: bad view shape");
  S3_REQUIRE(v->means && v->scales && v->rotations && v->sh && v->opacities && v->img,
             "s3w_gaussians_to_world: null view tensor");
  hipStream_t st = s3::as_stream(stream);
  const int64_t n = count_for(v);
  S3_REQUIRE(n < (int64_t)1 << 31, "s3w_gaussians_to_world: too many Gaussians");
  Grid g{v->H, v->W, v->stride, (int)s3::cdiv(v->W, v->stride)};
  if (n <= kSelMax && g_g2w_path != 1) {
    // two launches (the tracked frame's stride-4 view: n = 12288 at 512x384)
    const bool use_q = depth_max_percentile < 1.0f;
    uint32_t* slot = static_cast<uint32_t*>(workspace);
    k_g2w_select<<<1, kSelThreads, 0, st>>>((int)n, g, v->means, v->scales, v->conf, depth_min,
                                             use_q ? depth_max_percentile : 1.0f, max_scale,
                                             min_confidence, slot, count_dev);
    S3_LAUNCH_CHECK();
    k_g2w_emit<<<(unsigned)s3::cdiv(n, kThreads), kThreads, 0, st>>>(n, g, *v, T_WC, slot, out);
    S3_LAUNCH_CHECK();
    return S3_OK;
  }
  Ws w = carve(workspace, n);
  const int64_t blocks = nblocks(n);
  const bool use_q = depth_max_percentile < 1.0f;
  S3_HIP(hipMemsetAsync(w.hist, 0, sizeof(uint32_t) * 512 + 256, st));   // hist, sel, n0
  k_prep<<<(unsigned)blocks, kThreads, 0, st>>>(n, g, v->means, depth_min, w.keys, w.sel);
  S3_LAUNCH_CHECK();
  if (use_q) {
    const unsigned hb = (unsigned)std::min<int64_t>(blocks, 1024);
    uint32_t mask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
      k_sel_hist<<<hb, kThreads, 0, st>>>(n, w.keys, w.sel, mask, shift, w.hist);
      S3_LAUNCH_CHECK();
      k_sel_pick<<<1, 128, 0, st>>>(w.hist, w.sel, shift, depth_max_percentile);
      S3_LAUNCH_CHECK();
      mask |= 255u << shift;
    }
  }
  k_flags<<<(unsigned)blocks, kThreads, 0, st>>>(n, g, v->means, v->scales, v->conf, depth_min,
                                                 use_q ? depth_max_percentile : 1.0f, max_scale,
                                                 min_confidence, w.sel, w.flags, w.bsum);
  S3_LAUNCH_CHECK();
  k_scan_blocks<<<1, 1024, 0, st>>>(w.bsum, blocks, count_dev);
  S3_LAUNCH_CHECK();
  k_emit<<<(unsigned)blocks, kThreads, 0, st>>>(n, g, *v, T_WC, w.flags, w.bsum, out);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

// ------------------------------------------------------------ map buffer --
namespace {

struct MapWs {
  uint32_t* flags;
  uint32_t* bsum;  // per-block kept counts -> exclusive block offsets; [nblk] = total
  int64_t* n0;     // count after eviction (read by k_map_emit)
};

MapWs carve_map(void* base, int64_t n, size_t* total = nullptr) {
  char* p = static_cast<char*>(base);
  char* p0 = p;
  MapWs w;
  w.flags = (uint32_t*)p; p += align256(sizeof(uint32_t) * n);
  w.bsum = (uint32_t*)p; p += align256(sizeof(uint32_t) * (nblocks(n) + 1));
  w.n0 = (int64_t*)p; p += 256;
  if (total) *total = (size_t)(p - p0);
  return w;
}

__global__ void __launch_bounds__(kThreads)
k_map_flags(int64_t n_max, const float* __restrict__ rec, const int64_t* __restrict__ count,
            float thr, uint32_t* __restrict__ flags, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  uint32_t f = 0;
  if (i < n_max) {
    f = (i < *count && rec[i * 13 + 12] > thr) ? 1u : 0u;
    flags[i] = f;
  }
  uint32_t tot = 0;
  block_excl_scan(f, s_w, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// grid-stride: every block copies a slice of the newest half when full.
// A batch with no record left after the opacity filter (or a device count
// of 0) leaves the map untouched: frame.py:414-416 returns before the
// eviction when n_new == 0.
__global__ void __launch_bounds__(kThreads)
k_map_evict(s3w_map m, const uint32_t* __restrict__ kept_total, int64_t* __restrict__ n0) {
  const int64_t n = *m.n;
  const int64_t half = m.cap / 2;
  const int64_t kept = (int64_t)*kept_total;
  const bool full = n >= m.cap && kept > 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *n0 = full ? half : n;
  if (!full) return;
  const int64_t src = m.cap - half;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < half;
       i += (int64_t)gridDim.x * kThreads) {
#pragma unroll
    for (int k = 0; k < 3; ++k) m.means[i * 3 + k] = m.means[(src + i) * 3 + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) m.cov_triu[i * 6 + k] = m.cov_triu[(src + i) * 6 + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) m.colors[i * 3 + k] = m.colors[(src + i) * 3 + k];
    m.opacities[i] = m.opacities[src + i];
    m.kf_id[i] = m.kf_id[src + i];
  }
}

__global__ void __launch_bounds__(kThreads)
k_map_emit(int64_t n_max, s3w_map m, const float* __restrict__ rec,
           const uint32_t* __restrict__ flags, const uint32_t* __restrict__ bsum, int64_t nblk,
           const int64_t* __restrict__ n0p, int32_t kf) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint32_t f = i < n_max ? flags[i] : 0u;
  const int64_t off = (int64_t)bsum[blockIdx.x] + block_excl_scan(f, s_w, nullptr);
  const int64_t n0 = *n0p;
  const int64_t space = m.cap - n0;
  if (i == n_max - 1) {
    const int64_t kept = (int64_t)bsum[nblk];
    *m.n = n0 + (kept < space ? kept : space);
  }
  if (!f || off >= space) return;
  const int64_t j = n0 + off;
  const float* r = rec + i * 13;
#pragma unroll
  for (int k = 0; k < 3; ++k) m.means[j * 3 + k] = r[k];
#pragma unroll
  for (int k = 0; k < 6; ++k) m.cov_triu[j * 6 + k] = r[3 + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) m.colors[j * 3 + k] = r[9 + k];
  m.opacities[j] = r[12];
  m.kf_id[j] = kf;
}

__global__ void __launch_bounds__(kThreads)
k_map_scale(const float* __restrict__ means, const float* __restrict__ cov,
            const int64_t* __restrict__ n_dev, int64_t n_max, float s, float s2,
            float* __restrict__ mo, float* __restrict__ co) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n_max || i >= *n_dev) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) mo[i * 3 + k] = means[i * 3 + k] * s;
#pragma unroll
  for (int k = 0; k < 6; ++k) co[i * 6 + k] = cov[i * 6 + k] * s2;
}

}  // namespace

extern "C" size_t s3w_map_append_workspace_bytes(int64_t n_max) {
  size_t n = 0;
  carve_map(nullptr, n_max > 0 ? n_max : 1, &n);
  return n;
}

extern "C" int s3w_map_append(const s3w_map* map, const float* records, const int64_t* count_dev,
                              int64_t n_max, float opacity_threshold, int32_t kf_idx,
                              void* workspace, void* stream) {
  S3_REQUIRE(map && map->means && map->cov_triu && map->colors && map->opacities && map->kf_id &&
                 map->n && map->cap > 0,
             "s3w_map_append: bad map");
  S3_REQUIRE(n_max >= 0 && n_max < ((int64_t)1 << 31), "s3w_map_append: bad n_max");
  if (n_max == 0) return S3_OK;
  S3_REQUIRE(records && count_dev && workspace, "s3w_map_append: null argument");
  hipStream_t st = s3::as_stream(stream);
  MapWs w = carve_map(workspace, n_max);
  const int64_t blocks = nblocks(n_max);
  k_map_flags<<<(unsigned)blocks, kThreads, 0, st>>>(n_max, records, count_dev,
                                                     opacity_threshold, w.flags, w.bsum);
  S3_LAUNCH_CHECK();
  k_scan_blocks<<<1, 1024, 0, st>>>(w.bsum, blocks, nullptr);
  S3_LAUNCH_CHECK();
  const int64_t half = map->cap / 2;
  const int eb = (int)std::max<int64_t>(1, std::min<int64_t>(s3::cdiv(half, kThreads), 2048));
  k_map_evict<<<eb, kThreads, 0, st>>>(*map, w.bsum + blocks, w.n0);
  S3_LAUNCH_CHECK();
  k_map_emit<<<(unsigned)blocks, kThreads, 0, st>>>(n_max, *map, records, w.flags, w.bsum,
                                                    blocks, w.n0, kf_idx);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3w_map_scale(const float* means, const float* cov_triu, const int64_t* n_dev,
                             int64_t n_max, float s, float s2, float* means_out, float* cov_out,
                             void* stream) {
  S3_REQUIRE(n_max >= 0, "s3w_map_scale: n_max < 0");
  if (n_max == 0) return S3_OK;
  S3_REQUIRE(means && cov_triu && n_dev && means_out && cov_out, "s3w_map_scale: null argument");
  k_map_scale<<<(int)s3::cdiv(n_max, kThreads), kThreads, 0, s3::as_stream(stream)>>>(
      means, cov_triu, n_dev, n_max, s, s2, means_out, cov_out);
  S3_LAUNCH_CHECK();
  return S3_OK;
}
