// gaussians_to_world for one predicted view (include/s3w.h).
//
// k_prep    strided gather of z, "z > depth_min" keys (+inf otherwise) and
//           the valid count
// sort      hipcub radix sort of the keys (the quantile's order statistic)
// k_flags   torch.quantile (linear) bound + scale / confidence filters
// scan      hipcub exclusive sum of the flags (stable compaction order)
// k_emit    world transform, covariance, colour, opacity -> 13-float records
// All stream-ordered; the only host-visible result is *count_dev.
//
// Map buffer (SharedGaussians, frame.py:357-463):
// k_map_flags  opacity > threshold over the valid records
// scan         hipcub exclusive sum (record-order compaction)
// k_map_evict  if full: newest half -> front (one grid-stride copy), and the
//              post-eviction count for the append
// k_map_emit   scatter kept records into the SoA map, update the count
#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "s3w.h"

namespace {

constexpr int kThreads = 256;
constexpr float kC0 = 0.28209479177387814f;

struct Ws {
  float* keys_in;
  float* keys_out;
  uint32_t* flags;
  uint32_t* offsets;
  uint32_t* n_valid0;
  void* sort_tmp;
  size_t sort_bytes;
  void* scan_tmp;
  size_t scan_bytes;
};

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

size_t sort_bytes(int64_t n) {
  size_t b = 0;
  hipcub::DeviceRadixSort::SortKeys(nullptr, b, (float*)nullptr, (float*)nullptr, (int)n);
  return b;
}

size_t scan_bytes(int64_t n) {
  size_t b = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  return b;
}

Ws carve(void* base, int64_t n) {
  char* p = static_cast<char*>(base);
  Ws w;
  w.keys_in = (float*)p;  p += align256(sizeof(float) * n);
  w.keys_out = (float*)p; p += align256(sizeof(float) * n);
  w.flags = (uint32_t*)p; p += align256(sizeof(uint32_t) * n);
  w.offsets = (uint32_t*)p; p += align256(sizeof(uint32_t) * n);
  w.n_valid0 = (uint32_t*)p; p += 256;
  w.sort_bytes = sort_bytes(n);
  w.sort_tmp = p; p += align256(w.sort_bytes);
  w.scan_bytes = scan_bytes(n);
  w.scan_tmp = p;
  return w;
}

struct Grid {
  int H, W, s, ws;
  __device__ int64_t pix(int64_t i) const {
    const int64_t y = (i / ws) * s, x = (i % ws) * s;
    return y * W + x;
  }
};

__global__ void __launch_bounds__(kThreads)
k_prep(int64_t n, Grid g, const float* __restrict__ means, float depth_min,
       float* __restrict__ keys, uint32_t* __restrict__ n_valid0) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const float z = means[g.pix(i) * 3 + 2];
  const bool v = z > depth_min;
  keys[i] = v ? z : INFINITY;
  if (v) atomicAdd(n_valid0, 1u);
}

// torch.quantile(sorted[:n], q), interpolation='linear' (aten Sorting.cpp:
// ranks = q * (n - 1); below = long(ranks); above = ceil(ranks);
// lerp(v_below, v_above, ranks - below) with torch's two-sided lerp).
__device__ float quantile_linear(const float* sorted, uint32_t n, float q) {
  const float ranks = q * (float)(n - 1);
  const int64_t lo = (int64_t)ranks;
  const int64_t hi = (int64_t)ceilf(ranks);
  const float w = ranks - (float)lo;
  const float a = sorted[lo], b = sorted[hi];
  return fabsf(w) < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

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

__global__ void __launch_bounds__(kThreads)
k_flags(int64_t n, Grid g, const float* __restrict__ means, const float* __restrict__ scales,
        const float* __restrict__ conf, float depth_min, float q, float max_scale, float min_conf,
        const float* __restrict__ sorted, const uint32_t* __restrict__ n_valid0,
        uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const int64_t p = g.pix(i);
  const uint32_t n0 = *n_valid0;
  const bool use_q = n0 > 0 && q < 1.0f;
  flags[i] = keep(p, means, scales, conf, depth_min, use_q,
                  use_q ? quantile_linear(sorted, n0, q) : 0.0f, max_scale, min_conf) ? 1u : 0u;
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

__global__ void __launch_bounds__(kThreads)
k_emit(int64_t n, Grid g, s3w_view v, const float* __restrict__ T44, const uint32_t* __restrict__ flags,
       const uint32_t* __restrict__ offsets, float* __restrict__ out, int64_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  if (i == n - 1) *count = (int64_t)offsets[i] + flags[i];
  if (!flags[i]) return;
  emit_record(v, g, T44, g.pix(i), out + (int64_t)offsets[i] * 13);
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

int64_t count_for(const s3w_view* v) {
  return s3::cdiv(v->H, v->stride) * s3::cdiv(v->W, v->stride);
}

}  // namespace

extern "C" void s3w_set_path(int path) { g_g2w_path = path; }

extern "C" size_t s3w_workspace_bytes(int64_t n) {
  if (n <= 0) return 256;
  return 4 * align256(sizeof(float) * n) + 256 + align256(sort_bytes(n)) + scan_bytes(n);
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
  const int blocks = (int)s3::cdiv(n, kThreads);
  S3_HIP(hipMemsetAsync(w.n_valid0, 0, sizeof(uint32_t), st));
  k_prep<<<blocks, kThreads, 0, st>>>(n, g, v->means, depth_min, w.keys_in, w.n_valid0);
  S3_LAUNCH_CHECK();
  const bool use_q = depth_max_percentile < 1.0f;
  if (use_q) {
    size_t tb = w.sort_bytes;
    S3_HIP(hipcub::DeviceRadixSort::SortKeys(w.sort_tmp, tb, w.keys_in, w.keys_out, (int)n, 0,
                                             32, st));
  }
  k_flags<<<blocks, kThreads, 0, st>>>(n, g, v->means, v->scales, v->conf, depth_min,
                                       use_q ? depth_max_percentile : 1.0f, max_scale,
                                       min_confidence, w.keys_out, w.n_valid0, w.flags);
  S3_LAUNCH_CHECK();
  size_t sb = w.scan_bytes;
  S3_HIP(hipcub::DeviceScan::ExclusiveSum(w.scan_tmp, sb, w.flags, w.offsets, (int)n, st));
  k_emit<<<blocks, kThreads, 0, st>>>(n, g, *v, T_WC, w.flags, w.offsets, out, count_dev);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

// ------------------------------------------------------------ map buffer --
namespace {

struct MapWs {
  uint32_t* flags;
  uint32_t* offsets;
  int64_t* n0;  // count after eviction (read by k_map_emit)
  void* scan_tmp;
  size_t scan_bytes;
};

MapWs carve_map(void* base, int64_t n, size_t* total = nullptr) {
  char* p = static_cast<char*>(base);
  char* p0 = p;
  MapWs w;
  w.flags = (uint32_t*)p; p += align256(sizeof(uint32_t) * n);
  w.offsets = (uint32_t*)p; p += align256(sizeof(uint32_t) * n);
  w.n0 = (int64_t*)p; p += 256;
  w.scan_bytes = scan_bytes(n);
  w.scan_tmp = p; p += align256(w.scan_bytes);
  if (total) *total = (size_t)(p - p0);
  return w;
}

__global__ void __launch_bounds__(kThreads)
k_map_flags(int64_t n_max, const float* __restrict__ rec, const int64_t* __restrict__ count,
            float thr, uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n_max) return;
  flags[i] = (i < *count && rec[i * 13 + 12] > thr) ? 1u : 0u;
}

// grid-stride: every block copies a slice of the newest half when full.
// A batch with no record left after the opacity filter (or a device count
// of 0) leaves the map untouched: frame.py:414-416 returns before the
// eviction when n_new == 0.
__global__ void __launch_bounds__(kThreads)
k_map_evict(s3w_map m, int64_t n_max, const uint32_t* __restrict__ flags,
            const uint32_t* __restrict__ offsets, int64_t* __restrict__ n0) {
  const int64_t n = *m.n;
  const int64_t half = m.cap / 2;
  const int64_t kept = (int64_t)offsets[n_max - 1] + flags[n_max - 1];
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
           const uint32_t* __restrict__ flags, const uint32_t* __restrict__ offsets,
           const int64_t* __restrict__ n0p, int32_t kf) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n_max) return;
  const int64_t n0 = *n0p;
  const int64_t space = m.cap - n0;
  if (i == n_max - 1) {
    const int64_t kept = (int64_t)offsets[i] + flags[i];
    *m.n = n0 + (kept < space ? kept : space);
  }
  if (!flags[i] || (int64_t)offsets[i] >= space) return;
  const int64_t j = n0 + offsets[i];
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
  const int blocks = (int)s3::cdiv(n_max, kThreads);
  k_map_flags<<<blocks, kThreads, 0, st>>>(n_max, records, count_dev, opacity_threshold,
                                           w.flags);
  S3_LAUNCH_CHECK();
  size_t sb = w.scan_bytes;
  S3_HIP(hipcub::DeviceScan::ExclusiveSum(w.scan_tmp, sb, w.flags, w.offsets, (int)n_max, st));
  const int64_t half = map->cap / 2;
  const int eb = (int)std::max<int64_t>(1, std::min<int64_t>(s3::cdiv(half, kThreads), 2048));
  k_map_evict<<<eb, kThreads, 0, st>>>(*map, n_max, w.flags, w.offsets, w.n0);
  S3_LAUNCH_CHECK();
  k_map_emit<<<blocks, kThreads, 0, st>>>(n_max, *map, records, w.flags, w.offsets, w.n0,
                                          kf_idx);
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
