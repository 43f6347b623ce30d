// Tile-binned Gaussian splat rasterizer (include/gsr.h), written for gfx950.
//
// Forward:  preprocess (1 lane / Gaussian; per-workgroup reduction of the
//           instance total and depth-key range fused in) -> stable depth
//           sort of the P Gaussians (hand-written LSD radix passes of <= 9
//           bits over the live key width) -> tile binning: duplication
//           records gathered into depth order, instances emitted in depth
//           order (wave-cooperative), a stable LSD sort of the instances by
//           tile id, tile ranges -> blend (one 256-lane workgroup per 16x16
//           tile, Gaussians staged through LDS in 256-record batches,
//           block-wide early exit).  See "sorting" below.
// Backward: per-tile back-to-front replay; per-Gaussian gradients are
//           reduced across the wave with DPP/shuffles before one lane issues
//           the global atomics (64x fewer atomics than one per pixel), then a
//           per-Gaussian pass for the EWA / projection / SH chain rule.
// Tile blocks are remapped so that each XCD (private L2) receives a
// contiguous band of tiles: neighbouring tiles share most of their splats.
#include <algorithm>

#include "common.hpp"
#include "device_util.hpp"
#include "host_wait.hpp"
#include "gsr.h"
#include "raster_math.hpp"

using namespace gsr;

namespace {

constexpr int kThreads = 256;
constexpr size_t kAlign = 256;

inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

struct Carver {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t count) {
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += align_up(count * sizeof(T));
    return p;
  }
};

// Filled by k_preprocess (one set of atomics per workgroup, spread over
// kRedSlots 64-B slots so the atomics do not queue on one address) and read
// back by gsr_preprocess: instance total (num_rendered) and the depth-key
// range of the Gaussians that emit instances (it sets the number of depth
// sort passes).
constexpr int kRedSlots = 64;
struct RedSlot {
  unsigned long long total;  // instances (64-bit: no wrap)
  uint32_t kmax;             // max depth key
  uint32_t kmin_inv;         // ~min depth key (memset-0 start)
  uint32_t pad[12];
};
struct Reduce {
  RedSlot slot[kRedSlots];
};

// Hand-written stable LSD radix passes (see "sorting" below).
constexpr int kMaxDigitBits = 9, kMaxBins = 1 << kMaxDigitBits;
constexpr int kSortThreads = 512;
constexpr int kSortPerLane = 8;
constexpr int kSegItems = kSortThreads * kSortPerLane;  // 4096 items per segment

constexpr int kDupRanks = 512;  // depth ranks per duplication wave
inline int64_t nsegs(int64_t n) { return std::max<int64_t>(1, s3::cdiv(n, kSegItems)); }

struct GeomState {
  float4* rec0;  // x, y, conic.a, conic.b
  float4* rec1;  // conic.c, opacity, rgb.r, rgb.g (the blend's staged record)
  float* blue;   // [P] rgb.b (r, g ride in rec1)
  uint8_t* clamped;  // [P]: bit ch = colour channel ch clamped at 0 (SH path)
  // duplication record per Gaussian: x = x0 | y0 << 16, y = rect w | h << 16,
  // z/w = kept-tile mask (bit (y - y0) * w + (x - x0)) for rects of 2..64
  // tiles; one 16-B gather serves the depth-ordered passes
  uint4* dup;
  Reduce* red;
  // depth sort ping-pong: keys = depth bits (visible) / ~0u; values = index
  uint32_t* dkey[2];
  uint32_t* dval[2];
  uint32_t* dhist;  // [bins][segments]: digit counts -> exclusive offsets
  uint32_t* dtot;   // [bins]
  uint4* dup_sorted;  // dup records in depth order (k_order_gather)
  uint32_t* cnt_seg;  // [P / kDupRanks]: instances per depth-rank segment -> offsets
  uint32_t* dyn;      // [4] sync-free forward: kmin, span, instances kept
};

// One layout routine serves both sizing (base == nullptr) and carving.
GeomState carve_geom(void* base, int64_t P, size_t* total = nullptr) {
  Carver c{static_cast<char*>(base)};
  GeomState g;
  g.rec0 = c.take<float4>(P);
  g.rec1 = c.take<float4>(P);
  g.blue = c.take<float>(P);
  g.clamped = c.take<uint8_t>(P);
  g.dup = c.take<uint4>(P);
  g.red = c.take<Reduce>(1);
  g.dkey[0] = c.take<uint32_t>(P);
  g.dkey[1] = c.take<uint32_t>(P);
  g.dval[0] = c.take<uint32_t>(P);
  g.dval[1] = c.take<uint32_t>(P);
  g.dhist = c.take<uint32_t>((size_t)kMaxBins * nsegs(P));
  g.dtot = c.take<uint32_t>(kMaxBins);
  g.dup_sorted = c.take<uint4>(P);
  g.cnt_seg = c.take<uint32_t>(std::max<int64_t>(1, s3::cdiv(P, kDupRanks)));
  g.dyn = c.take<uint32_t>(4);
  if (total) *total = c.off;
  return g;
}
size_t geom_bytes(int64_t P) {
  size_t n = 0;
  carve_geom(nullptr, P, &n);
  return n;
}

struct BinningState {
  uint32_t* keys[2];  // tile id per instance (ping-pong)
  uint32_t* vals[2];  // Gaussian index per instance (ping-pong)
  uint32_t* hist;     // [bins][segments]
  uint32_t* tot;      // [bins]
};

BinningState carve_binning(void* base, int64_t R, size_t* total = nullptr) {
  Carver c{static_cast<char*>(base)};
  BinningState b;
  b.keys[0] = c.take<uint32_t>(R);
  b.keys[1] = c.take<uint32_t>(R);
  b.vals[0] = c.take<uint32_t>(R);
  b.vals[1] = c.take<uint32_t>(R);
  b.hist = c.take<uint32_t>((size_t)kMaxBins * nsegs(R));
  b.tot = c.take<uint32_t>(kMaxBins);
  if (total) *total = c.off;
  return b;
}
size_t binning_bytes(int64_t R) {
  size_t n = 0;
  carve_binning(nullptr, R, &n);
  return n;
}

struct ImageState {
  uint2* ranges;       // [tiles]
  uint32_t* n_contrib; // [H*W]
  float* final_T;      // [H*W]
  uint32_t* cursor;    // [tiles] per-tile binning: counts -> fill cursors
};
ImageState carve_image(void* base, int H, int W, size_t* total = nullptr) {
  Carver c{static_cast<char*>(base)};
  int tiles = ((W + BX - 1) / BX) * ((H + BY - 1) / BY);
  ImageState s;
  s.ranges = c.take<uint2>(tiles);
  s.cursor = c.take<uint32_t>(tiles);
  s.n_contrib = c.take<uint32_t>((size_t)H * W);
  s.final_T = c.take<float>((size_t)H * W);
  if (total) *total = c.off;
  return s;
}
size_t image_bytes(int H, int W) {
  size_t n = 0;
  carve_image(nullptr, H, W, &n);
  return n;
}

int bit_length(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

// Bijective XCD-aware tile order: consecutive workgroup ids round-robin over
// the 8 XCDs; give each XCD a contiguous run of tiles (guide §5, T1).
__device__ __forceinline__ int xcd_tile(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, k = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// ------------------------------------------------------------ preprocess --
struct Cam {
  int W, H;
  float tanfx, tanfy, fx, fy, scale_mod;
  int D, M;
  int gx, gy;
  bool prefiltered;
};

// One Gaussian: returns its kept-tile count (0 = culled) and its depth key.
__device__ __forceinline__ uint32_t
preprocess_one(int64_t i, Cam cam, const float* __restrict__ means,
             const float* __restrict__ scales, const float* __restrict__ rots,
             const float* __restrict__ cov_pre, const float* __restrict__ shs,
             const float* __restrict__ colors_pre, const float* __restrict__ opac,
             const float* __restrict__ vm, const float* __restrict__ pm,
             const float* __restrict__ campos, int32_t* __restrict__ radii, GeomState g,
             uint32_t* key_out) {
  // depth-sort key (fused here instead of a separate pass; the first sort
  // pass takes the index as its value): culled Gaussians sort last and emit
  // nothing.  Every per-Gaussian output is stored once: a culled Gaussian's
  // here, a kept one's at the end.
  auto cull = [&]() -> uint32_t {
    radii[i] = 0;
    g.dup[i] = make_uint4(0u, 0u, 0u, 0u);
    g.dkey[0][i] = 0xFFFFFFFFu;
    return 0u;
  };
  const float mx = means[i * 3 + 0], my = means[i * 3 + 1], mz = means[i * 3 + 2];
  float pv[3];
  xform43(vm, mx, my, mz, pv);
  if (pv[2] <= 0.2f) return cull();  // in_frustum near-plane cull
  float ph[4];
  xform44(pm, mx, my, mz, ph);
  const float pw = 1.0f / (ph[3] + 0.0000001f);
  const float ppx = ph[0] * pw, ppy = ph[1] * pw;

  float cov3[6];
  if (cov_pre) {
#pragma unroll
    for (int k = 0; k < 6; ++k) cov3[k] = cov_pre[i * 6 + k];
  } else {
    // not stored: the backward recomputes it from the same inputs (bit for
    // bit), 24 B per Gaussian less written by every forward
    cov3d_from_scale_rot(scales + i * 3, cam.scale_mod, rots + i * 4, cov3);
  }
  Ewa e = ewa_project(mx, my, mz, cov3, vm, cam.fx, cam.fy, cam.tanfx, cam.tanfy);
  const float a = e.a + 0.3f, b = e.b, c = e.c + 0.3f;
  const float det = a * c - b * b;
  if (det == 0.0f) return cull();
  const float det_inv = 1.0f / det;
  const float mid = 0.5f * (a + c);
  const float disc = sqrtf(fmaxf(0.1f, mid * mid - det));
  const float l1 = mid + disc, l2 = mid - disc;
  const int r = (int)ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
  const float px = ndc2pix(ppx, cam.W), py = ndc2pix(ppy, cam.H);
  int x0, y0, x1, y1;
  get_rect(px, py, r, cam.gx, cam.gy, &x0, &y0, &x1, &y1);
  if ((x1 - x0) * (y1 - y0) == 0) return cull();

  float rgb[3];
  if (colors_pre) {
    rgb[0] = colors_pre[i * 3 + 0]; rgb[1] = colors_pre[i * 3 + 1]; rgb[2] = colors_pre[i * 3 + 2];
  } else {
    float B[16];
    if (cam.D == 0) {
      B[0] = SH_C0;   // degree 0: the view direction does not enter
    } else {
      float dx = mx - campos[0], dy = my - campos[1], dz = mz - campos[2];
      float len = sqrtf(dx * dx + dy * dy + dz * dz);
      dx = dx / len; dy = dy / len; dz = dz / len;
      sh_basis(cam.D, dx, dy, dz, B);
    }
    const int nb = (cam.D + 1) * (cam.D + 1);
    const float* sh = shs + i * (int64_t)cam.M * 3;
    uint32_t cl = 0;
    for (int ch = 0; ch < 3; ++ch) {
      float acc = B[0] * sh[ch];
      for (int k = 1; k < nb; ++k) acc = acc + B[k] * sh[k * 3 + ch];
      acc = acc + 0.5f;
      cl |= (uint32_t)(acc < 0.0f) << ch;
      rgb[ch] = fmaxf(acc, 0.0f);
    }
    g.clamped[i] = (uint8_t)cl;       // one byte store instead of three
  }
  g.blue[i] = rgb[2];
  radii[i] = r;
  g.rec0[i] = make_float4(px, py, c * det_inv, -b * det_inv);
  g.rec1[i] = make_float4(a * det_inv, opac[i], rgb[0], rgb[1]);
  // tiles the blend can actually use; the reference lists every tile of the
  // rect, whose extra entries are all skipped per pixel.  Rects of <= 64
  // tiles keep only the tiles the blend can use (tile_cull /
  // tile_mask_rows, raster_math.hpp) as a bit mask; larger rects keep every tile
  const int rw = x1 - x0, area = rw * (y1 - y0);
  uint64_t mask = area == 1 ? 1ull : ~0ull;
  uint32_t n = (uint32_t)area;
  if (area > 1 && area <= 64) {
    const float cA = c * det_inv, cB = -b * det_inv, cC = a * det_inv;
    const TileCull tc = tile_cull(px, py, cA, cB, cC, opac[i], x0, y0, x1, y1);
    mask = tile_mask_rows(tc, px, py, cA, cB, cC, x0, y0, rw, y1 - y0, cam.H);
    n = (uint32_t)__popcll(mask);
  }
  g.dup[i] = make_uint4((uint32_t)x0 | ((uint32_t)y0 << 16),
                        (uint32_t)rw | ((uint32_t)(y1 - y0) << 16), (uint32_t)mask,
                        (uint32_t)(mask >> 32));
  // stable depth sort key: positive depth bits order like the floats
  // (~0u is reserved for culled Gaussians so that every emitting Gaussian
  // ranks below `visible`; no finite depth reaches it)
  const uint32_t key = n > 0 ? min(__float_as_uint(pv[2]), 0xFFFFFFFEu) : 0xFFFFFFFFu;
  g.dkey[0][i] = key;
  *key_out = key;
  return n;
}

__global__ void __launch_bounds__(kThreads)
k_preprocess(int64_t P, Cam cam, const float* __restrict__ means,
             const float* __restrict__ scales, const float* __restrict__ rots,
             const float* __restrict__ cov_pre, const float* __restrict__ shs,
             const float* __restrict__ colors_pre, const float* __restrict__ opac,
             const float* __restrict__ vm, const float* __restrict__ pm,
             const float* __restrict__ campos, int32_t* __restrict__ radii, GeomState g) {
  __shared__ unsigned long long s_sum[kThreads / 64];
  __shared__ uint32_t s_max[kThreads / 64], s_min[kThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t n = 0, key = 0;
  if (i < P)
    n = preprocess_one(i, cam, means, scales, rots, cov_pre, shs, colors_pre, opac, vm, pm,
                       campos, radii, g, &key);
  // workgroup total and key range, then one set of atomics (replaces a
  // reduction pass)
  unsigned long long s = n;
  uint32_t kmax = n > 0 ? key : 0u, kmin_inv = n > 0 ? ~key : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    kmax = max(kmax, (uint32_t)__shfl_xor(kmax, o, 64));
    kmin_inv = max(kmin_inv, (uint32_t)__shfl_xor(kmin_inv, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    s_sum[threadIdx.x >> 6] = s;
    s_max[threadIdx.x >> 6] = kmax;
    s_min[threadIdx.x >> 6] = kmin_inv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long bs = 0;
    uint32_t bmax = 0, bmin = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
      bs += s_sum[w];
      bmax = max(bmax, s_max[w]);
      bmin = max(bmin, s_min[w]);
    }
    if (bs > 0) {
      RedSlot* sl = &g.red->slot[blockIdx.x & (kRedSlots - 1)];
      atomicAdd(&sl->total, bs);
      atomicMax(&sl->kmax, bmax);
      atomicMax(&sl->kmin_inv, bmin);
    }
  }
}

// ------------------------------------------------------------- sorting ----
//
// The reference binning (rasterizer_impl.cu duplicateWithKeys + SortPairs
// over tile << 32 | depth) orders instances by (tile, depth, index).  Here
// two hand-written stable LSD radix sorts, each pass over <= 9-bit digits:
//
//   depth sort   the P Gaussians by depth key (equal keys keep index
//                order).  Keys are offset by the minimum visible key (read
//                back with num_rendered), so the pass count follows the live
//                key width: 24 bits -> 3 passes of 8 bits.
//   gather       the duplication records in depth order + instances per
//                512-rank segment, scanned (k_order_gather, k_seg_scan).
//   duplication  instances written in depth order (wave-cooperative,
//                coalesced), tile id as key.
//   tile sort    the instances by tile id (11 bits at 960x540 -> 6 + 5).
//
// Each pass: k_rs_hist (digit counts of every 4096-item segment ->
// hist[digit][segment]) -> k_row_scan (one wave per digit row, exclusive
// offsets in place, row total) -> k_rs_scatter: per-wave digit counts in
// LDS, the segment's items ranked within each 64-item window by a ballot
// match on the digit (stable by construction), staged in LDS in digit order
// and written out as runs of consecutive addresses (a random scatter of
// single words would cost one partial-line write-back per item).

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// lanes of `active` holding the same `bits`-bit value as this lane
__device__ __forceinline__ uint64_t match_peers(uint32_t d, bool active, int bits) {
  uint64_t peers = __ballot(active);
  for (int b = 0; b < bits; ++b) {
    const bool set = (d >> b) & 1u;
    const uint64_t m = __ballot(active && set);
    peers &= set ? m : ~m;
  }
  return peers;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// exclusive scan of one value per thread across the workgroup; total too
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w,
                                                    uint32_t* total = nullptr) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v, lane);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t base = 0, all = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    base += k < w ? s_w[k] : 0u;
    all += s_w[k];
  }
  __syncthreads();
  if (total) *total = all;
  return base + inc - v;
}

// Per row: exclusive scan over `cols` columns in place, row total to
// tot[row].  One workgroup per row; wave w owns a contiguous quarter of the
// columns: quarter totals first, then the scan with the quarter's carry-in.
__global__ void __launch_bounds__(kThreads)
k_row_scan(uint32_t* __restrict__ hist, int64_t cols, uint32_t* __restrict__ tot) {
  constexpr int NW = kThreads / 64, kCh = 8;
  __shared__ uint32_t s_q[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t* h = hist + (size_t)blockIdx.x * cols;
  const int64_t per = (cols + NW - 1) / NW;
  const int64_t q0 = min(cols, (int64_t)w * per), q1 = min(cols, q0 + per);
  uint32_t sum = 0;
  for (int64_t c0 = q0; c0 < q1; c0 += kCh * 64) {
    uint32_t v[kCh];
#pragma unroll
    for (int j = 0; j < kCh; ++j) {
      const int64_t c = c0 + j * 64 + lane;
      v[j] = c < q1 ? h[c] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kCh; ++j) sum += v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if (lane == 0) s_q[w] = sum;
  __syncthreads();
  uint32_t carry = 0, all = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    carry += k < w ? s_q[k] : 0u;
    all += s_q[k];
  }
  for (int64_t c0 = q0; c0 < q1; c0 += kCh * 64) {
    uint32_t v[kCh];
#pragma unroll
    for (int j = 0; j < kCh; ++j) {
      const int64_t c = c0 + j * 64 + lane;
      v[j] = c < q1 ? h[c] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kCh; ++j) {
      const int64_t c = c0 + j * 64 + lane;
      const uint32_t inc = wave_incl_scan(v[j], lane);
      if (c < q1) h[c] = carry + inc - v[j];
      carry += __shfl(inc, 63, 64);
    }
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = all;
}

// digit of a key: (min(key - kmin, span) >> shift) & mask
struct Digit {
  uint32_t kmin, span;
  int shift, bits;
  // device (kmin, span) of the sync-free forward (gsr_forward_deferred);
  // null: the host values above
  const uint32_t* dyn;
  __device__ __forceinline__ uint32_t operator()(uint32_t key) const {
    uint32_t k = key - kmin;
    k = k < span ? k : span;
    return (k >> shift) & ((1u << bits) - 1u);
  }
  __device__ __forceinline__ Digit live() const {
    Digit d = *this;
    if (dyn) { d.kmin = dyn[0]; d.span = dyn[1]; }
    return d;
  }
};

// item count of a pass: the host bound, or the device count when given
__device__ __forceinline__ int64_t live_n(int64_t n, const uint32_t* dn) {
  return dn ? min(n, (int64_t)*dn) : n;
}

template <typename K>
__global__ void __launch_bounds__(kSortThreads)
k_rs_hist(int64_t n, const K* __restrict__ keys, Digit dg_in, int64_t nseg,
          uint32_t* __restrict__ hist, const uint32_t* __restrict__ dn) {
  __shared__ uint32_t cnt[kMaxBins];
  const Digit dg = dg_in.live();
  n = live_n(n, dn);
  const int bins = 1 << dg.bits;
  for (int d = threadIdx.x; d < bins; d += kSortThreads) cnt[d] = 0u;
  __syncthreads();
  const int64_t s = blockIdx.x;
  const int64_t i0 = s * kSegItems;
  uint32_t key[kSortPerLane];
#pragma unroll
  for (int j = 0; j < kSortPerLane; ++j) {
    const int64_t i = i0 + j * kSortThreads + threadIdx.x;
    key[j] = i < n ? (uint32_t)keys[i] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kSortPerLane; ++j) {
    // counts do not depend on the order: one LDS atomic per item (a ballot
    // match per window costs a VALU op per digit bit)
    if (i0 + j * kSortThreads + threadIdx.x < n) atomicAdd(&cnt[dg(key[j])], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < bins; d += kSortThreads) hist[(size_t)d * nseg + s] = cnt[d];
}

// One segment of kSegItems items: wave w owns items [w * 512, (w + 1) *
// 512) of it, in 8 windows of 64.
template <typename K, typename V>
__global__ void __launch_bounds__(kSortThreads)
k_rs_scatter(int64_t n, const K* __restrict__ kin, const V* __restrict__ vin,
             K* __restrict__ kout, V* __restrict__ vout, Digit dg_in, int64_t nseg,
             const uint32_t* __restrict__ hist, const uint32_t* __restrict__ tot,
             const uint32_t* __restrict__ dn) {
  constexpr int NW = kSortThreads / 64;
  const Digit dg = dg_in.live();
  n = live_n(n, dn);
  __shared__ uint32_t cnt[NW][kMaxBins];  // per-wave counts -> local slots
  __shared__ uint32_t gdelta[kMaxBins];   // global slot - local slot, per digit
  __shared__ uint32_t s_w[NW];
  __shared__ K sk[kSegItems];
  __shared__ V sv[kSegItems];
  const int bins = 1 << dg.bits;
  for (int d = threadIdx.x; d < NW * kMaxBins; d += kSortThreads) (&cnt[0][0])[d] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t s = blockIdx.x;
  const int64_t seg0 = s * kSegItems;
  const int64_t base_w = seg0 + (int64_t)w * 64 * kSortPerLane;
  uint32_t key[kSortPerLane];
  V val[kSortPerLane];
  // phase A: every load issued first, then digits, window matches and
  // per-wave counts
#pragma unroll
  for (int j = 0; j < kSortPerLane; ++j) {
    const int64_t i = base_w + j * 64 + lane;
    key[j] = i < n ? (uint32_t)kin[i] : 0u;
    // vin == nullptr: the item's own index (first pass of the depth sort)
    val[j] = i < n ? (vin ? vin[i] : (V)i) : V(0);
  }
#pragma unroll
  for (int j = 0; j < kSortPerLane; ++j)   // counts: order-free, one LDS atomic per item
    if (base_w + j * 64 + lane < n) atomicAdd(&cnt[w][dg(key[j])], 1u);
  __syncthreads();
  // phase B: local slots (digit-major within the segment) and the global
  // offset of each digit's run; bins <= 2 * kSortThreads
  {
    constexpr int PER = kMaxBins / kSortThreads;
    uint32_t tb[PER], gt[PER], lsum = 0, gsum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int d = threadIdx.x * PER + q;
      tb[q] = 0;
      gt[q] = 0;
      if (d < bins) {
#pragma unroll
        for (int k = 0; k < NW; ++k) tb[q] += cnt[k][d];
        gt[q] = tot[d];
      }
      lsum += tb[q];
      gsum += gt[q];
    }
    uint32_t lbase = block_excl_scan<kSortThreads>(lsum, s_w);
    uint32_t gbase = block_excl_scan<kSortThreads>(gsum, s_w);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int d = threadIdx.x * PER + q;
      if (d < bins) {
        gdelta[d] = gbase + hist[(size_t)d * nseg + s] - lbase;
        uint32_t b = lbase;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
          const uint32_t c = cnt[k][d];
          cnt[k][d] = b;
          b += c;
        }
      }
      lbase += tb[q];
      gbase += gt[q];
    }
  }
  __syncthreads();
  // phase C: local slot = wave's running slot + rank among equal digits in
  // the window; stage key and value there
#pragma unroll
  for (int j = 0; j < kSortPerLane; ++j) {
    const bool ok = base_w + j * 64 + lane < n;
    const uint32_t d = dg(key[j]);
    const uint64_t peers = match_peers(d, ok, dg.bits);
    if (ok) {
      const uint32_t b = cnt[w][d];
      const uint32_t lp = b + (uint32_t)__popcll(peers & lanemask_lt(lane));
      if ((peers >> lane) == 1ull) cnt[w][d] = b + (uint32_t)__popcll(peers);
      sk[lp] = (K)key[j];
      sv[lp] = val[j];
    }
    wave_lds_sync();
  }
  __syncthreads();
  // phase D: runs of equal digits go to consecutive global slots
  const int m = (int)min<int64_t>(kSegItems, n - seg0);
#pragma unroll
  for (int j = 0; j < kSortPerLane; ++j) {
    const int lp = j * kSortThreads + threadIdx.x;
    if (lp < m) {
      const K k = sk[lp];
      const uint32_t gp = (uint32_t)lp + gdelta[dg((uint32_t)k)];
      if (kout) kout[gp] = k;
      vout[gp] = sv[lp];
    }
  }
}

__device__ __forceinline__ uint32_t dup_count(const uint4 d) {
  const uint32_t w = d.y & 0xFFFFu, h = d.y >> 16;
  return w * h <= 64u ? (uint32_t)__popcll((uint64_t)d.z | ((uint64_t)d.w << 32)) : w * h;
}

// The duplication records in depth order (one coalesced copy instead of a
// random gather inside the emission loop), and the instances of every
// kDupRanks-rank segment (one wave each; all gathers of a lane in flight).
__global__ void __launch_bounds__(kThreads)
k_order_gather(int64_t P, const uint32_t* __restrict__ order, const uint4* __restrict__ dup,
               int64_t nwseg, uint4* __restrict__ dsorted, uint32_t* __restrict__ cnt_seg) {
  constexpr int NWIN = kDupRanks / 64;
  const int lane = threadIdx.x & 63;
  const int64_t ws = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (ws >= nwseg) return;
  uint4 d[NWIN];
#pragma unroll
  for (int j = 0; j < NWIN; ++j) {
    const int64_t k = ws * kDupRanks + j * 64 + lane;
    d[j] = k < P ? dup[order[k]] : make_uint4(0u, 0u, 0u, 0u);
  }
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < NWIN; ++j) {
    const int64_t k = ws * kDupRanks + j * 64 + lane;
    if (k < P) {
      dsorted[k] = d[j];
      c += dup_count(d[j]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) cnt_seg[ws] = c;
}

// exclusive scan of the segment counts in place (one workgroup)
__global__ void __launch_bounds__(1024) k_seg_scan(uint32_t* __restrict__ cnt_seg, int64_t nseg) {
  __shared__ uint32_t s_w[16];
  uint32_t carry = 0;
  for (int64_t c0 = 0; c0 < nseg; c0 += 1024) {
    const int64_t c = c0 + threadIdx.x;
    const uint32_t v = c < nseg ? cnt_seg[c] : 0u;
    uint32_t total = 0;
    const uint32_t ex = block_excl_scan<1024>(v, s_w, &total);
    if (c < nseg) cnt_seg[c] = carry + ex;
    carry += total;
  }
}

// Instances in depth order.  Each wave owns kDupRanks consecutive depth
// ranks, which start at the segment's scanned offset; 64 ranks at a time own
// a contiguous output range, produced in chunks of DCH slots: every lane
// enumerates its own instances that fall in the chunk (kept-tile mask bits
// in rect order, or the plain rect for rects of more than 64 tiles) into the
// wave's LDS slice, then the wave copies the slice out with coalesced
// stores.  Waves are independent (no workgroup barriers).
constexpr int DCH = 512;

template <typename K>
__global__ void __launch_bounds__(kThreads)
k_duplicate(int64_t P, int gx, const uint32_t* __restrict__ order,
            const uint4* __restrict__ dsorted,
            const uint32_t* __restrict__ seg_off, int64_t nwseg, K* __restrict__ keys,
            uint32_t* __restrict__ vals, uint32_t cap) {
  __shared__ K s_key[kThreads / 64][DCH];
  __shared__ uint32_t s_val[kThreads / 64][DCH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ws = (int64_t)blockIdx.x * (kThreads / 64) + w;
  if (ws >= nwseg) return;
  K* sk = s_key[w];
  uint32_t* sv = s_val[w];
  uint32_t running = seg_off[ws];
  const int64_t k_base = ws * kDupRanks + lane;
  // records are in depth order (coalesced); windows r + 1 and r + 2 are in
  // flight while window r is emitted
  constexpr int NWIN = kDupRanks / 64;
  auto ld_o = [&](int r) { const int64_t k = k_base + r * 64; return k < P ? order[k] : 0u; };
  auto ld_d = [&](int r) {
    const int64_t k = k_base + r * 64;
    return k < P ? dsorted[k] : make_uint4(0u, 0u, 0u, 0u);
  };
  uint32_t o1 = ld_o(0), o2 = NWIN > 1 ? ld_o(1) : 0u;
  uint4 d1 = ld_d(0), d2 = NWIN > 1 ? ld_d(1) : make_uint4(0u, 0u, 0u, 0u);
  for (int r = 0; r < NWIN; ++r) {
    const uint32_t i = o1;
    const uint4 d = d1;
    o1 = o2;
    d1 = d2;
    if (r + 2 < NWIN) {
      o2 = ld_o(r + 2);
      d2 = ld_d(r + 2);
    }
    const uint32_t cnt = dup_count(d);
    const int x0 = (int)(d.x & 0xFFFFu), y0 = (int)(d.x >> 16);
    const int rw = max(1, (int)(d.y & 0xFFFFu));
    const bool use_mask = rw * (int)(d.y >> 16) <= 64;
    const uint64_t mask = (uint64_t)d.z | ((uint64_t)d.w << 32);
    const uint32_t inc = wave_incl_scan(cnt, lane);
    const uint32_t start = running + inc - cnt;
    const uint32_t lo = running;
    const uint32_t hi = running + __shfl(inc, 63, 64);
    running = hi;
    for (uint32_t c0 = lo; c0 < hi; c0 += DCH) {
      const uint32_t c1 = min(c0 + (uint32_t)DCH, hi);
      if (cnt > 0 && start < c1 && start + cnt > c0) {
        if (use_mask) {
          uint64_t m = mask;
          const uint32_t e = min(c1, start + cnt);
          for (uint32_t q = start; m && q < e; ++q) {
            const int pos = __builtin_ctzll(m);
            m &= m - 1;
            if (q >= c0) {
              sk[q - c0] = (K)((y0 + pos / rw) * gx + x0 + pos % rw);
              sv[q - c0] = i;
            }
          }
        } else {
          const uint32_t j0 = max(c0, start) - start, j1 = min(c1, start + cnt) - start;
          for (uint32_t j = j0; j < j1; ++j) {
            sk[start + j - c0] = (K)((y0 + (int)j / rw) * gx + x0 + (int)j % rw);
            sv[start + j - c0] = i;
          }
        }
      }
      wave_lds_sync();
      // cap: the instance capacity of the sync-free forward (instances past
      // it are dropped and the frame is flagged by k_red_finalize)
      for (uint32_t t = lane; t < c1 - c0 && c0 + t < cap; t += 64) {
        keys[c0 + t] = sk[t];
        vals[c0 + t] = sv[t];
      }
      wave_lds_sync();
    }
  }
}

template <typename K>
__global__ void __launch_bounds__(kThreads)
k_ranges(int64_t R, const K* __restrict__ keys, uint2* __restrict__ ranges,
         const uint32_t* __restrict__ dn) {
  R = live_n(R, dn);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R) return;
  const uint32_t cur = keys[i];
  if (i == 0) {
    ranges[cur].x = 0;
  } else {
    const uint32_t prev = keys[i - 1];
    if (cur != prev) {
      ranges[prev].y = (uint32_t)i;
      ranges[cur].x = (uint32_t)i;
    }
  }
  if (i == R - 1) ranges[cur].y = (uint32_t)R;
}

// k_ranges for 16-bit tile keys, 8 keys per thread: one 16-B load per
// thread (the previous key from the neighbouring lane), 8x fewer threads
__global__ void __launch_bounds__(kThreads)
k_ranges16(int64_t R, const uint16_t* __restrict__ keys, uint2* __restrict__ ranges,
           const uint32_t* __restrict__ dn) {
  R = live_n(R, dn);
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  uint16_t k[8];
  if (i0 + 8 <= R) {
    const uint4 v = *reinterpret_cast<const uint4*>(keys + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      k[2 * e] = (uint16_t)(w[e] & 0xFFFFu);
      k[2 * e + 1] = (uint16_t)(w[e] >> 16);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) k[e] = i0 + e < R ? keys[i0 + e] : (uint16_t)0;
  }
  // the key before i0: the neighbouring lane's last key, or a load at a
  // wave's first lane
  const int lane = threadIdx.x & 63;
  uint32_t prev = (uint32_t)__shfl_up((int)k[7], 1, 64);
  if (lane == 0 && i0 > 0 && i0 <= R) prev = keys[i0 - 1];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int64_t i = i0 + e;
    if (i >= R) break;
    const uint32_t cur = k[e];
    const uint32_t pk = e == 0 ? prev : (uint32_t)k[e - 1];
    if (i == 0) {
      ranges[cur].x = 0;
    } else if (cur != pk) {
      ranges[pk].y = (uint32_t)i;
      ranges[cur].x = (uint32_t)i;
    }
    if (i == R - 1) ranges[cur].y = (uint32_t)R;
  }
}

// One stable LSD sort: passes over `bits` bits of (key - kmin), each of
// <= kMaxDigitBits.  Returns the index (0/1) of the ping-pong buffers that
// hold the result.
inline int sort_passes(int bits) { return std::max(1, (bits + kMaxDigitBits - 1) / kMaxDigitBits); }
// ping-pong index holding the tile-sorted instances (gsr_render, gsr_backward)
inline int tile_sort_buffer(int ntiles) {
  return sort_passes(bit_length((uint64_t)(ntiles - 1))) & 1;
}

// dyn / dn: device (kmin, span) and item count of the sync-free forward
// (kernels sized for the host bound n, items past *dn ignored).
template <typename K, typename V>
int radix_sort(int64_t n, K* keys[2], V* vals[2], uint32_t kmin, uint32_t span, int bits,
               bool keep_keys, uint32_t* hist, uint32_t* tot, hipStream_t st,
               bool index_vals = false, const uint32_t* dyn = nullptr,
               const uint32_t* dn = nullptr) {
  const int passes = sort_passes(bits);
  const int width = (bits + passes - 1) / passes;
  const int64_t nseg = nsegs(n);
  int src = 0;
  for (int p = 0; p < passes; ++p) {
    const int hi = std::min(bits, (p + 1) * width);
    const Digit dg{kmin, span, p * width, std::max(1, hi - p * width), dyn};
    k_rs_hist<K><<<(unsigned)nseg, kSortThreads, 0, st>>>(n, keys[src], dg, nseg, hist, dn);
    k_row_scan<<<1u << dg.bits, kThreads, 0, st>>>(hist, nseg, tot);
    const bool last = p == passes - 1;
    k_rs_scatter<K, V><<<(unsigned)nseg, kSortThreads, 0, st>>>(
        n, keys[src], (p == 0 && index_vals) ? nullptr : vals[src], (!last || keep_keys) ? keys[src ^ 1] : nullptr, vals[src ^ 1],
        dg, nseg, hist, tot, dn);
    src ^= 1;
  }
  return src;
}

// The sync-free forward's bookkeeping (one wave, after k_preprocess): the
// reduction slots -> instance total and depth-key range; dyn = {kmin, span,
// instances kept (<= cap)}; info = {status, instances, live key bits}, status
// bit 0 = more instances than the binning capacity, bit 1 = a key range wider
// than the depth sort's passes cover (the image is then not valid).
__global__ void __launch_bounds__(64)
k_red_finalize(const Reduce* __restrict__ red, uint32_t cap, int key_bits,
               uint32_t* __restrict__ dyn, int64_t* __restrict__ info) {
  const int lane = threadIdx.x;
  unsigned long long total = red->slot[lane].total;
  uint32_t kmax = red->slot[lane].kmax, kmin_inv = red->slot[lane].kmin_inv;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    total += __shfl_xor(total, o, 64);
    kmax = max(kmax, (uint32_t)__shfl_xor(kmax, o, 64));
    kmin_inv = max(kmin_inv, (uint32_t)__shfl_xor(kmin_inv, o, 64));
  }
  if (lane != 0) return;
  const uint32_t kmin = total ? ~kmin_inv : 0u;
  const uint32_t span = total ? kmax - kmin + 1u : 1u;
  const int bits = 32 - __clz(span);
  const int status = (total > cap ? 1 : 0) | (bits > key_bits ? 2 : 0);
  dyn[0] = kmin;
  dyn[1] = span;
  dyn[2] = (uint32_t)min(total, (unsigned long long)cap);
  info[0] = status;
  info[1] = (int64_t)total;
  info[2] = bits;
}

// -------------------------------------------------- per-tile binning ----
//
// An alternative binning, selected by
// gsr_set_binning(1); measured slower than the global sorts and therefore not
// the default (C3 forward 1.22 vs 0.86 ms, profiles/r05l_*): sorting the R
// instances by depth inside their tiles ranks 3.8x more items per depth pass
// than sorting the P Gaussians once (R = 15.8M, P = 4.19M), the ballot rank
// costs a VALU op per digit bit per item, and the fill's scattered 4-B
// writes land in partial lines.  Instead of sorting all P Gaussians by depth
// and then all R instances by tile (3 + 2 global LSD passes and a gather of
// the duplication records into depth order), the instances are binned by
// tile straight from the Gaussians in index order and every tile sorts its
// own list in LDS:
//
//   k_tile_count  per-tile instance counts (a workgroup of 1,024 Gaussians
//                 counts into an LDS histogram, then one global atomic per
//                 touched tile: Splatt3R's Gaussians come in pixel order, so a
//                 workgroup touches few tiles)
//   k_tile_scan   tile offsets -> ranges and fill cursors (one workgroup)
//   k_tile_fill   (depth key, index) per instance into its tile's range: LDS
//                 counts, one global cursor reservation per (workgroup, tile),
//                 LDS ranks (arrival order inside the tile)
//   k_tile_sort   one workgroup per tile: a stable LSD radix sort of the
//                 tile's list by depth key in LDS (<= 16,384 instances; larger
//                 tiles run the same passes chunk by chunk through the binning
//                 buffers), 8-bit digits ranked exactly as k_rs_scatter does.
//                 The fill order is arbitrary, so runs of equal depth keys
//                 are put in index order (in place for runs of <= 32, else by
//                 index passes + depth passes): the order is always (depth
//                 key, Gaussian index), the reference's (tile, depth, index)
//                 order of duplicateWithKeys + SortPairs.
//
// The sorted list lands in the buffer tile_sort_buffer() names, so the
// backward (and the two-call render) read it as before.
constexpr int kBinThreads = 256, kBinPer = 4;     // Gaussians per thread
constexpr int kTileLdsMax = 8192;                 // tiles counted in LDS (fill: 64 KiB)
// k_tile_sort's LDS image is sized for gfx950's 160 KiB (2 x 16384 x 4 B +
// counts, ~145 KiB); a device pass for a 64-KiB-LDS target (S3_OFFLOAD_ARCH)
// gets a quarter of the chunk so the library still builds there (the kernel
// walks longer tiles in chunks either way).  Only device code reads kTSCap.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
constexpr int kTSIptArch = 4;
#else
constexpr int kTSIptArch = 16;
#endif
constexpr int kTSThreads = 1024, kTSWaves = kTSThreads / 64, kTSIpt = kTSIptArch;
constexpr int kTSCap = kTSThreads * kTSIpt;        // instances sorted in LDS

// the kept tiles of one duplication record, in k_duplicate's order
template <typename F>
__device__ __forceinline__ void for_each_tile(const uint4 d, int gx, F&& f) {
  const int rw = (int)(d.y & 0xFFFFu), rh = (int)(d.y >> 16);
  if (rw * rh == 0) return;                       // culled
  const int x0 = (int)(d.x & 0xFFFFu), y0 = (int)(d.x >> 16);
  if (rw * rh <= 64) {
    uint64_t m = (uint64_t)d.z | ((uint64_t)d.w << 32);
    while (m) {
      const int pos = __builtin_ctzll(m);
      m &= m - 1;
      f((y0 + pos / rw) * gx + x0 + pos % rw);
    }
  } else {
    for (int j = 0; j < rw * rh; ++j) f((y0 + j / rw) * gx + x0 + j % rw);
  }
}

// A workgroup bins `per_wg` consecutive Gaussians (a multiple of
// kBinThreads * kBinPer, in batches of kBinPer per thread): with the C3
// microbench's uniformly scattered Gaussians every workgroup touches every
// tile, so the global atomics per launch are (workgroups x tiles) and the
// workgroups are made few and large.
__global__ void __launch_bounds__(kBinThreads)
k_tile_count(int64_t P, int64_t per_wg, int gx, int ntiles, const uint4* __restrict__ dup,
             uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t s_hist[];
  for (int t = threadIdx.x; t < ntiles; t += kBinThreads) s_hist[t] = 0u;
  __syncthreads();
  const int64_t g0 = (int64_t)blockIdx.x * per_wg, g1 = min(P, g0 + per_wg);
  for (int64_t b0 = g0; b0 < g1; b0 += kBinThreads * kBinPer) {
    uint4 d[kBinPer];
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
      const int64_t i = b0 + k * kBinThreads + threadIdx.x;
      d[k] = i < g1 ? dup[i] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < kBinPer; ++k)
      for_each_tile(d[k], gx, [&](int t) { atomicAdd(&s_hist[t], 1u); });
  }
  __syncthreads();
  for (int t = threadIdx.x; t < ntiles; t += kBinThreads)
    if (s_hist[t]) atomicAdd(&counts[t], s_hist[t]);
}

// counts -> offsets in place (the fill cursors) and ranges clipped to the
// binning capacity
__global__ void __launch_bounds__(1024)
k_tile_scan(int ntiles, uint32_t* __restrict__ cursor, uint2* __restrict__ ranges, uint32_t cap) {
  __shared__ uint32_t s_w[16];
  uint32_t carry = 0;
  for (int c0 = 0; c0 < ntiles; c0 += 1024) {
    const int c = c0 + threadIdx.x;
    const uint32_t v = c < ntiles ? cursor[c] : 0u;
    uint32_t total = 0;
    const uint32_t ex = block_excl_scan<1024>(v, s_w, &total);
    if (c < ntiles) {
      const uint32_t off = carry + ex;
      cursor[c] = off;
      ranges[c] = make_uint2(min(off, cap), (uint32_t)min((uint64_t)off + v, (uint64_t)cap));
    }
    carry += total;
  }
}

__global__ void __launch_bounds__(kBinThreads)
k_tile_fill(int64_t P, int64_t per_wg, int gx, int ntiles, const uint4* __restrict__ dup,
            const uint32_t* __restrict__ dkey, uint32_t* __restrict__ cursor,
            uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, uint32_t cap) {
  extern __shared__ uint32_t s_mem[];
  uint32_t* s_cnt = s_mem;
  uint32_t* s_base = s_mem + ntiles;
  for (int t = threadIdx.x; t < ntiles; t += kBinThreads) s_cnt[t] = 0u;
  __syncthreads();
  const int64_t g0 = (int64_t)blockIdx.x * per_wg, g1 = min(P, g0 + per_wg);
  for (int64_t b0 = g0; b0 < g1; b0 += kBinThreads * kBinPer) {
    uint4 d[kBinPer];
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
      const int64_t i = b0 + k * kBinThreads + threadIdx.x;
      d[k] = i < g1 ? dup[i] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < kBinPer; ++k)
      for_each_tile(d[k], gx, [&](int t) { atomicAdd(&s_cnt[t], 1u); });
  }
  __syncthreads();
  // one cursor reservation per touched tile
  for (int t = threadIdx.x; t < ntiles; t += kBinThreads) {
    const uint32_t c = s_cnt[t];
    if (c) {
      s_base[t] = atomicAdd(&cursor[t], c);
      s_cnt[t] = 0u;
    }
  }
  __syncthreads();
  for (int64_t b0 = g0; b0 < g1; b0 += kBinThreads * kBinPer) {
    uint4 d[kBinPer];
    uint32_t key[kBinPer];
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
      const int64_t i = b0 + k * kBinThreads + threadIdx.x;
      d[k] = i < g1 ? dup[i] : make_uint4(0u, 0u, 0u, 0u);
      key[k] = i < g1 ? dkey[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
      const uint32_t i = (uint32_t)(b0 + k * kBinThreads + threadIdx.x);
      for_each_tile(d[k], gx, [&](int t) {
        const uint32_t pos = s_base[t] + atomicAdd(&s_cnt[t], 1u);
        if (pos < cap) {
          kout[pos] = key[k];
          vout[pos] = i;
        }
      });
    }
  }
}

// One radix pass of k_tile_sort: digits of the depth key (Digit) or of the
// Gaussian index (shift / bits)
struct TsPass {
  bool index;
  int shift, bits;
};

__device__ __forceinline__ uint32_t ts_digit(const TsPass& ps, const Digit& dg, uint32_t key,
                                             uint32_t val) {
  if (ps.index) return (val >> ps.shift) & ((1u << ps.bits) - 1u);
  Digit d = dg;
  d.shift = ps.shift;
  d.bits = ps.bits;
  return d(key);
}

struct TsLds {
  uint32_t k[kTSCap];
  uint32_t v[kTSCap];
  uint32_t cnt[kTSWaves][256];  // per (wave, digit) counts -> first slots
  uint32_t run[256];            // chunked passes: next slot per digit
  uint32_t w[kTSWaves];
};

// per-(wave, digit) counts of one chunk's items (added to t.cnt)
__device__ __forceinline__ void ts_count(TsLds& t, const TsPass& ps, const Digit& dg,
                                         const uint32_t (&key)[kTSIpt],
                                         const uint32_t (&val)[kTSIpt], int ipt, int m,
                                         int base_w) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < kTSIpt; ++j)   // order-free: one LDS atomic per item
    if (j < ipt && base_w + j * 64 + lane < m) atomicAdd(&t.cnt[w][ts_digit(ps, dg, key[j], val[j])], 1u);
}

// slots of one chunk's items in item order (t.cnt holds each (wave, digit)'s
// first slot and is advanced); put(j, slot) stores item j
template <typename Put>
__device__ __forceinline__ void ts_rank(TsLds& t, const TsPass& ps, const Digit& dg,
                                        const uint32_t (&key)[kTSIpt],
                                        const uint32_t (&val)[kTSIpt], int ipt, int m,
                                        int base_w, Put&& put) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < kTSIpt; ++j) {
    if (j < ipt) {
      const bool ok = base_w + j * 64 + lane < m;
      const uint32_t d = ts_digit(ps, dg, key[j], val[j]);
      const uint64_t peers = match_peers(d, ok, ps.bits);
      if (ok) {
        const uint32_t b = t.cnt[w][d];
        put(j, b + (uint32_t)__popcll(peers & lanemask_lt(lane)));
        if ((peers >> lane) == 1ull) t.cnt[w][d] = b + (uint32_t)__popcll(peers);
      }
      wave_lds_sync();
    }
  }
}

__device__ __forceinline__ void ts_zero_cnt(TsLds& t) {
  for (int k = threadIdx.x; k < kTSWaves * 256; k += kTSThreads) (&t.cnt[0][0])[k] = 0u;
}

// digit-major first slots from the per-wave counts, starting at run[] (or
// at the exclusive scan of the digit totals when `scan`)
__device__ __forceinline__ void ts_offsets(TsLds& t, bool scan) {
  const int d = threadIdx.x;
  uint32_t tot = 0;
  if (d < 256) {
#pragma unroll
    for (int k = 0; k < kTSWaves; ++k) tot += t.cnt[k][d];
  }
  uint32_t b = 0;
  if (scan) b = block_excl_scan<kTSThreads>(d < 256 ? tot : 0u, t.w);
  if (d < 256) {
    if (!scan) b = t.run[d];
#pragma unroll
    for (int k = 0; k < kTSWaves; ++k) {
      const uint32_t c = t.cnt[k][d];
      t.cnt[k][d] = b;
      b += c;
    }
    t.run[d] = b;
  }
}

__global__ void __launch_bounds__(kTSThreads)
k_tile_sort(int ntiles, const uint2* __restrict__ ranges, uint32_t* __restrict__ kA,
            uint32_t* __restrict__ vA, uint32_t* __restrict__ kB, uint32_t* __restrict__ vB,
            Digit dg_in, int dbits, int ibits) {
  __shared__ TsLds t;
  const Digit dg = dg_in.live();
  const int tile = xcd_tile(blockIdx.x, ntiles);
  const uint2 r = ranges[tile];
  const int n = (int)(r.y - r.x);
  const int64_t lo = r.x;
  if (n <= 1) {
    if (n == 1 && threadIdx.x == 0) vB[lo] = vA[lo];
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // pass plan: depth digits; on a tie, index digits then depth digits again
  auto plan = [](int bits, int p, int& shift, int& width) {
    const int passes = max(1, (bits + 7) / 8);
    width = (bits + passes - 1) / passes;
    shift = p * width;
    return passes;
  };
  const int dpass = max(1, (dbits + 7) / 8), ipass = max(1, (ibits + 7) / 8);
  auto pass_of = [&](int q, bool tie) -> TsPass {
    int shift, width;
    if (!tie || q >= ipass + dpass) {
      const int p = tie ? q - ipass - dpass : q;
      plan(dbits, p, shift, width);
      return {false, shift, min(dbits, shift + width) - shift};
    }
    if (q < dpass) {                      // (the first depth passes: redone)
      plan(dbits, q, shift, width);
      return {false, shift, min(dbits, shift + width) - shift};
    }
    plan(ibits, q - dpass, shift, width);
    return {true, shift, min(ibits, shift + width) - shift};
  };

  if (n <= kTSCap) {
    // ---- LDS-resident: items in registers, each pass ranks and stages
    const int ipt = (n + kTSThreads - 1) / kTSThreads;
    const int base_w = w * 64 * ipt;
    uint32_t key[kTSIpt], val[kTSIpt];
#pragma unroll
    for (int j = 0; j < kTSIpt; ++j) {
      const int s = base_w + j * 64 + lane;
      const bool ok = j < ipt && s < n;
      key[j] = ok ? kA[lo + s] : 0u;
      val[j] = ok ? vA[lo + s] : 0u;
    }
    bool tie = false;
    int total = dpass;
    for (int q = 0; q < total; ++q) {
      const TsPass ps = pass_of(q, tie);
      ts_zero_cnt(t);
      __syncthreads();
      ts_count(t, ps, dg, key, val, ipt, n, base_w);
      __syncthreads();
      ts_offsets(t, true);
      __syncthreads();
      ts_rank(t, ps, dg, key, val, ipt, n, base_w, [&](int j, uint32_t sl) {
        t.k[sl] = key[j];
        t.v[sl] = val[j];
      });
      __syncthreads();
      bool eq = false;
#pragma unroll
      for (int j = 0; j < kTSIpt; ++j) {
        const int s = base_w + j * 64 + lane;
        if (j < ipt && s < n) {
          key[j] = t.k[s];
          val[j] = t.v[s];
          eq |= q == total - 1 && !tie && s + 1 < n && t.k[s + 1] == key[j];
        }
      }
      // equal depth keys after the depth passes keep their (arbitrary) fill
      // order: a run of <= 32 equal keys is put in index order in place by
      // the thread holding its first item; a longer run sends the tile
      // through the index passes and the depth passes again
      if (q == total - 1 && !tie && __syncthreads_or(eq)) {
        bool longrun = false;
#pragma unroll 1
        for (int j = 0; j < ipt; ++j) {
          const int s = base_w + j * 64 + lane;
          const uint32_t kj = s < n ? t.k[s] : 0u;
          if (s + 1 < n && t.k[s + 1] == kj && (s == 0 || t.k[s - 1] != kj)) {
            int L = 2;
            while (L <= 32 && s + L < n && t.k[s + L] == kj) ++L;
            if (L > 32) {
              longrun = true;
            } else {
              for (int a = s + 1; a < s + L; ++a) {
                const uint32_t x = t.v[a];
                int b = a - 1;
                while (b >= s && t.v[b] > x) {
                  t.v[b + 1] = t.v[b];
                  --b;
                }
                t.v[b + 1] = x;
              }
            }
          }
        }
        if (__syncthreads_or(longrun)) {
          tie = true;
          total = dpass + ipass + dpass;
        } else {
#pragma unroll
          for (int j = 0; j < kTSIpt; ++j) {
            const int s = base_w + j * 64 + lane;
            if (j < ipt && s < n) val[j] = t.v[s];
          }
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kTSIpt; ++j) {
      const int s = base_w + j * 64 + lane;
      if (j < ipt && s < n) vB[lo + s] = val[j];
    }
    return;
  }

  // ---- larger tiles: the same passes chunk by chunk, ping-pong between
  // (kA, vA) and (kB, vB) over the tile's range
  uint32_t* ks = kA + lo;
  uint32_t* vs = vA + lo;
  uint32_t* kd = kB + lo;
  uint32_t* vd = vB + lo;
  bool tie = false;
  int total = dpass;
  for (int q = 0; q < total; ++q) {
    const TsPass ps = pass_of(q, tie);
    // sweep 1: digit totals -> first slot of every digit
    ts_zero_cnt(t);
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += kTSCap) {
      const int m = min(kTSCap, n - c0);
      const int ipt = (m + kTSThreads - 1) / kTSThreads, base_w = w * 64 * ipt;
      uint32_t key[kTSIpt], val[kTSIpt];
#pragma unroll
      for (int j = 0; j < kTSIpt; ++j) {
        const int s = base_w + j * 64 + lane;
        const bool ok = j < ipt && s < m;
        key[j] = ok ? ks[c0 + s] : 0u;
        val[j] = ok ? vs[c0 + s] : 0u;
      }
      ts_count(t, ps, dg, key, val, ipt, m, base_w);
    }
    __syncthreads();
    {
      const int d = threadIdx.x;
      uint32_t tot = 0;
      if (d < 256) {
#pragma unroll
        for (int k = 0; k < kTSWaves; ++k) tot += t.cnt[k][d];
      }
      const uint32_t b = block_excl_scan<kTSThreads>(d < 256 ? tot : 0u, t.w);
      if (d < 256) t.run[d] = b;
    }
    __syncthreads();
    // sweep 2: every chunk in order, slots continuing from run[]
    for (int c0 = 0; c0 < n; c0 += kTSCap) {
      const int m = min(kTSCap, n - c0);
      const int ipt = (m + kTSThreads - 1) / kTSThreads, base_w = w * 64 * ipt;
      uint32_t key[kTSIpt], val[kTSIpt];
#pragma unroll
      for (int j = 0; j < kTSIpt; ++j) {
        const int s = base_w + j * 64 + lane;
        const bool ok = j < ipt && s < m;
        key[j] = ok ? ks[c0 + s] : 0u;
        val[j] = ok ? vs[c0 + s] : 0u;
      }
      ts_zero_cnt(t);
      __syncthreads();
      ts_count(t, ps, dg, key, val, ipt, m, base_w);
      __syncthreads();
      ts_offsets(t, false);
      __syncthreads();
      ts_rank(t, ps, dg, key, val, ipt, m, base_w, [&](int j, uint32_t sl) {
        kd[sl] = key[j];
        vd[sl] = val[j];
      });
      __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    uint32_t* tk = ks;
    ks = kd;
    kd = tk;
    uint32_t* tv = vs;
    vs = vd;
    vd = tv;
    if (q == total - 1 && !tie) {
      bool eq = false;
      for (int s = threadIdx.x; s + 1 < n; s += kTSThreads) eq |= ks[s] == ks[s + 1];
      if (__syncthreads_or(eq)) {
        tie = true;
        total = dpass + ipass + dpass;
      }
    }
  }
  // the sorted values are in vs; the output range is vB's
  if (vs != vB + lo)
    for (int s = threadIdx.x; s < n; s += kTSThreads) vB[lo + s] = vs[s];
}

// --------------------------------------------------------------- blend ----
__global__ void __launch_bounds__(BS)
k_blend(int W, int H, int gx, int ntiles, const uint2* __restrict__ ranges,
        const uint32_t* __restrict__ point_list, GeomState g, const float* __restrict__ bg,
        float* __restrict__ final_T, uint32_t* __restrict__ n_contrib,
        float* __restrict__ out) {
  __shared__ float4 s_r0[BS];
  __shared__ float4 s_r1[BS];  // (conic.c, opacity, r, g)
  __shared__ float s_b[BS];
  const int tile = xcd_tile(blockIdx.x, ntiles);
  const int tx = tile % gx, ty = tile / gx;
  const int lx = threadIdx.x % BX, ly = threadIdx.x / BX;
  const int px = tx * BX + lx, py = ty * BY + ly;
  const bool inside = px < W && py < H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];
  const int todo_total = (int)(range.y - range.x);
  const int rounds = (todo_total + BS - 1) / BS;
  bool done = !inside;
  float T = 1.0f;
  uint32_t contributor = 0, last_contributor = 0;
  float C0 = 0.f, C1 = 0.f, C2 = 0.f;
  int todo = todo_total;
  for (int rd = 0; rd < rounds; ++rd, todo -= BS) {
    if (__syncthreads_count(done) == BS) break;
    const int prog = rd * BS + threadIdx.x;
    if ((int64_t)range.x + prog < range.y) {
      const uint32_t id = point_list[range.x + prog];
      s_r0[threadIdx.x] = g.rec0[id];
      s_r1[threadIdx.x] = g.rec1[id];
      s_b[threadIdx.x] = g.blue[id];
    }
    __syncthreads();
    const int n = todo < BS ? todo : BS;
    for (int j = 0; !done && j < n; ++j) {
      ++contributor;
      const float4 a = s_r0[j];
      const float4 b = s_r1[j];
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = -0.5f * (a.z * dx * dx + b.x * dy * dy) - a.w * dx * dy;
      if (power > 0.0f) continue;
      const float alpha = fminf(0.99f, b.y * fexp(power));
      if (alpha < 1.0f / 255.0f) continue;
      const float test_T = T * (1.0f - alpha);
      if (test_T < 0.0001f) {
        done = true;
        continue;
      }
      // C += feature * alpha * T, evaluated left to right as the reference
      C0 = C0 + b.z * alpha * T;
      C1 = C1 + b.w * alpha * T;
      C2 = C2 + s_b[j] * alpha * T;
      T = test_T;
      last_contributor = contributor;
    }
  }
  if (inside) {
    const int pid = py * W + px;
    final_T[pid] = T;
    n_contrib[pid] = last_contributor;
    out[pid] = C0 + T * bg[0];
    out[H * W + pid] = C1 + T * bg[1];
    out[2 * H * W + pid] = C2 + T * bg[2];
  }
}

// ----------------------------------------------------------- backward -----
struct ZeroList {
  float* p[10];
  int64_t n[10];
  int cnt;
};

// grid (chunks, list entries): zero every listed array, 16 B per store
// where the base is 16-B aligned
__global__ void __launch_bounds__(kThreads) k_zero_multi(ZeroList z) {
  float* __restrict__ p = z.p[blockIdx.y];
  const int64_t n = z.n[blockIdx.y];
  const int64_t i0 = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 4;
  if (i0 >= n) return;
  if (i0 + 4 <= n && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    *reinterpret_cast<float4*>(p + i0) = make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    for (int64_t e = i0; e < n && e < i0 + 4; ++e) p[e] = 0.0f;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Transposed wave reduction of 8 values: each halving step keeps half of
// the values and trades the other half with the partner lane, so 8 sums
// cost 4 + 2 + 1 + 3 shuffles instead of 8 x 6.  Lane l ends with the full
// sum of value ((l >> 5) & 1) * 4 + ((l >> 4) & 1) * 2 + ((l >> 3) & 1).
__device__ __forceinline__ float wave_sum8_t(const float (&v)[8], int lane) {
  float w[4], x[2];
  const bool b32 = lane & 32, b16 = lane & 16, b8 = lane & 8;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float send = b32 ? v[k] : v[k + 4];
    const float keep = b32 ? v[k + 4] : v[k];
    w[k] = keep + __shfl_xor(send, 32, 64);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float send = b16 ? w[k] : w[k + 2];
    const float keep = b16 ? w[k + 2] : w[k];
    x[k] = keep + __shfl_xor(send, 16, 64);
  }
  float y = (b8 ? x[1] : x[0]) + __shfl_xor(b8 ? x[0] : x[1], 8, 64);
  y += __shfl_xor(y, 4, 64);
  y += __shfl_xor(y, 2, 64);
  y += __shfl_xor(y, 1, 64);
  return y;
}

// Gradient slots per Gaussian in the LDS batch accumulator: mean2D x/y,
// conic x/y/w, opacity, colour r/g/b.
constexpr int kGS = 9;

__global__ void __launch_bounds__(BS)
k_blend_backward(int W, int H, int gx, int ntiles, const uint2* __restrict__ ranges,
                 const uint32_t* __restrict__ point_list, GeomState g,
                 const float* __restrict__ bg, const float* __restrict__ final_Ts,
                 const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix,
                 float* __restrict__ dL_dmean2D, float* __restrict__ dL_dconic,
                 float* __restrict__ dL_dopacity, float* __restrict__ dL_dcolors) {
  __shared__ float4 s_r0[BS];
  __shared__ float4 s_r1[BS];
  __shared__ float s_b[BS];
  __shared__ uint32_t s_id[BS];
  // per-batch block sums: the 4 waves' reduced gradients meet in LDS and
  // each (Gaussian, tile) pair issues its 9 global atomics once, from the
  // lane that owns the Gaussian, instead of once per wave from lane 0
  __shared__ float s_acc[BS * kGS];
  __shared__ int s_hit[BS];
  const int tile = xcd_tile(blockIdx.x, ntiles);
  const int tx = tile % gx, ty = tile / gx;
  const int lx = threadIdx.x % BX, ly = threadIdx.x / BX;
  const int px = tx * BX + lx, py = ty * BY + ly;
  const bool inside = px < W && py < H;
  const int pid = py * W + px;
  const float pxf = (float)px, pyf = (float)py;
  __shared__ uint32_t s_maxlc;
  const uint2 range = ranges[tile];
  const uint32_t last_contributor = inside ? n_contrib[pid] : 0;
  // Entries at or past every pixel's last contributor (the forward pass
  // stopped before them) contribute nothing: the replay starts at the
  // tile's largest n_contrib instead of the back of the list.
  const int lane = threadIdx.x & 63;
  {
    uint32_t m = last_contributor;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if (threadIdx.x == 0) s_maxlc = 0;
    __syncthreads();
    if (lane == 0) atomicMax(&s_maxlc, m);
    __syncthreads();
  }
  const int todo_total = (int)min(range.y - range.x, s_maxlc);
  const uint32_t end = range.x + (uint32_t)todo_total;
  const int rounds = (todo_total + BS - 1) / BS;
  const float T_final = inside ? final_Ts[pid] : 0.0f;
  float T = T_final;
  uint32_t contributor = (uint32_t)todo_total;
  float dpix0 = 0.f, dpix1 = 0.f, dpix2 = 0.f;
  if (inside) {
    dpix0 = dL_dpix[pid];
    dpix1 = dL_dpix[H * W + pid];
    dpix2 = dL_dpix[2 * H * W + pid];
  }
  const float bg_dot = bg[0] * dpix0 + bg[1] * dpix1 + bg[2] * dpix2;
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
  float last_alpha = 0.f, lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  const int vslot = ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
  int todo = todo_total;
  auto flush = [&](int n) {
    // one lane per Gaussian of the finished batch
    const int t = threadIdx.x;
    if (t < n && s_hit[t]) {
      const uint32_t id = s_id[t];
      const float* a = s_acc + t * kGS;
      atomicAdd(&dL_dmean2D[id * 3 + 0], a[0]);
      atomicAdd(&dL_dmean2D[id * 3 + 1], a[1]);
      atomicAdd(&dL_dconic[id * 4 + 0], a[2]);
      atomicAdd(&dL_dconic[id * 4 + 1], a[3]);
      atomicAdd(&dL_dconic[id * 4 + 3], a[4]);
      atomicAdd(&dL_dopacity[id], a[5]);
      atomicAdd(&dL_dcolors[id * 3 + 0], a[6]);
      atomicAdd(&dL_dcolors[id * 3 + 1], a[7]);
      atomicAdd(&dL_dcolors[id * 3 + 2], a[8]);
    }
  };
  for (int rd = 0; rd < rounds; ++rd, todo -= BS) {
    __syncthreads();
    if (rd > 0) flush(BS);
    __syncthreads();
    const int prog = rd * BS + threadIdx.x;
    if (prog < todo_total) {
      const uint32_t id = point_list[end - prog - 1];
      s_id[threadIdx.x] = id;
      s_r0[threadIdx.x] = g.rec0[id];
      s_r1[threadIdx.x] = g.rec1[id];
      s_b[threadIdx.x] = g.blue[id];
    }
#pragma unroll
    for (int k = 0; k < kGS; ++k) s_acc[threadIdx.x * kGS + k] = 0.f;
    s_hit[threadIdx.x] = 0;
    __syncthreads();
    const int n = todo < BS ? todo : BS;
    for (int j = 0; j < n; ++j) {
      --contributor;
      bool ok = inside && contributor < last_contributor;
      const float4 a = s_r0[j];
      const float4 b = s_r1[j];
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = -0.5f * (a.z * dx * dx + b.x * dy * dy) - a.w * dx * dy;
      ok = ok && !(power > 0.0f);
      const float G = fexp(power);
      const float alpha = fminf(0.99f, b.y * G);
      ok = ok && !(alpha < 1.0f / 255.0f);
      if (!__any(ok)) continue;
      float gv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      float gb = 0.f;
      if (ok) {
        T = T / (1.0f - alpha);
        const float dchannel_dcolor = alpha * T;
        const float c0 = b.z, c1 = b.w, c2 = s_b[j];
        acc0 = last_alpha * lc0 + (1.0f - last_alpha) * acc0;
        acc1 = last_alpha * lc1 + (1.0f - last_alpha) * acc1;
        acc2 = last_alpha * lc2 + (1.0f - last_alpha) * acc2;
        lc0 = c0; lc1 = c1; lc2 = c2;
        float dL_dalpha = (c0 - acc0) * dpix0 + (c1 - acc1) * dpix1 + (c2 - acc2) * dpix2;
        gv[6] = dchannel_dcolor * dpix0;
        gv[7] = dchannel_dcolor * dpix1;
        gb = dchannel_dcolor * dpix2;
        dL_dalpha = dL_dalpha * T;
        last_alpha = alpha;
        dL_dalpha = dL_dalpha + (-T_final / (1.0f - alpha)) * bg_dot;
        const float dL_dG = b.y * dL_dalpha;
        const float gdx = G * dx, gdy = G * dy;
        const float dG_ddelx = -gdx * a.z - gdy * a.w;
        const float dG_ddely = -gdy * b.x - gdx * a.w;
        gv[0] = dL_dG * dG_ddelx * ddelx_dx;
        gv[1] = dL_dG * dG_ddely * ddely_dy;
        gv[2] = -0.5f * gdx * dx * dL_dG;
        gv[3] = -0.5f * gdx * dy * dL_dG;
        gv[4] = -0.5f * gdy * dy * dL_dG;
        gv[5] = G * dL_dalpha;
      }
      const float r8 = wave_sum8_t(gv, lane);
      gb = wave_sum(gb);
      if ((lane & 7) == 0) atomicAdd(&s_acc[j * kGS + vslot], r8);
      if (lane == 0) {
        atomicAdd(&s_acc[j * kGS + 8], gb);
        s_hit[j] = 1;
      }
    }
  }
  __syncthreads();
  if (rounds > 0) flush(todo_total - (rounds - 1) * BS);
}

// Per-Gaussian chain rule: conic -> 2-D cov -> (3-D cov, view mean) and
// screen mean -> world mean; SH colour -> coefficients / view direction;
// 3-D cov -> scale / rotation.
__global__ void __launch_bounds__(kThreads)
k_preprocess_backward(int64_t P, Cam cam, const float* __restrict__ means,
                      const float* __restrict__ scales, const float* __restrict__ rots,
                      const float* __restrict__ cov_pre, const float* __restrict__ shs,
                      const int32_t* __restrict__ radii, GeomState g,
                      const float* __restrict__ vm, const float* __restrict__ pm,
                      const float* __restrict__ campos, const float* __restrict__ dL_dmean2D,
                      const float* __restrict__ dL_dconic, const float* __restrict__ dL_dcolor,
                      float* __restrict__ dL_dmeans, float* __restrict__ dL_dcov,
                      float* __restrict__ dL_dsh, float* __restrict__ dL_dscale,
                      float* __restrict__ dL_drot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  if (!(radii[i] > 0)) {
    // culled: every per-Gaussian gradient is zero (written here, so the
    // caller's buffers need no memset)
#pragma unroll
    for (int k = 0; k < 3; ++k) dL_dmeans[i * 3 + k] = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) dL_dcov[i * 6 + k] = 0.f;
    if (shs)
      for (int k = 0; k < cam.M * 3; ++k) dL_dsh[i * (int64_t)cam.M * 3 + k] = 0.f;
    if (scales && dL_dscale) {
#pragma unroll
      for (int k = 0; k < 3; ++k) dL_dscale[i * 3 + k] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) dL_drot[i * 4 + k] = 0.f;
    }
    return;
  }
  const float mx = means[i * 3 + 0], my = means[i * 3 + 1], mz = means[i * 3 + 2];
  float cov3[6];   // the forward's 3-D covariance, recomputed (not stored)
  if (cov_pre) {
#pragma unroll
    for (int k = 0; k < 6; ++k) cov3[k] = cov_pre[i * 6 + k];
  } else {
    cov3d_from_scale_rot(scales + i * 3, cam.scale_mod, rots + i * 4, cov3);
  }
  Ewa e = ewa_project(mx, my, mz, cov3, vm, cam.fx, cam.fy, cam.tanfx, cam.tanfy);
  const float a = e.a + 0.3f, b = e.b, c = e.c + 0.3f;
  const float dcx = dL_dconic[i * 4 + 0], dcy = dL_dconic[i * 4 + 1], dcz = dL_dconic[i * 4 + 3];
  const float denom = a * c - b * b;
  const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
  float da = 0.f, db = 0.f, dc = 0.f;
  float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* T = e.T;  // T[0..2] row 0, T[3..5] row 1
  if (denom2inv != 0.0f) {
    da = denom2inv * (-c * c * dcx + 2.0f * b * c * dcy + (denom - a * c) * dcz);
    dc = denom2inv * (-a * a * dcz + 2.0f * a * b * dcy + (denom - a * c) * dcx);
    db = denom2inv * 2.0f * (b * c * dcx - (denom + 2.0f * b * b) * dcy + a * b * dcz);
    dcov[0] = T[0] * T[0] * da + T[0] * T[3] * db + T[3] * T[3] * dc;
    dcov[3] = T[1] * T[1] * da + T[1] * T[4] * db + T[4] * T[4] * dc;
    dcov[5] = T[2] * T[2] * da + T[2] * T[5] * db + T[5] * T[5] * dc;
    dcov[1] = 2.0f * T[0] * T[1] * da + (T[0] * T[4] + T[1] * T[3]) * db + 2.0f * T[3] * T[4] * dc;
    dcov[2] = 2.0f * T[0] * T[2] * da + (T[0] * T[5] + T[2] * T[3]) * db + 2.0f * T[3] * T[5] * dc;
    dcov[4] = 2.0f * T[2] * T[1] * da + (T[1] * T[5] + T[2] * T[4]) * db + 2.0f * T[4] * T[5] * dc;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) dL_dcov[i * 6 + k] = dcov[k];
  const float V[9] = {cov3[0], cov3[1], cov3[2], cov3[1], cov3[3], cov3[4],
                      cov3[2], cov3[4], cov3[5]};
  float dT0[3], dT1[3];
  for (int k = 0; k < 3; ++k) {
    const float t0v = T[0] * V[k] + T[1] * V[3 + k] + T[2] * V[6 + k];
    const float t1v = T[3] * V[k] + T[4] * V[3 + k] + T[5] * V[6 + k];
    dT0[k] = 2.0f * t0v * da + t1v * db;
    dT1[k] = 2.0f * t1v * dc + t0v * db;
  }
  // T = J Wv, Wv[r][c] = vm[r + 4c]
  const float dJ00 = vm[0] * dT0[0] + vm[4] * dT0[1] + vm[8] * dT0[2];
  const float dJ02 = vm[2] * dT0[0] + vm[6] * dT0[1] + vm[10] * dT0[2];
  const float dJ11 = vm[1] * dT1[0] + vm[5] * dT1[1] + vm[9] * dT1[2];
  const float dJ12 = vm[2] * dT1[0] + vm[6] * dT1[1] + vm[10] * dT1[2];
  const float tz = 1.0f / e.tz, tz2 = tz * tz, tz3 = tz2 * tz;
  const float dtx = e.xmul * -cam.fx * tz2 * dJ02;
  const float dty = e.ymul * -cam.fy * tz2 * dJ12;
  const float dtz = -cam.fx * tz2 * dJ00 - cam.fy * tz2 * dJ11 +
                    (2.0f * cam.fx * e.tx) * tz3 * dJ02 + (2.0f * cam.fy * e.ty) * tz3 * dJ12;
  float gmx = vm[0] * dtx + vm[1] * dty + vm[2] * dtz;
  float gmy = vm[4] * dtx + vm[5] * dty + vm[6] * dtz;
  float gmz = vm[8] * dtx + vm[9] * dty + vm[10] * dtz;

  // screen-space mean -> world mean
  float ph[4];
  xform44(pm, mx, my, mz, ph);
  const float mw = 1.0f / (ph[3] + 0.0000001f);
  const float mul1 = (pm[0] * mx + pm[4] * my + pm[8] * mz + pm[12]) * mw * mw;
  const float mul2 = (pm[1] * mx + pm[5] * my + pm[9] * mz + pm[13]) * mw * mw;
  const float d2x = dL_dmean2D[i * 3 + 0], d2y = dL_dmean2D[i * 3 + 1];
  gmx = gmx + ((pm[0] * mw - pm[3] * mul1) * d2x + (pm[1] * mw - pm[3] * mul2) * d2y);
  gmy = gmy + ((pm[4] * mw - pm[7] * mul1) * d2x + (pm[5] * mw - pm[7] * mul2) * d2y);
  gmz = gmz + ((pm[8] * mw - pm[11] * mul1) * d2x + (pm[9] * mw - pm[11] * mul2) * d2y);

  if (shs) {
    const float ox = mx - campos[0], oy = my - campos[1], oz = mz - campos[2];
    const float len = sqrtf(ox * ox + oy * oy + oz * oz);
    const float x = ox / len, y = oy / len, z = oz / len;
    float B[16], dX[16], dY[16], dZ[16];
    sh_basis(cam.D, x, y, z, B);
    sh_basis_grad(cam.D, x, y, z, dX, dY, dZ);
    const int nb = (cam.D + 1) * (cam.D + 1);
    const float* sh = shs + i * (int64_t)cam.M * 3;
    float* dsh = dL_dsh + i * (int64_t)cam.M * 3;
    float drgb[3];
    for (int ch = 0; ch < 3; ++ch)
      drgb[ch] = ((g.clamped[i] >> ch) & 1u) ? 0.0f : dL_dcolor[i * 3 + ch];
    for (int k = 0; k < cam.M; ++k)
      for (int ch = 0; ch < 3; ++ch) dsh[k * 3 + ch] = k < nb ? B[k] * drgb[ch] : 0.0f;
    float ddx = 0.f, ddy = 0.f, ddz = 0.f;
    for (int k = 1; k < nb; ++k)
      for (int ch = 0; ch < 3; ++ch) {
        const float s = sh[k * 3 + ch] * drgb[ch];
        ddx = ddx + dX[k] * s;
        ddy = ddy + dY[k] * s;
        ddz = ddz + dZ[k] * s;
      }
    // d normalize(o) / d o applied to (ddx, ddy, ddz)
    const float s2 = ox * ox + oy * oy + oz * oz;
    const float inv32 = 1.0f / sqrtf(s2 * s2 * s2);
    gmx = gmx + ((s2 - ox * ox) * ddx - oy * ox * ddy - oz * ox * ddz) * inv32;
    gmy = gmy + (-ox * oy * ddx + (s2 - oy * oy) * ddy - oz * oy * ddz) * inv32;
    gmz = gmz + (-ox * oz * ddx - oy * oz * ddy + (s2 - oz * oz) * ddz) * inv32;
  }
  dL_dmeans[i * 3 + 0] = gmx;
  dL_dmeans[i * 3 + 1] = gmy;
  dL_dmeans[i * 3 + 2] = gmz;

  if (scales && dL_dscale) {
    // Sigma = M M^T, M = R diag(s): dL/dM = (G + G^T) M with G = dL/dSigma
    const float* q = rots + i * 4;
    const float r = q[0], x = q[1], y = q[2], z = q[3];
    const float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                        2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                        2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
    const float s[3] = {cam.scale_mod * scales[i * 3 + 0], cam.scale_mod * scales[i * 3 + 1],
                        cam.scale_mod * scales[i * 3 + 2]};
    const float* dc6 = dcov;
    // symmetric gradient matrix: off-diagonal entries shared by (i,j),(j,i)
    const float Gs[9] = {dc6[0], 0.5f * dc6[1], 0.5f * dc6[2], 0.5f * dc6[1], dc6[3],
                         0.5f * dc6[4], 0.5f * dc6[2], 0.5f * dc6[4], dc6[5]};
    float dM[9];
    for (int ii = 0; ii < 3; ++ii)
      for (int jj = 0; jj < 3; ++jj) {
        float acc = 0.f;
        for (int k = 0; k < 3; ++k) acc = acc + 2.0f * Gs[3 * ii + k] * R[3 * k + jj] * s[jj];
        dM[3 * ii + jj] = acc;
      }
    for (int jj = 0; jj < 3; ++jj)
      dL_dscale[i * 3 + jj] =
          cam.scale_mod * (dM[jj] * R[jj] + dM[3 + jj] * R[3 + jj] + dM[6 + jj] * R[6 + jj]);
    float dR[9];
    for (int k = 0; k < 9; ++k) dR[k] = dM[k] * s[k % 3];
    // dR/dq for the (unnormalised) quaternion formula above
    dL_drot[i * 4 + 0] = 2.f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
    dL_drot[i * 4 + 1] = 2.f * (y * dR[1] + z * dR[2] + y * dR[3] - 2.f * x * dR[4] - r * dR[5] +
                                z * dR[6] + r * dR[7] - 2.f * x * dR[8]);
    dL_drot[i * 4 + 2] = 2.f * (-2.f * y * dR[0] + x * dR[1] + r * dR[2] + x * dR[3] + z * dR[5] -
                                r * dR[6] + z * dR[7] - 2.f * y * dR[8]);
    dL_drot[i * 4 + 3] = 2.f * (-2.f * z * dR[0] - r * dR[1] + x * dR[2] + r * dR[3] -
                                2.f * z * dR[4] + y * dR[5] + x * dR[6] + y * dR[7]);
  }
}

__global__ void k_mark_visible(int64_t P, const float* __restrict__ means,
                               const float* __restrict__ vm, uint8_t* __restrict__ present) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float pv[3];
  xform43(vm, means[i * 3 + 0], means[i * 3 + 1], means[i * 3 + 2], pv);
  present[i] = pv[2] > 0.2f;
}

// ------------------------------------------------------------- timing -----
struct Timing {
  bool enabled = false;
  hipEvent_t ev[7] = {};
  bool created = false;
  bool valid = false;
};
thread_local Timing g_timing;

// forward binning: 1 = per-tile binning + LDS depth sort, 0 = the global
// depth sort + tile sort (the default; gsr_set_binning, A/B hook)
int g_binning = 0;

// depth-key range of the last gsr_preprocess on this thread (read back with
// num_rendered), keyed by its geometry buffer
struct KeyRange {
  const void* geom = nullptr;
  int64_t P = 0;
  uint32_t kmin = 0, kmax = 0;
};
thread_local KeyRange g_keyrange;

void tmark(int k, hipStream_t s) {
  if (!g_timing.enabled) return;
  if (!g_timing.created) {
    for (auto& e : g_timing.ev) (void)hipEventCreate(&e);
    g_timing.created = true;
  }
  (void)hipEventRecord(g_timing.ev[k], s);
  if (k == 6) g_timing.valid = true;
}

Cam make_cam(const gsr_settings* s, int M) {
  Cam c;
  c.W = s->image_width;
  c.H = s->image_height;
  c.tanfx = s->tanfovx;
  c.tanfy = s->tanfovy;
  c.fx = c.W / (2.0f * s->tanfovx);
  c.fy = c.H / (2.0f * s->tanfovy);
  c.scale_mod = s->scale_modifier;
  c.D = s->sh_degree;
  c.M = M;
  c.gx = (c.W + BX - 1) / BX;
  c.gy = (c.H + BY - 1) / BY;
  c.prefiltered = s->prefiltered != 0;
  return c;
}

}  // namespace

extern "C" {

size_t gsr_geom_bytes(int64_t P) { return geom_bytes(P > 0 ? P : 1); }
size_t gsr_image_bytes(int height, int width) { return image_bytes(height, width); }
size_t gsr_binning_bytes(int64_t R) { return binning_bytes(R > 0 ? R : 1); }

void gsr_set_timing(int enabled) { g_timing.enabled = enabled != 0; }

void gsr_set_binning(int mode) { g_binning = mode == 1 ? 1 : 0; }

int gsr_last_timing(float* phases_ms, int n) {
  if (!g_timing.valid) return S3_ERR_INVALID;
  S3_HIP(hipEventSynchronize(g_timing.ev[6]));
  // (preprocess, reduce (fused into preprocess: ~0), depth sort, tile
  // binning, blend); event 2 -> 3 spans the host read-back of num_rendered
  // and is not a device phase.
  const int from[5] = {0, 1, 3, 4, 5};
  for (int k = 0; k < n && k < 5; ++k) {
    float ms = 0.f;
    S3_HIP(hipEventElapsedTime(&ms, g_timing.ev[from[k]], g_timing.ev[from[k] + 1]));
    phases_ms[k] = ms;
  }
  return S3_OK;
}

int gsr_preprocess(const gsr_settings* s, int64_t P, int M, const float* means3D,
                   const float* scales, const float* rotations, const float* cov3D_precomp,
                   const float* shs, const float* colors_precomp, const float* opacities,
                   int32_t* radii, void* geom, int64_t* num_rendered, void* stream) {
  S3_REQUIRE(s && num_rendered && P >= 0, "gsr_preprocess: bad arguments");
  S3_REQUIRE(P < (int64_t)1 << 31, "gsr_preprocess: P too large");
  S3_REQUIRE((shs == nullptr) != (colors_precomp == nullptr),
             "Please provide excatly one of either SHs or precomputed colors!");
  S3_REQUIRE((cov3D_precomp == nullptr) != (scales == nullptr || rotations == nullptr),
             "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  S3_REQUIRE(s->sh_degree >= 0 && s->sh_degree <= 3, "gsr_preprocess: sh_degree must be 0..3");
  S3_REQUIRE(shs == nullptr || M >= (s->sh_degree + 1) * (s->sh_degree + 1),
             "gsr_preprocess: M=%d too small for sh_degree %d", M, s->sh_degree);
  *num_rendered = 0;
  if (P == 0) return S3_OK;
  hipStream_t st = s3::as_stream(stream);
  Cam cam = make_cam(s, M);
  GeomState g = carve_geom(geom, P);
  tmark(0, st);
  S3_HIP(hipMemsetAsync(g.red, 0, sizeof(Reduce), st));
  k_preprocess<<<(unsigned)s3::cdiv(P, kThreads), kThreads, 0, st>>>(
      P, cam, means3D, scales, rotations, cov3D_precomp, shs, colors_precomp, opacities,
      s->viewmatrix, s->projmatrix, s->campos, radii, g);
  S3_LAUNCH_CHECK();
  tmark(1, st);
  tmark(2, st);
  // read-back into a pinned slot (a pageable destination takes a staged
  // copy) behind a polled event (a blocking wait adds its wake-up latency to
  // every forward of the two-call API).  The slot and its event belong to
  // the device of `st` (the caller's current device may be another one): one
  // per (thread, device), the event created under that device.
  constexpr int kMaxDev = 64;
  static thread_local Reduce* red_hosts[kMaxDev] = {};
  static thread_local hipEvent_t red_evs[kMaxDev] = {};
  int sdev = -1;
  S3_HIP(s3::stream_device(st, &sdev));
  S3_REQUIRE(sdev >= 0 && sdev < kMaxDev, "gsr_preprocess: device %d out of range", sdev);
  if (!red_hosts[sdev]) {
    s3::DeviceGuard guard(sdev);
    Reduce* h = nullptr;
    hipEvent_t ev = nullptr;
    S3_HIP(hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(Reduce), hipHostMallocDefault));
    const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) (void)hipHostFree(h);
    S3_HIP(e);
    red_hosts[sdev] = h;
    red_evs[sdev] = ev;
  }
  Reduce* red_host = red_hosts[sdev];
  hipEvent_t red_ev = red_evs[sdev];
  S3_HIP(hipMemcpyAsync(red_host, g.red, sizeof(Reduce), hipMemcpyDeviceToHost, st));
  S3_HIP(hipEventRecord(red_ev, st));
  S3_HIP(s3::wait_event_spin(red_ev));
  const Reduce& red = *red_host;
  unsigned long long total = 0;
  uint32_t kmax = 0, kmin_inv = 0;
  for (int k = 0; k < kRedSlots; ++k) {
    total += red.slot[k].total;
    kmax = std::max(kmax, red.slot[k].kmax);
    kmin_inv = std::max(kmin_inv, red.slot[k].kmin_inv);
  }
  // the binning pass indexes instances with 32-bit offsets
  S3_REQUIRE(total < ((unsigned long long)1 << 32),
             "gsr_preprocess: %llu tile instances exceed 2^32", total);
  *num_rendered = (int64_t)total;
  g_keyrange = {geom, P, ~kmin_inv, kmax};
  return S3_OK;
}

}  // extern "C"

namespace {
// Binning + blend of gsr_render.  R: instances (host count; the binning
// capacity in the sync-free forward).  kmin / span / bits: the depth sort's
// key range and pass width.  dyn (sync-free): device {kmin, span, instances}
// that override kmin / span and bound the instance passes.
int render_impl(const gsr_settings* s, int64_t P, int64_t R, void* geom, void* binning,
                void* image, float* out_color, hipStream_t st, uint32_t kmin, uint32_t span,
                int bits, const uint32_t* dyn) {
  const int W = s->image_width, H = s->image_height;
  const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY, ntiles = gx * gy;
  if (P == 0) {
    S3_HIP(hipMemsetAsync(out_color, 0, sizeof(float) * 3 * (size_t)H * W, st));
    return S3_OK;
  }
  GeomState g = carve_geom(geom, P);
  BinningState b = carve_binning(binning, R);
  ImageState im = carve_image(image, H, W);
  tmark(3, st);
  const uint32_t* point_list = b.vals[0];
  const uint32_t* dn = dyn ? dyn + 2 : nullptr;
  const uint32_t cap = dyn ? (uint32_t)R : 0xFFFFFFFFu;
  if (R > 0 && g_binning == 1 && ntiles <= kTileLdsMax) {
    // per-tile binning + LDS depth sort (see "per-tile binning")
    const int o = tile_sort_buffer(ntiles), f = o ^ 1;
    S3_HIP(hipMemsetAsync(im.cursor, 0, sizeof(uint32_t) * ntiles, st));
    // ~512 workgroups (few global atomics per tile), each a whole number of
    // kBinThreads x kBinPer batches
    const int64_t batch = kBinThreads * kBinPer;
    const int64_t per_wg = batch * std::max<int64_t>(1, s3::cdiv(s3::cdiv(P, 512), batch));
    const unsigned bb = (unsigned)s3::cdiv(P, per_wg);
    k_tile_count<<<bb, kBinThreads, sizeof(uint32_t) * ntiles, st>>>(P, per_wg, gx, ntiles,
                                                                      g.dup, im.cursor);
    k_tile_scan<<<1, 1024, 0, st>>>(ntiles, im.cursor, im.ranges, cap);
    tmark(4, st);
    k_tile_fill<<<bb, kBinThreads, 2 * sizeof(uint32_t) * ntiles, st>>>(
        P, per_wg, gx, ntiles, g.dup, g.dkey[0], im.cursor, b.keys[f], b.vals[f], cap);
    const Digit dg{kmin, span, 0, 1, dyn};
    k_tile_sort<<<ntiles, kTSThreads, 0, st>>>(ntiles, im.ranges, b.keys[f], b.vals[f], b.keys[o],
                                               b.vals[o], dg, bits,
                                               std::max(1, bit_length((uint64_t)(P - 1))));
    S3_LAUNCH_CHECK();
    point_list = b.vals[o];
  } else if (R > 0) {
    S3_HIP(hipMemsetAsync(im.ranges, 0, sizeof(uint2) * ntiles, st));
    const int dsrc = radix_sort<uint32_t, uint32_t>(P, g.dkey, g.dval, kmin, span, bits, false,
                                                    g.dhist, g.dtot, st, true, dyn);
    const uint32_t* order = g.dval[dsrc];
    tmark(4, st);
    const int64_t nwseg = s3::cdiv(P, kDupRanks);
    const unsigned dup_blocks = (unsigned)s3::cdiv(nwseg, kThreads / 64);
    k_order_gather<<<dup_blocks, kThreads, 0, st>>>(P, order, g.dup, nwseg, g.dup_sorted,
                                                    g.cnt_seg);
    k_seg_scan<<<1, 1024, 0, st>>>(g.cnt_seg, nwseg);
    // tile ids as 16-bit keys up to 65536 tiles: the two tile passes and the
    // ranges pass move 6 B per instance instead of 8
    const int tbits = bit_length((uint64_t)(ntiles - 1));
    int tsrc;
    if (ntiles <= 65536) {
      uint16_t* k16[2] = {reinterpret_cast<uint16_t*>(b.keys[0]),
                          reinterpret_cast<uint16_t*>(b.keys[1])};
      k_duplicate<uint16_t><<<dup_blocks, kThreads, 0, st>>>(P, gx, order, g.dup_sorted,
                                                             g.cnt_seg, nwseg, k16[0], b.vals[0],
                                                             cap);
      tsrc = radix_sort<uint16_t, uint32_t>(R, k16, b.vals, 0u, 0xFFFFFFFFu, tbits, true, b.hist,
                                            b.tot, st, false, nullptr, dn);
      k_ranges16<<<(unsigned)s3::cdiv(s3::cdiv(R, 8), kThreads), kThreads, 0, st>>>(
          R, k16[tsrc], im.ranges, dn);
    } else {
      k_duplicate<uint32_t><<<dup_blocks, kThreads, 0, st>>>(P, gx, order, g.dup_sorted,
                                                             g.cnt_seg, nwseg, b.keys[0], b.vals[0],
                                                             cap);
      tsrc = radix_sort<uint32_t, uint32_t>(R, b.keys, b.vals, 0u, 0xFFFFFFFFu, tbits, true,
                                            b.hist, b.tot, st, false, nullptr, dn);
      k_ranges<uint32_t><<<(unsigned)s3::cdiv(R, kThreads), kThreads, 0, st>>>(R, b.keys[tsrc],
                                                                             im.ranges, dn);
    }
    S3_REQUIRE(tsrc == tile_sort_buffer(ntiles), "gsr_render: tile sort buffer mismatch");
    point_list = b.vals[tsrc];
    S3_LAUNCH_CHECK();
  } else {
    S3_HIP(hipMemsetAsync(im.ranges, 0, sizeof(uint2) * ntiles, st));
    tmark(4, st);
  }
  tmark(5, st);
  k_blend<<<ntiles, BS, 0, st>>>(W, H, gx, ntiles, im.ranges, point_list, g, s->bg, im.final_T,
                                 im.n_contrib, out_color);
  S3_LAUNCH_CHECK();
  tmark(6, st);
  return S3_OK;
}
}  // namespace

extern "C" {

int gsr_render(const gsr_settings* s, int64_t P, int64_t R, const int32_t* radii,
               void* geom, void* binning, void* image, float* out_color, void* stream) {
  S3_REQUIRE(s && P >= 0 && R >= 0, "gsr_render: bad arguments");
  S3_REQUIRE(R < ((int64_t)1 << 32), "gsr_render: too many tile instances");
  (void)radii;
  // the depth-key range of this geometry buffer, from gsr_preprocess's
  // read-back (full 32-bit width if the buffer was filled elsewhere)
  uint32_t kmin = 0, kmax = 0xFFFFFFFEu;
  if (g_keyrange.geom == geom && g_keyrange.P == P) {
    kmin = g_keyrange.kmin;
    kmax = g_keyrange.kmax;
  }
  // visible keys map to [0, kmax - kmin], culled ones (~0u) to span
  const uint32_t span = kmax - kmin + 1u;
  return render_impl(s, P, R, geom, binning, image, out_color, s3::as_stream(stream), kmin, span,
                     bit_length(span), nullptr);
}

int gsr_forward_deferred(const gsr_settings* s, int64_t P, int M, const float* means3D,
                         const float* scales, const float* rotations, const float* cov3D_precomp,
                         const float* shs, const float* colors_precomp, const float* opacities,
                         int32_t* radii, void* geom, void* binning, int64_t capacity,
                         int key_bits, void* image, float* out_color, int64_t* info,
                         void* stream) {
  S3_REQUIRE(s && info && P >= 0, "gsr_forward_deferred: bad arguments");
  S3_REQUIRE(P < (int64_t)1 << 31, "gsr_forward_deferred: P too large");
  S3_REQUIRE(capacity >= 1 && capacity < ((int64_t)1 << 32) && key_bits >= 1 && key_bits <= 32,
             "gsr_forward_deferred: capacity 1..2^32-1, key_bits 1..32");
  S3_REQUIRE((shs == nullptr) != (colors_precomp == nullptr),
             "Please provide excatly one of either SHs or precomputed colors!");
  S3_REQUIRE((cov3D_precomp == nullptr) != (scales == nullptr || rotations == nullptr),
             "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  S3_REQUIRE(s->sh_degree >= 0 && s->sh_degree <= 3, "gsr_forward_deferred: sh_degree 0..3");
  S3_REQUIRE(shs == nullptr || M >= (s->sh_degree + 1) * (s->sh_degree + 1),
             "gsr_forward_deferred: M=%d too small for sh_degree %d", M, s->sh_degree);
  hipStream_t st = s3::as_stream(stream);
  if (P == 0) {
    S3_HIP(hipMemsetAsync(info, 0, 3 * sizeof(int64_t), st));
    return render_impl(s, 0, 0, geom, binning, image, out_color, st, 0, 1, 1, nullptr);
  }
  Cam cam = make_cam(s, M);
  GeomState g = carve_geom(geom, P);
  tmark(0, st);
  S3_HIP(hipMemsetAsync(g.red, 0, sizeof(Reduce), st));
  k_preprocess<<<(unsigned)s3::cdiv(P, kThreads), kThreads, 0, st>>>(
      P, cam, means3D, scales, rotations, cov3D_precomp, shs, colors_precomp, opacities,
      s->viewmatrix, s->projmatrix, s->campos, radii, g);
  S3_LAUNCH_CHECK();
  k_red_finalize<<<1, 64, 0, st>>>(g.red, (uint32_t)capacity, key_bits, g.dyn, info);
  S3_LAUNCH_CHECK();
  tmark(1, st);
  tmark(2, st);
  const uint32_t span_bound = key_bits >= 32 ? 0xFFFFFFFFu : ((1u << key_bits) - 1u);
  return render_impl(s, P, capacity, geom, binning, image, out_color, st, 0u, span_bound,
                     key_bits, g.dyn);
}

int gsr_backward(const gsr_settings* s, int64_t P, int M, int64_t R, const float* means3D,
                 const float* scales, const float* rotations, const float* cov3D_precomp,
                 const float* shs, const float* colors_precomp, const float* opacities,
                 const int32_t* radii, const void* geom, const void* binning,
                 const void* image, const float* dL_dout, float* dL_dmeans2D,
                 float* dL_dconic, float* dL_dopacity, float* dL_dcolors, float* dL_dmeans3D,
                 float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                 void* stream) {
  S3_REQUIRE(s && P >= 0 && R >= 0, "gsr_backward: bad arguments");
  (void)colors_precomp;
  (void)opacities;
  hipStream_t st = s3::as_stream(stream);
  // the accumulated gradient outputs start at zero: one launch for all
  ZeroList zl{};
  auto add = [&](float* p, int64_t n) {
    if (p && n > 0) { zl.p[zl.cnt] = p; zl.n[zl.cnt] = n; ++zl.cnt; }
  };
  // (only the blend's atomic accumulators: k_preprocess_backward writes
  // every element of the per-Gaussian outputs, zeros for culled ones)
  add(dL_dmeans2D, P * 3);
  add(dL_dconic, P * 4);
  add(dL_dopacity, P);
  add(dL_dcolors, P * 3);
  if (zl.cnt > 0) {
    int64_t nmax = 0;
    for (int k = 0; k < zl.cnt; ++k) nmax = zl.n[k] > nmax ? zl.n[k] : nmax;
    k_zero_multi<<<dim3((unsigned)s3::cdiv(nmax, kThreads * 4), zl.cnt), kThreads, 0, st>>>(zl);
    S3_LAUNCH_CHECK();
  }
  if (P == 0) return S3_OK;
  const int W = s->image_width, H = s->image_height;
  const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY, ntiles = gx * gy;
  GeomState g = carve_geom(const_cast<void*>(geom), P);
  BinningState b = carve_binning(const_cast<void*>(binning), R);
  ImageState im = carve_image(const_cast<void*>(image), H, W);
  k_blend_backward<<<ntiles, BS, 0, st>>>(W, H, gx, ntiles, im.ranges,
                                          b.vals[R > 0 ? tile_sort_buffer(ntiles) : 0], g, s->bg,
                                          im.final_T, im.n_contrib, dL_dout, dL_dmeans2D,
                                          dL_dconic, dL_dopacity, dL_dcolors);
  S3_LAUNCH_CHECK();
  Cam cam = make_cam(s, M);
  k_preprocess_backward<<<(unsigned)s3::cdiv(P, kThreads), kThreads, 0, st>>>(
      P, cam, means3D, scales, rotations, cov3D_precomp, shs, radii, g, s->viewmatrix,
      s->projmatrix, s->campos, dL_dmeans2D, dL_dconic, dL_dcolors, dL_dmeans3D, dL_dcov3D,
      dL_dsh, dL_dscales, dL_drotations);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int gsr_mark_visible(int64_t P, const float* means3D, const float* viewmatrix,
                     const float* projmatrix, uint8_t* present, void* stream) {
  (void)projmatrix;
  S3_REQUIRE(P >= 0, "gsr_mark_visible: P < 0");
  if (P == 0) return S3_OK;
  k_mark_visible<<<(unsigned)s3::cdiv(P, kThreads), kThreads, 0, s3::as_stream(stream)>>>(
      P, means3D, viewmatrix, present);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

}  // extern "C"
