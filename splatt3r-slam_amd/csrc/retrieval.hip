// Keyframe retrieval features + codebook quantisation (include/s3q.h),
// restating splatt3r_slam/retrieval_database.py:24-41 (prep_features) and
// :95-104 (quantize_custom) with mast3r/retrieval/model.py:55-103.
//
//  * k_affine<T>: the two fp64 Whiteners and the fp32 projector Linear as
//    one LDS-tiled GEMM template (64x64 tile, 4x4 outputs per thread),
//    centring / bias / residual fused.
//  * k_select: how_select_local with 'l2norm' attention — token norms into
//    LDS, an all-pairs rank (value desc, index asc) per token, then the
//    selected rows are gathered; one workgroup per image.
//  * k_l2_chunk: distances of a 64-query x 256-centroid tile (fp32 FMA,
//    K staged through LDS 32 at a time) followed by a per-row top-k of
//    the tile in registers (32-lane argmin rounds), candidates to the
//    workspace; k_l2_merge: one wave per query merges the chunk
//    candidates.  (dist, index) lexicographic order everywhere, so ties
//    keep the lower centroid index.
#include <cfloat>

#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "s3q.h"

namespace {

constexpr int kThreads = 256;

// ---------------------------------------------------------------- GEMM ----
// out[m, n] = sum_k (x[m, k] - mu[k]) * B(k, n) (+ bias[n]) (+ x[m, n]),
// accumulated in T.  B(k, n) = BT ? B[n * K + k] : B[k * N + n].
template <typename T, bool BT>
__global__ void __launch_bounds__(kThreads)
k_affine(const float* __restrict__ x, const double* __restrict__ mu, const T* __restrict__ B,
         const float* __restrict__ bias, float* __restrict__ out, int M, int K, int N,
         int residual) {
  constexpr int TM = 64, TN = 64, TK = 16;
  __shared__ T As[TK][TM + 1];
  __shared__ T Bs[TK][TN + 1];
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int tid = threadIdx.x, ty = tid / 16, tx = tid % 16;
  T acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = T(0);
  for (int k0 = 0; k0 < K; k0 += TK) {
    // A tile 64 x 16: 4 elements per thread
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int li = tid + e * kThreads;
      const int r = li / TK, c = li % TK;
      const int m = m0 + r, k = k0 + c;
      T v = T(0);
      if (m < M && k < K) {
        v = (T)x[(int64_t)m * K + k];
        if (mu) v = (T)((double)v - mu[k]);
      }
      As[c][r] = v;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int li = tid + e * kThreads;
      int r, c;
      if (BT) { r = li / TK; c = li % TK; }     // r = n, c = k (k contiguous)
      else    { c = li / TN; r = li % TN; }     // n contiguous
      const int n = n0 + r, k = k0 + c;
      T v = T(0);
      if (n < N && k < K) v = BT ? B[(int64_t)n * K + k] : B[(int64_t)k * N + n];
      Bs[c][r] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      T a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty + 16 * i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx + 16 * j;
      if (n >= N) continue;
      float v;
      if (bias) v = (float)acc[i][j] + bias[n];
      else v = (float)acc[i][j];
      if (residual) v += x[(int64_t)m * K + n];
      out[(int64_t)m * N + n] = v;
    }
  }
}

// ------------------------------------------------------ select local ----
constexpr int kMaxT = 4096;

__global__ void __launch_bounds__(kThreads)
k_select(const float* __restrict__ src, const float* __restrict__ feat, int T, int D, int nfeat,
         float* __restrict__ feat_out, float* __restrict__ attn_out,
         int64_t* __restrict__ idx_out) {
  __shared__ float a[kMaxT];
  __shared__ int sel[kMaxT];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* S = src + (int64_t)b * T * D;
  for (int t = wave; t < T; t += kThreads / 64) {
    float s = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float v = S[(int64_t)t * D + d];
      s += v * v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) a[t] = sqrtf(s);
  }
  __syncthreads();
  for (int t = tid; t < T; t += kThreads) {
    const float v = a[t];
    int r = 0;
    for (int j = 0; j < T; ++j) {
      const float w = a[j];
      r += (w > v) || (w == v && j < t);
    }
    if (r < nfeat) {
      sel[r] = t;
      attn_out[(int64_t)b * nfeat + r] = v;
      idx_out[(int64_t)b * nfeat + r] = t;
    }
  }
  __syncthreads();
  const float* F = feat + (int64_t)b * T * D;
  float* O = feat_out + (int64_t)b * nfeat * D;
  for (int r = wave; r < nfeat; r += kThreads / 64) {
    const int t = sel[r];
    for (int d = lane; d < D; d += 64) O[(int64_t)r * D + d] = F[(int64_t)t * D + d];
  }
}

__global__ void __launch_bounds__(kThreads)
k_row_sqnorm(const float* __restrict__ x, int R, int D, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float v = x[(int64_t)r * D + d];
    s += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[r] = s;
}

// ------------------------------------------------------- L2 top-k ----
constexpr int QM = 64, QC = 256, QK = 32, KMAX = 8;

__device__ __forceinline__ bool lt(float d0, int i0, float d1, int i1) {
  return d0 < d1 || (d0 == d1 && i0 < i1);
}

// Argmin over `width` lanes (xor butterfly within aligned groups).
template <int WIDTH>
__device__ __forceinline__ void argmin_lanes(float& d, int& i) {
#pragma unroll
  for (int o = 1; o < WIDTH; o <<= 1) {
    const float d2 = __shfl_xor(d, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (lt(d2, i2, d, i)) { d = d2; i = i2; }
  }
}

// grid (ceil(C / 256), ceil(M / 64)); cand [M, nchunks, k] (dist, idx)
__global__ void __launch_bounds__(kThreads)
k_l2_chunk(const float* __restrict__ q, const float* __restrict__ c, const float* __restrict__ cn,
           int M, int C, int D, int k, float* __restrict__ cand_d, int* __restrict__ cand_i) {
  __shared__ float Qs[QK][QM + 4];
  __shared__ float Cs[QK][QC + 4];
  __shared__ float qn_s[QM];
  const int chunk = blockIdx.x, nchunks = gridDim.x;
  const int m0 = blockIdx.y * QM, c0 = chunk * QC;
  const int tid = threadIdx.x, ty = tid / 32, tx = tid % 32;
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  for (int k0 = 0; k0 < D; k0 += QK) {
    // Q tile 64 x 32 (8 per thread)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int li = tid + e * kThreads;
      const int r = li / QK, cc = li % QK;
      const int m = m0 + r, kk = k0 + cc;
      Qs[cc][r] = (m < M && kk < D) ? q[(int64_t)m * D + kk] : 0.f;
    }
    // C tile 256 x 32 (32 per thread)
#pragma unroll 8
    for (int e = 0; e < 32; ++e) {
      const int li = tid + e * kThreads;
      const int r = li / QK, cc = li % QK;
      const int ci = c0 + r, kk = k0 + cc;
      Cs[cc][r] = (ci < C && kk < D) ? c[(int64_t)ci * D + kk] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < QK; ++kk) {
      float av[8], bv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) av[i] = Qs[kk][ty * 8 + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = Cs[kk][tx + 32 * j];
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  // |q|^2 per row (same arithmetic as s3q_row_sqnorm: lane-strided partial
  // sums + xor butterfly), one wave per row
  {
    const int lane = tid & 63, wave = tid >> 6;
    for (int r = wave; r < QM; r += kThreads / 64) {
      const int m = m0 + r;
      float s = 0.f;
      if (m < M)
        for (int d = lane; d < D; d += 64) {
          const float v = q[(int64_t)m * D + d];
          s += v * v;
        }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0) qn_s[r] = s;
    }
  }
  __syncthreads();
  float cnv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ci = c0 + tx + 32 * j;
    cnv[j] = ci < C ? cn[ci] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = ty * 8 + i, m = m0 + r;
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ci = c0 + tx + 32 * j;
      // quantize_custom: (|q|^2 + |c|^2) - 2 (q c^T)
      const float t = qn_s[r] + cnv[j];
      d[j] = ci < C ? t - 2.0f * acc[i][j] : FLT_MAX;
    }
    for (int s = 0; s < k; ++s) {
      float bd = FLT_MAX;
      int bi = INT32_MAX, bj = -1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = c0 + tx + 32 * j;
        if (lt(d[j], ci, bd, bi)) { bd = d[j]; bi = ci; bj = j; }
      }
      float wd = bd;
      int wi = bi;
      argmin_lanes<32>(wd, wi);
      if (bi == wi && bj >= 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j == bj) d[j] = FLT_MAX;
      }
      if (tx == 0 && m < M) {
        const int64_t o = ((int64_t)m * nchunks + chunk) * k + s;
        cand_d[o] = wd;
        cand_i[o] = wi;
      }
    }
  }
}

// one wave per query row: merge nchunks * k candidates -> k
__global__ void __launch_bounds__(kThreads)
k_l2_merge(const float* __restrict__ cand_d, const int* __restrict__ cand_i, int M, int nc,
           int k, int64_t* __restrict__ idx_out, float* __restrict__ dist_out) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const float* Dd = cand_d + (int64_t)m * nc;
  const int* Ii = cand_i + (int64_t)m * nc;
  float last_d = -FLT_MAX;
  int last_i = -1;
  for (int s = 0; s < k; ++s) {
    // smallest candidate strictly after (last_d, last_i) in (dist, idx) order
    float bd = FLT_MAX;
    int bi = INT32_MAX;
    for (int j = lane; j < nc; j += 64) {
      const float dj = Dd[j];
      const int ij = Ii[j];
      if (lt(last_d, last_i, dj, ij) && lt(dj, ij, bd, bi)) { bd = dj; bi = ij; }
    }
    argmin_lanes<64>(bd, bi);
    if (lane == 0) {
      idx_out[(int64_t)m * k + s] = bi;
      if (dist_out) dist_out[(int64_t)m * k + s] = bd;
    }
    last_d = bd;
    last_i = bi;
  }
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" int s3q_whiten(const float* x, const double* m, const double* P, float* out, int M,
                          int K, int N, void* stream) {
  S3_REQUIRE(x && P && out && M >= 0 && K > 0 && N > 0, "s3q_whiten: bad arguments");
  if (M == 0) return S3_OK;
  dim3 grid((unsigned)s3::cdiv(N, 64), (unsigned)s3::cdiv(M, 64));
  k_affine<double, false><<<grid, kThreads, 0, s3::as_stream(stream)>>>(x, m, P, nullptr, out, M,
                                                                        K, N, 0);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3q_linear(const float* x, const float* W, const float* b, float* out, int M,
                          int K, int N, int residual, void* stream) {
  S3_REQUIRE(x && W && out && M >= 0 && K > 0 && N > 0, "s3q_linear: bad arguments");
  S3_REQUIRE(!residual || N == K, "s3q_linear: residual needs N == K (%d vs %d)", N, K);
  if (M == 0) return S3_OK;
  dim3 grid((unsigned)s3::cdiv(N, 64), (unsigned)s3::cdiv(M, 64));
  k_affine<float, true><<<grid, kThreads, 0, s3::as_stream(stream)>>>(x, nullptr, W, b, out, M,
                                                                      K, N, residual);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3q_select_local(const float* attn_src, const float* feat, int B, int T, int D,
                                int nfeat, float* feat_out, float* attn_out, int64_t* idx_out,
                                void* stream) {
  S3_REQUIRE(attn_src && feat && feat_out && attn_out && idx_out, "s3q_select_local: null");
  S3_REQUIRE(B >= 0 && T > 0 && T <= kMaxT && D > 0 && nfeat > 0 && nfeat <= T,
             "s3q_select_local: bad sizes (B %d, T %d, D %d, nfeat %d; T <= %d)", B, T, D, nfeat,
             kMaxT);
  if (B == 0) return S3_OK;
  k_select<<<B, kThreads, 0, s3::as_stream(stream)>>>(attn_src, feat, T, D, nfeat, feat_out,
                                                      attn_out, idx_out);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3q_row_sqnorm(const float* x, int R, int D, float* out, void* stream) {
  S3_REQUIRE(x && out && R >= 0 && D > 0, "s3q_row_sqnorm: bad arguments");
  if (R == 0) return S3_OK;
  k_row_sqnorm<<<(unsigned)s3::cdiv(R, kThreads / 64), kThreads, 0, s3::as_stream(stream)>>>(
      x, R, D, out);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" size_t s3q_l2_topk_workspace_bytes(int M, int C, int k) {
  const size_t nc = (size_t)s3::cdiv(C > 0 ? C : 1, QC) * (k > 0 ? k : 1);
  return align256(sizeof(float) * (size_t)M * nc) + align256(sizeof(int) * (size_t)M * nc);
}

extern "C" int s3q_l2_topk(const float* q, const float* c, const float* c_sqnorm, int M, int C,
                           int D, int k, int64_t* idx_out, float* dist_out, void* workspace,
                           void* stream) {
  S3_REQUIRE(q && c && c_sqnorm && idx_out && workspace, "s3q_l2_topk: null argument");
  S3_REQUIRE(M >= 0 && C > 0 && D > 0 && k >= 1 && k <= KMAX && k <= C,
             "s3q_l2_topk: bad sizes (M %d, C %d, D %d, k %d; k <= %d)", M, C, D, k, KMAX);
  if (M == 0) return S3_OK;
  hipStream_t st = s3::as_stream(stream);
  const int nchunks = (int)s3::cdiv(C, QC);
  const size_t nc = (size_t)nchunks * k;
  float* cand_d = static_cast<float*>(workspace);
  int* cand_i = reinterpret_cast<int*>(static_cast<char*>(workspace) +
                                       align256(sizeof(float) * (size_t)M * nc));
  k_l2_chunk<<<dim3(nchunks, (unsigned)s3::cdiv(M, QM)), kThreads, 0, st>>>(q, c, c_sqnorm, M, C,
                                                                           D, k, cand_d, cand_i);
  S3_LAUNCH_CHECK();
  k_l2_merge<<<(unsigned)s3::cdiv(M, kThreads / 64), kThreads, 0, st>>>(cand_d, cand_i, M,
                                                                        (int)nc, k, idx_out,
                                                                        dist_out);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

// ------------------------------------------------------------------ ASMK --
// aggregate: one workgroup sorts the n*k (word, descriptor) pairs in LDS
// (bitonic; keys word << 16 | descriptor are unique) and writes the
// unique-word list + segment starts; then one workgroup per unique word sums
// the residuals over its descriptors (fp64) and packs the sign bits with
// wave ballots.  search: one lane per inverted-file entry, XOR + popcount
// against the query code of the same word (found through a word -> slot
// table), exact int64 score accumulation.
namespace {

constexpr int kAggMax = 4096;
constexpr int kAggThreads = 1024;
constexpr int kAggItems = kAggMax / kAggThreads;

struct AggWs {
  int32_t* seg_start;   // [m + 1]
  int32_t* seg_desc;    // [m] descriptor index per sorted pair
};

AggWs carve_agg(void* base, int m, size_t* total = nullptr) {
  char* p = static_cast<char*>(base);
  char* p0 = p;
  AggWs w;
  w.seg_start = (int32_t*)p; p += align256(sizeof(int32_t) * (m + 1));
  w.seg_desc = (int32_t*)p; p += align256(sizeof(int32_t) * m);
  if (total) *total = (size_t)(p - p0);
  return w;
}

__global__ void __launch_bounds__(kAggThreads)
k_asmk_sort(const int64_t* __restrict__ words, int m, int k, int32_t* __restrict__ out_words,
            int32_t* __restrict__ out_count, AggWs w) {
  typedef hipcub::BlockScan<int, kAggThreads> Scan;
  __shared__ uint64_t key[kAggMax];
  __shared__ typename Scan::TempStorage scan_tmp;
  int L = 1;
  while (L < m) L <<= 1;
  for (int i = threadIdx.x; i < L; i += kAggThreads)
    key[i] = i < m ? ((uint64_t)words[i] << 16) | (uint64_t)(i / k) : ~0ull;
  __syncthreads();
  for (int size = 2; size <= L; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < L; i += kAggThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const uint64_t a = key[i], b = key[j];
          if ((a > b) == up) { key[i] = b; key[j] = a; }
        }
      }
      __syncthreads();
    }
  }
  // segment heads -> unique index by a block exclusive scan (blocked items)
  int hd[kAggItems];
  const int base = threadIdx.x * kAggItems;
#pragma unroll
  for (int t = 0; t < kAggItems; ++t) {
    const int i = base + t;
    hd[t] = (i < m && (i == 0 || (key[i] >> 16) != (key[i - 1] >> 16))) ? 1 : 0;
  }
  int total = 0;
  Scan(scan_tmp).ExclusiveSum(hd, hd, total);
#pragma unroll
  for (int t = 0; t < kAggItems; ++t) {
    const int i = base + t;
    if (i >= m) break;
    w.seg_desc[i] = (int32_t)(key[i] & 0xFFFF);
    const bool head = i == 0 || (key[i] >> 16) != (key[i - 1] >> 16);
    if (head) {
      out_words[hd[t]] = (int32_t)(key[i] >> 16);
      w.seg_start[hd[t]] = i;
    }
  }
  if (threadIdx.x == 0) {
    w.seg_start[total] = m;
    *out_count = total;
  }
}

// one workgroup (256 lanes) per unique word; lanes stride the D dimensions
__global__ void __launch_bounds__(kThreads)
k_asmk_codes(const float* __restrict__ feats, const float* __restrict__ cen, int D,
             const int32_t* __restrict__ uwords, const int32_t* __restrict__ count, AggWs w,
             uint32_t* __restrict__ codes) {
  const int u = blockIdx.x;
  if (u >= *count) return;
  const int word = uwords[u];
  const int s0 = w.seg_start[u], s1 = w.seg_start[u + 1];
  const float* c = cen + (int64_t)word * D;
  const int lane = threadIdx.x & 63;
  for (int d0 = 0; d0 < D; d0 += kThreads) {
    const int d = d0 + threadIdx.x;
    double acc = 0.0;
    if (d < D) {
      const float cd = c[d];
      for (int s = s0; s < s1; ++s) acc += (double)(feats[(int64_t)w.seg_desc[s] * D + d] - cd);
    }
    const uint64_t bits = __ballot(d < D && acc > 0.0);
    if (lane == 0 && d < D) {
      uint32_t* o = codes + (int64_t)u * (D / 32) + d / 32;
      o[0] = (uint32_t)bits;
      if (d + 32 < D) o[1] = (uint32_t)(bits >> 32);
    }
  }
}

__global__ void __launch_bounds__(kThreads)
k_slot_set(const int32_t* __restrict__ qw, const int32_t* __restrict__ q_count, int q_max,
           int32_t* __restrict__ slot, int set) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= q_max || i >= *q_count) return;
  slot[qw[i]] = set ? i : -1;
}

__global__ void __launch_bounds__(kThreads)
k_asmk_search(const uint32_t* __restrict__ q_codes, const int32_t* __restrict__ db_words,
              const int32_t* __restrict__ db_images, const uint32_t* __restrict__ db_codes,
              int64_t n_db, int D, int alpha, int s_min, const int32_t* __restrict__ slot,
              unsigned long long* __restrict__ scores) {
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= n_db) return;
  const int q = slot[db_words[e]];
  if (q < 0) return;
  const int nw = D / 32;
  const uint32_t* a = db_codes + e * nw;
  const uint32_t* b = q_codes + (int64_t)q * nw;
  int ham = 0;
  for (int i = 0; i < nw; ++i) ham += __popc(a[i] ^ b[i]);
  const int s = D - 2 * ham;
  if (s < s_min) return;
  long long v = s;
  if (alpha >= 2) v *= s;
  if (alpha >= 3) v *= s;
  atomicAdd(&scores[db_images[e]], (unsigned long long)v);
}

}  // namespace

extern "C" size_t s3q_asmk_aggregate_workspace_bytes(int n, int k) {
  size_t t = 0;
  carve_agg(nullptr, n * k > 0 ? n * k : 1, &t);
  return t;
}

extern "C" int s3q_asmk_aggregate(const float* feats, const int64_t* words, const float* centroids,
                                  int n, int k, int D, int32_t* out_words, uint32_t* out_codes,
                                  int32_t* out_count, void* workspace, void* stream) {
  S3_REQUIRE(n >= 0 && k >= 1 && n * k <= kAggMax && n < 65536,
             "s3q_asmk_aggregate: n*k=%d exceeds %d", n * k, kAggMax);
  S3_REQUIRE(D > 0 && D % 32 == 0 && D <= 4096, "s3q_asmk_aggregate: D=%d (multiple of 32)", D);
  hipStream_t st = s3::as_stream(stream);
  if (n == 0) {
    S3_HIP(hipMemsetAsync(out_count, 0, sizeof(int32_t), st));
    return S3_OK;
  }
  S3_REQUIRE(feats && words && centroids && out_words && out_codes && out_count && workspace,
             "s3q_asmk_aggregate: null argument");
  const int m = n * k;
  AggWs w = carve_agg(workspace, m);
  k_asmk_sort<<<1, kAggThreads, 0, st>>>(words, m, k, out_words, out_count, w);
  S3_LAUNCH_CHECK();
  k_asmk_codes<<<m, kThreads, 0, st>>>(feats, centroids, D, out_words, out_count, w, out_codes);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3q_asmk_search(const int32_t* q_words, const uint32_t* q_codes,
                               const int32_t* q_count, int q_max, const int32_t* db_words,
                               const int32_t* db_images, const uint32_t* db_codes, int64_t n_db,
                               int D, int alpha, float sim_threshold, int32_t* word_slot,
                               int n_words, unsigned long long* scores, void* stream) {
  S3_REQUIRE(alpha >= 1 && alpha <= 3, "s3q_asmk_search: alpha=%d (1..3)", alpha);
  S3_REQUIRE(D > 0 && D % 32 == 0, "s3q_asmk_search: D=%d", D);
  S3_REQUIRE(q_max >= 0 && n_db >= 0 && n_words > 0, "s3q_asmk_search: bad sizes");
  if (q_max == 0 || n_db == 0) return S3_OK;
  S3_REQUIRE(q_words && q_codes && q_count && db_words && db_images && db_codes && word_slot &&
                 scores,
             "s3q_asmk_search: null argument");
  hipStream_t st = s3::as_stream(stream);
  // s / D >= threshold  <=>  s >= ceil(threshold * D)
  const int s_min = (int)ceil((double)sim_threshold * D);
  const int qb = (int)s3::cdiv(q_max, kThreads);
  k_slot_set<<<qb, kThreads, 0, st>>>(q_words, q_count, q_max, word_slot, 1);
  S3_LAUNCH_CHECK();
  k_asmk_search<<<(unsigned)s3::cdiv(n_db, kThreads), kThreads, 0, st>>>(
      q_codes, db_words, db_images, db_codes, n_db, D, alpha, s_min, word_slot, scores);
  S3_LAUNCH_CHECK();
  k_slot_set<<<qb, kThreads, 0, st>>>(q_words, q_count, q_max, word_slot, 0);
  S3_LAUNCH_CHECK();
  return S3_OK;
}
