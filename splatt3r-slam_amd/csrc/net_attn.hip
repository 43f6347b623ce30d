// Fused RoPE2D + multi-head attention, head_dim 64 (include/s3n.h).
//
// One 256-lane workgroup = 64 query rows of one (group, batch, head); each
// wave owns 16 rows.  S = Q K^T and O += P V run on v_mfma_f32_16x16x32_f16
// with fp32 accumulation; softmax is online (running max / sum per row,
// base-2 exponent).  K and V tiles of 64 keys are staged global -> registers
// -> LDS (double buffered): K with RoPE applied while staging (each lane
// rotates a (d, d+16) chunk pair), V row-major and consumed through the
// gfx950 transpose read ds_read_b64_tr_b16 so it needs no transpose pass.
// P goes through a 2 KiB per-wave LDS scratch to change from the MFMA C
// layout (key on the lane) to the A layout (query on the lane).
// RoPE (croco/models/pos_embed.py:106-159): head dims [0,32) rotate with
// the y position, [32,64) with x; within each half, dim d pairs with d+16:
// out[d] = x[d] cos - x[d+16] sin, out[d+16] = x[d+16] cos + x[d] sin.
#include "common.hpp"
#include "s3n.h"

namespace {

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int QT = 64;   // query rows per workgroup
constexpr int KT = 64;   // keys per tile
constexpr int D = 64;
constexpr int kThreads = 256;

struct AttnP {
  int B, Nq, Nk, H, groups;
  const f16* Q[S3N_MAX_GROUPS];
  const f16* K[S3N_MAX_GROUPS];
  const f16* V[S3N_MAX_GROUPS];
  int64_t qs, ks, vs;
  const int64_t* qpos[S3N_MAX_GROUPS];
  const int64_t* kpos[S3N_MAX_GROUPS];
  const float* cosT;
  const float* sinT;
  int maxpos;
  f16* O[S3N_MAX_GROUPS];
  int64_t os;
  float scale_log2;
  int nqt;      // query tiles per (group, batch, head) (k_attn_st 1-D grid)
  int xcd;      // k_attn_st: 1 = XCD-aware workgroup order
};

// Bijective XCD-aware order for a 1-D grid of n workgroups: consecutive ids
// round-robin over the 8 XCDs (private L2 each), so id b is given logical
// tile (b % 8)'s contiguous run + b / 8 (cdna_hip_programming.md §5 'XCD
// swizzle must be bijective').  The query tiles of one (group, batch, head)
// then share an XCD and read its K / V from that L2 instead of each XCD
// fetching them.
__device__ __forceinline__ int xcd_order(int b, int n) {
  const int q = n / 8, r = n % 8;
  const int xcd = b % 8, k = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

__device__ __forceinline__ int kswz(int row, int c) { return c ^ ((row >> 1) & 7); }

// 2^x as the bare v_exp_f32.  The library exp2f wraps it in a denormal-range
// rescale (compare, select, add 64, exp, select, ldexp: six instructions
// instead of one) for x < -126; the softmax arguments here are <= 0 and a
// weight under 2^-126 is zero in the fp16 P operand and leaves the fp32 row
// sum (>= 1) unchanged, so every output is the same bit for bit while the
// per-key VALU work of the score tile drops by half.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Rotate chunk `c` (8 dims) of a head row given both it and its partner
// chunk c^2; returns the rotated chunk c.
__device__ __forceinline__ f16x8 rope_chunk(f16x8 x, f16x8 partner, int c, int64_t py, int64_t px,
                                            const float* cosT, const float* sinT) {
  const int half = c >> 2;             // 0: y dims, 1: x dims
  const int lo = ((c & 3) < 2);        // chunk holds dims [0,16) of its half
  const int64_t pos = half ? px : py;
  const int f0 = (c & 1) * 8;          // frequency index of the first dim
  f16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float cs = cosT[pos * 16 + f0 + j];
    const float sn = sinT[pos * 16 + f0 + j];
    const float a = (float)x[j], b = (float)partner[j];
    out[j] = lo ? (f16)(a * cs - b * sn) : (f16)(a * cs + b * sn);
  }
  return out;
}

__global__ void __launch_bounds__(kThreads) k_attn(AttnP p) {
  __shared__ __attribute__((aligned(16))) f16 Ks[2][KT * D];
  __shared__ __attribute__((aligned(16))) f16 Vs[2][KT * D];
  __shared__ __attribute__((aligned(16))) f16 Ps[4][16 * KT];

  const int qtile = blockIdx.x;
  const int bh = blockIdx.y;
  const int b = bh / p.H, h = bh % p.H;
  const int g = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const f16* __restrict__ Qg = p.Q[g];
  const f16* __restrict__ Kg = p.K[g];
  const f16* __restrict__ Vg = p.V[g];
  const int64_t* __restrict__ qpos = p.qpos[g];
  const int64_t* __restrict__ kpos = p.kpos[g];

  // ---- Q fragments (A operand of 16x16x32): row = lane&15, dims chunk
  // (4*ks + (lane>>4)) for ks = 0,1.
  const int qrow = qtile * QT + wave * 16 + (lane & 15);
  const bool qok = qrow < p.Nq;
  f16x8 qf[2];
  {
    const f16* qp = Qg + ((int64_t)b * p.Nq + (qok ? qrow : 0)) * p.qs + h * D;
    int64_t py = 0, px = 0;
    if (qpos) {
      py = qpos[((int64_t)b * p.Nq + (qok ? qrow : 0)) * 2 + 0];
      px = qpos[((int64_t)b * p.Nq + (qok ? qrow : 0)) * 2 + 1];
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 4 * ks + (lane >> 4);
      f16x8 x = *reinterpret_cast<const f16x8*>(qp + c * 8);
      if (qpos) {
        const f16x8 y = *reinterpret_cast<const f16x8*>(qp + (c ^ 2) * 8);
        x = rope_chunk(x, y, c, py, px, p.cosT, p.sinT);
      }
      if (!qok) x = f16x8{};
      qf[ks] = x;
    }
  }

  // ---- staging assignment: K: one (row, chunk pair) per lane; V: 2 chunks
  const int k_row = tid >> 2;              // 0..63
  const int k_pair = tid & 3;              // pairs (0,2) (1,3) (4,6) (5,7)
  const int k_c0 = (k_pair & 1) + (k_pair >> 1) * 4;
  const int k_c1 = k_c0 ^ 2;
  f16x8 rk0, rk1, rv0, rv1;
  const int v_row0 = tid >> 3, v_c0 = tid & 7;   // chunk tid and tid+256
  auto gload = [&](int t) {
    const int key = t * KT + k_row;
    const bool ok = key < p.Nk;
    const f16* kp = Kg + ((int64_t)b * p.Nk + (ok ? key : 0)) * p.ks + h * D;
    f16x8 a = *reinterpret_cast<const f16x8*>(kp + k_c0 * 8);
    f16x8 c = *reinterpret_cast<const f16x8*>(kp + k_c1 * 8);
    if (kpos) {
      const int64_t py = kpos[((int64_t)b * p.Nk + (ok ? key : 0)) * 2 + 0];
      const int64_t px = kpos[((int64_t)b * p.Nk + (ok ? key : 0)) * 2 + 1];
      rk0 = rope_chunk(a, c, k_c0, py, px, p.cosT, p.sinT);
      rk1 = rope_chunk(c, a, k_c1, py, px, p.cosT, p.sinT);
    } else {
      rk0 = a;
      rk1 = c;
    }
    if (!ok) { rk0 = f16x8{}; rk1 = f16x8{}; }
    const int key0 = t * KT + v_row0, key1 = key0 + 32;
    rv0 = key0 < p.Nk ? *reinterpret_cast<const f16x8*>(Vg + ((int64_t)b * p.Nk + key0) * p.vs + h * D + v_c0 * 8) : f16x8{};
    rv1 = key1 < p.Nk ? *reinterpret_cast<const f16x8*>(Vg + ((int64_t)b * p.Nk + key1) * p.vs + h * D + v_c0 * 8) : f16x8{};
  };
  auto sstore = [&](int buf) {
    *reinterpret_cast<f16x8*>(&Ks[buf][k_row * D + kswz(k_row, k_c0) * 8]) = rk0;
    *reinterpret_cast<f16x8*>(&Ks[buf][k_row * D + kswz(k_row, k_c1) * 8]) = rk1;
    *reinterpret_cast<f16x8*>(&Vs[buf][v_row0 * D + v_c0 * 8]) = rv0;
    *reinterpret_cast<f16x8*>(&Vs[buf][(v_row0 + 32) * D + v_c0 * 8]) = rv1;
  };

  // running state for the 4 rows this lane touches: rows 4*(lane>>4) + r
  float m_run[4], l_run[4];
  f32x4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m_run[r] = -INFINITY; l_run[r] = 0.f; }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int NT = (p.Nk + KT - 1) / KT;
  gload(0);
  sstore(0);
  __syncthreads();
  f16* Pw = Ps[wave];
  for (int t = 0; t < NT; ++t) {
    const int cur = t & 1;
    if (t + 1 < NT) gload(t + 1);
    // S = Q K^T for 4 blocks of 16 keys
    f32x4 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = kb * 16 + (lane & 15);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = 4 * ks + (lane >> 4);
        const f16x8 kf = *reinterpret_cast<const f16x8*>(&Ks[cur][krow * D + kswz(krow, c) * 8]);
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[ks], kf, s[kb], 0, 0, 0);
      }
    }
    // mask keys beyond Nk (lane holds key kb*16 + (lane&15))
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const bool kok = t * KT + kb * 16 + (lane & 15) < p.Nk;
#pragma unroll
      for (int r = 0; r < 4; ++r) s[kb][r] = kok ? s[kb][r] * p.scale_log2 : -INFINITY;
    }
    // online softmax per row (16 lanes with equal lane>>4 share a row)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      const float m_new = fmaxf(m_run[r], mx);
      const float alpha = fexp2(m_run[r] - m_new);
      m_run[r] = m_new;
      l_run[r] *= alpha;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb][r] *= alpha;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float e = fexp2(s[kb][r] - m_new);
        s[kb][r] = e;
        l_run[r] += e;
      }
    }
    // P -> per-wave LDS scratch as [q row 16][key 64] (A-operand layout)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qr = 4 * (lane >> 4) + r;
        Pw[qr * KT + kb * 16 + (lane & 15)] = (f16)s[kb][r];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P writes landed
    __builtin_amdgcn_wave_barrier();
    // O += P V
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const f16x8 pa = *reinterpret_cast<const f16x8*>(&Pw[(lane & 15) * KT + ks * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        // B operand: V[key = 32ks + 8(lane>>4) + j][d = 16nb + (lane&15)]
        // via two transpose reads of 4 rows x 16 cols (lane 4q+p supplies
        // row q, cols 4p..4p+3 of its 16-lane group's block).
        const int grp = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
        const int key0 = ks * 32 + 8 * grp + q4;
        const int dcol = nb * 16 + 4 * p4;
        typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_i16x4*)(&Vs[cur][key0 * D + dcol]));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_i16x4*)(&Vs[cur][(key0 + 4) * D + dcol]));
        f16x8 vb;
        const f16x4 lo16 = __builtin_bit_cast(f16x4, lo);
        const f16x4 hi16 = __builtin_bit_cast(f16x4, hi);
        vb[0] = lo16[0]; vb[1] = lo16[1]; vb[2] = lo16[2]; vb[3] = lo16[3];
        vb[4] = hi16[0]; vb[5] = hi16[1]; vb[6] = hi16[2]; vb[7] = hi16[3];
        o[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa, vb, o[nb], 0, 0, 0);
      }
    }
    if (t + 1 < NT) sstore(cur ^ 1);
    __syncthreads();
  }
  // finalize: reduce row sums across the 16 lanes, normalise, store fp16
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float l = l_run[r];
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) l += __shfl_xor(l, o2, 64);
    l_run[r] = 1.0f / l;
  }
  f16* Og = p.O[g];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = qtile * QT + wave * 16 + 4 * (lane >> 4) + r;
    if (row >= p.Nq) continue;
    f16* op = Og + ((int64_t)b * p.Nq + row) * p.os + h * D;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) op[nb * 16 + (lane & 15)] = (f16)(o[nb][r] * l_run[r]);
  }
}

// ---------------------------------------------------------------------------
// No-RoPE variant (q/k already rotated by the projection GEMM's epilogue):
// K and V tiles are streamed global -> LDS by buffer_load ... lds into a
// kStages-deep ring (no register staging, no per-tile VALU), so up to
// kStages-1 tiles are in flight while one is consumed.  Same math and
// fragment layouts as k_attn.
constexpr int kStages = 4;
constexpr uint32_t kOOB = 0x80000000u;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int PERW, int MAXA>
__device__ __forceinline__ void wait_tiles(int after) {
  if constexpr (MAXA <= 0) {
    wait_vm<0>();
  } else {
    if (after >= MAXA) wait_vm<PERW * MAXA>();
    else wait_tiles<PERW, MAXA - 1>(after);
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const int64_t lim = bytes < 0x7fffffff ? bytes : 0x7fffffff;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)lim,
                                           0x00020000);
}

#define S3_BLDS(rsrc, lptr, voff, soff)                                               \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(                                          \
      (rsrc), (__attribute__((address_space(3))) void*)(lptr), 16, (int)(voff), (int)(soff), 0, 0)

__global__ void __launch_bounds__(kThreads) k_attn_dma(AttnP p) {
  // one array: stages of [K tile | V tile], then the per-wave P scratch
  __shared__ __attribute__((aligned(1024))) f16 smem[kStages * 2 * KT * D + 4 * 16 * KT];
  const int qtile = blockIdx.x;
  const int bh = blockIdx.y;
  const int b = bh / p.H, h = bh % p.H;
  const int g = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const f16* __restrict__ Qg = p.Q[g];
  f16* Pw = smem + kStages * 2 * KT * D + wave * 16 * KT;

  const int qrow = qtile * QT + wave * 16 + (lane & 15);
  const bool qok = qrow < p.Nq;
  f16x8 qf[2];
  {
    const f16* qp = Qg + ((int64_t)b * p.Nq + (qok ? qrow : 0)) * p.qs + h * D;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 4 * ks + (lane >> 4);
      f16x8 x = *reinterpret_cast<const f16x8*>(qp + c * 8);
      qf[ks] = qok ? x : f16x8{};
    }
  }

  // DMA assignment: per tile 8 K + 8 V wave-instructions (8 key rows of
  // 128 B each), 2 + 2 per wave.  Lane l -> key row (l >> 3) of its group,
  // LDS chunk (l & 7); K's global chunk is pre-swizzled (kswz involution).
  const __amdgpu_buffer_rsrc_t rk =
      make_rsrc(p.K[g], (((int64_t)b + 1) * p.Nk - 1) * p.ks * 2 + (h + 1) * D * 2);
  const __amdgpu_buffer_rsrc_t rv =
      make_rsrc(p.V[g], (((int64_t)b + 1) * p.Nk - 1) * p.vs * 2 + (h + 1) * D * 2);
  const int lr = lane >> 3, lc = lane & 7;
  uint32_t k_off[2], v_off[2];
  int k_key[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wave * 2 + j) * 8 + lr;   // key row within the tile
    k_key[j] = row;
    k_off[j] = (uint32_t)((((int64_t)b * p.Nk + row) * p.ks + h * D + kswz(row, lc) * 8) * 2);
    v_off[j] = (uint32_t)((((int64_t)b * p.Nk + row) * p.vs + h * D + lc * 8) * 2);
  }
  const int NT = (p.Nk + KT - 1) / KT;
  auto issue = [&](int t, int st) {
    f16* Ks = smem + st * 2 * KT * D;
    f16* Vs = Ks + KT * D;
    const int key0 = t * KT;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = key0 + k_key[j] < p.Nk;
      S3_BLDS(rk, Ks + (wave * 2 + j) * 512, ok ? k_off[j] : kOOB, (int64_t)key0 * p.ks * 2);
      S3_BLDS(rv, Vs + (wave * 2 + j) * 512, ok ? v_off[j] : kOOB, (int64_t)key0 * p.vs * 2);
    }
  };

  float m_run[4], l_run[4];
  f32x4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m_run[r] = -INFINITY; l_run[r] = 0.f; }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int AHEAD = kStages - 1;
#pragma unroll
  for (int i = 0; i < AHEAD; ++i)
    if (i < NT) issue(i, i);
  for (int t = 0; t < NT; ++t) {
    wait_tiles<4, AHEAD - 1>(NT - 1 - t);
    s3::ring_barrier();
    if (t + AHEAD < NT) issue(t + AHEAD, (t + AHEAD) % kStages);
    const f16* Ks = smem + (t % kStages) * 2 * KT * D;
    const f16* Vs = Ks + KT * D;
    f32x4 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = kb * 16 + (lane & 15);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = 4 * ks + (lane >> 4);
        const f16x8 kf = *reinterpret_cast<const f16x8*>(&Ks[krow * D + kswz(krow, c) * 8]);
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[ks], kf, s[kb], 0, 0, 0);
      }
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const bool kok = t * KT + kb * 16 + (lane & 15) < p.Nk;
#pragma unroll
      for (int r = 0; r < 4; ++r) s[kb][r] = kok ? s[kb][r] * p.scale_log2 : -INFINITY;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      const float m_new = fmaxf(m_run[r], mx);
      const float alpha = fexp2(m_run[r] - m_new);
      m_run[r] = m_new;
      l_run[r] *= alpha;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb][r] *= alpha;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float e = fexp2(s[kb][r] - m_new);
        s[kb][r] = e;
        l_run[r] += e;
      }
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qr = 4 * (lane >> 4) + r;
        Pw[qr * KT + kb * 16 + (lane & 15)] = (f16)s[kb][r];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only: this wave's P writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const f16x8 pa = *reinterpret_cast<const f16x8*>(&Pw[(lane & 15) * KT + ks * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int grp = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
        const int key0 = ks * 32 + 8 * grp + q4;
        const int dcol = nb * 16 + 4 * p4;
        typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(&Vs[key0 * D + dcol]));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(&Vs[(key0 + 4) * D + dcol]));
        f16x8 vb;
        const f16x4 lo16 = __builtin_bit_cast(f16x4, lo);
        const f16x4 hi16 = __builtin_bit_cast(f16x4, hi);
        vb[0] = lo16[0]; vb[1] = lo16[1]; vb[2] = lo16[2]; vb[3] = lo16[3];
        vb[4] = hi16[0]; vb[5] = hi16[1]; vb[6] = hi16[2]; vb[7] = hi16[3];
        o[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa, vb, o[nb], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float l = l_run[r];
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) l += __shfl_xor(l, o2, 64);
    l_run[r] = 1.0f / l;
  }
  f16* Og = p.O[g];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = qtile * QT + wave * 16 + 4 * (lane >> 4) + r;
    if (row >= p.Nq) continue;
    f16* op = Og + ((int64_t)b * p.Nq + row) * p.os + h * D;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) op[nb * 16 + (lane & 15)] = (f16)(o[nb][r] * l_run[r]);
  }
}

// ---------------------------------------------------------------------------
// Transposed-score variant of k_attn_dma: S^T = K Q^T (the same two MFMA
// operands in swapped order), so every lane owns ONE query (lane & 15) and
// 4 keys per 16-key block.  Consequences:
//  * the softmax max / sum over keys is in-lane (16 values per tile) plus a
//    2-step exchange over the four 16-lane rows, instead of 4 rows x 4
//    cross-lane steps;
//  * P^T is already in the B-operand layout of O^T = V^T P^T: the 8 keys a
//    lane feeds to one 16x16x32 MFMA are its own 4 + 4 scores of two
//    adjacent key blocks (MFMA k-order is free as long as V^T uses the same
//    permutation), so P never goes through LDS;
//  * V^T comes from the same ds_read_b64_tr_b16 transpose reads with the key
//    bases of that permutation, and the rescale by alpha is one factor per
//    lane.
__device__ __forceinline__ float xchg16(float x) { return __shfl_xor(x, 16, 64); }
__device__ __forceinline__ float xchg32(float x) { return __shfl_xor(x, 32, 64); }

// SPLIT key-range groups of 4 waves per workgroup (SPLIT x 256 threads):
// group s streams every SPLIT-th key tile through its own LDS-DMA ring, and
// the groups' (max, sum, O) partials are merged through LDS at the end.
// More waves per SIMD for the same 64-query tile, half the serial tile
// chain per wave.
template <int QW, int SPLIT, int STAGES>
__global__ void __launch_bounds__(64 * QW * SPLIT) k_attn_st(AttnP p) {
  constexpr int RING = STAGES * 2 * KT * D;        // fp16 elements per group
  constexpr int NJ = 8 / QW;                       // K (and V) DMA pieces per wave per tile
  static_assert(QW == 1 || QW == 2 || QW == 4 || QW == 8, "query waves");
  __shared__ __attribute__((aligned(1024))) f16 smem[SPLIT * RING];
  // 1-D grid: logical id = qtile + nqt * (bh + B H g)
  const int lin = p.xcd ? xcd_order(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int qtile = lin % p.nqt;
  const int bh = (lin / p.nqt) % (p.B * p.H);
  const int b = bh / p.H, h = bh % p.H;
  const int g = lin / (p.nqt * p.B * p.H);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sp = wid / QW, wave = wid % QW;         // key group, query wave
  const int grp = lane >> 4, li = lane & 15;
  const f16* __restrict__ Qg = p.Q[g];
  f16* ring = smem + sp * RING;

  const int qrow = qtile * 16 * QW + wave * 16 + li;
  const bool qok = qrow < p.Nq;
  f16x8 qf[2];
  {
    const f16* qp = Qg + ((int64_t)b * p.Nq + (qok ? qrow : 0)) * p.qs + h * D;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 x = *reinterpret_cast<const f16x8*>(qp + (4 * ks + grp) * 8);
      qf[ks] = qok ? x : f16x8{};
    }
  }

  const __amdgpu_buffer_rsrc_t rk =
      make_rsrc(p.K[g], (((int64_t)b + 1) * p.Nk - 1) * p.ks * 2 + (h + 1) * D * 2);
  const __amdgpu_buffer_rsrc_t rv =
      make_rsrc(p.V[g], (((int64_t)b + 1) * p.Nk - 1) * p.vs * 2 + (h + 1) * D * 2);
  const int lr = lane >> 3, lc = lane & 7;
  uint32_t k_off[NJ], v_off[NJ];
  int k_key[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int row = (wave * NJ + j) * 8 + lr;
    k_key[j] = row;
    k_off[j] = (uint32_t)((((int64_t)b * p.Nk + row) * p.ks + h * D + kswz(row, lc) * 8) * 2);
    v_off[j] = (uint32_t)((((int64_t)b * p.Nk + row) * p.vs + h * D + lc * 8) * 2);
  }
  const int NT = (p.Nk + KT - 1) / KT;
  const int NTs = (NT - sp + SPLIT - 1) / SPLIT;     // this group's tiles: sp, sp+SPLIT, ...
  const int NTmax = (NT + SPLIT - 1) / SPLIT;        // every group runs as many barriers
  auto issue = [&](int i, int st) {
    f16* Ks = ring + st * 2 * KT * D;
    f16* Vs = Ks + KT * D;
    const int key0 = (i * SPLIT + sp) * KT;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bool ok = key0 + k_key[j] < p.Nk;
      S3_BLDS(rk, Ks + (wave * NJ + j) * 512, ok ? k_off[j] : kOOB, (int64_t)key0 * p.ks * 2);
      S3_BLDS(rv, Vs + (wave * NJ + j) * 512, ok ? v_off[j] : kOOB, (int64_t)key0 * p.vs * 2);
    }
  };

  float m_run = -INFINITY, l_run = 0.f;   // per lane: its query, its keys
  f32x4 o[4];                              // O^T blocks: d = 16 nb + 4 grp + r, query li
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int AHEAD = STAGES - 1;
#pragma unroll
  for (int i = 0; i < AHEAD; ++i)
    if (i < NTs) issue(i, i);
  for (int i = 0; i < NTmax; ++i) {
    if (i < NTs) wait_tiles<2 * NJ, AHEAD - 1>(NTs - 1 - i);
    s3::ring_barrier();
    if (i >= NTs) continue;
    if (i + AHEAD < NTs) issue(i + AHEAD, (i + AHEAD) % STAGES);
    const int t = i * SPLIT + sp;
    const f16* Ks = ring + (i % STAGES) * 2 * KT * D;
    const f16* Vs = Ks + KT * D;
    f32x4 s[4];   // S^T blocks: key 16 kb + 4 grp + r, query li
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = kb * 16 + li;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = 4 * ks + grp;
        const f16x8 kf = *reinterpret_cast<const f16x8*>(&Ks[krow * D + kswz(krow, c) * 8]);
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[ks], s[kb], 0, 0, 0);
      }
    }
    // raw scores: the max of s * scale is max(s) * scale (scale > 0, exact);
    // keys past Nk exist only in the last tile (wave-uniform test)
    float mx = -INFINITY;
    if ((t + 1) * KT <= p.Nk) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kb][r]);
    } else {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (t * KT + kb * 16 + 4 * grp + r >= p.Nk) s[kb][r] = -INFINITY;
          mx = fmaxf(mx, s[kb][r]);
        }
    }
    mx = fmaxf(mx, xchg16(mx));
    mx = fmaxf(mx, xchg32(mx));
    const float m_new = fmaxf(m_run, mx * p.scale_log2);
    const float alpha = fexp2(m_run - m_new);
    m_run = m_new;
    float ls = 0.f;
    {
      // s * scale - m as one fma (the row maximum's exponent is then within
      // half an ulp of 0 instead of exactly 0: exp2 ~ 1 - 4e-8); one VALU
      // op per key fewer than the rounded product and a difference
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = fexp2(fmaf(s[kb][r], p.scale_log2, -m_new));
          s[kb][r] = e;
          ls += e;
        }
    }
    l_run = l_run * alpha + ls;
    // the running max of most rows stops moving after the first tiles:
    // alpha == 1 for the whole wave skips the rescale (exact)
    if (__any(alpha != 1.0f)) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb] *= alpha;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pb[r] = (f16)s[2 * ks][r];
        pb[4 + r] = (f16)s[2 * ks + 1][r];
      }
      const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int dcol = nb * 16 + 4 * p4;
        const int klo = ks * 32 + 4 * grp + q4, khi = klo + 16;
        typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(&Vs[klo * D + dcol]));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(&Vs[khi * D + dcol]));
        const f16x4 lo16 = __builtin_bit_cast(f16x4, lo);
        const f16x4 hi16 = __builtin_bit_cast(f16x4, hi);
        f16x8 va;
        va[0] = lo16[0]; va[1] = lo16[1]; va[2] = lo16[2]; va[3] = lo16[3];
        va[4] = hi16[0]; va[5] = hi16[1]; va[6] = hi16[2]; va[7] = hi16[3];
        o[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb, o[nb], 0, 0, 0);
      }
    }
  }
  if constexpr (SPLIT > 1) {
    // merge the key groups: groups 1.. publish (m, l, O) per lane, group 0
    // rescales to the common max and sums
    constexpr int REC = 18;                        // m, l, 16 O values
    static_assert((SPLIT - 1) * QW * 64 * REC * 4 <= SPLIT * RING * 2, "merge scratch");
    float* xs = reinterpret_cast<float*>(smem);
    __syncthreads();                               // all rings drained
    if (sp > 0) {
      float* rec = xs + (((sp - 1) * QW + wave) * 64 + lane) * REC;
      rec[0] = m_run;
      rec[1] = l_run;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) rec[2 + nb * 4 + r] = o[nb][r];
    }
    __syncthreads();
    if (sp > 0) return;
#pragma unroll
    for (int s2 = 1; s2 < SPLIT; ++s2) {
      const float* rec = xs + (((s2 - 1) * QW + wave) * 64 + lane) * REC;
      const float m2 = rec[0];
      const float m = fmaxf(m_run, m2);
      const float a1 = fexp2(m_run - m), a2 = fexp2(m2 - m);
      l_run = l_run * a1 + rec[1] * a2;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[nb][r] = o[nb][r] * a1 + rec[2 + nb * 4 + r] * a2;
      m_run = m;
    }
  }
  float l = l_run;
  l += xchg16(l);
  l += xchg32(l);
  const float inv = 1.0f / l;
  if (!qok) return;
  f16* op = p.O[g] + ((int64_t)b * p.Nq + qrow) * p.os + h * D;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    f16x4 w;
#pragma unroll
    for (int r = 0; r < 4; ++r) w[r] = (f16)(o[nb][r] * inv);
    *reinterpret_cast<f16x4*>(op + nb * 16 + 4 * grp) = w;
  }
}

}  // namespace

static int g_attn_variant = 0;
static int g_attn_xcd = 1;
// tuning hook: v >= 0 picks the kernel variant; v == -1 / -2 switches the
// XCD-aware workgroup order of k_attn_st off / on
extern "C" void s3n_attention_set_variant(int v) {
  if (v == -1 || v == -2) g_attn_xcd = v == -2;
  else g_attn_variant = v;
}

extern "C" int s3n_attention(const s3n_attn_args* a, void* stream) {
  S3_REQUIRE(a && a->B > 0 && a->Nq >= 0 && a->Nk > 0 && a->H > 0, "s3n_attention: bad sizes");
  S3_REQUIRE(a->groups >= 1 && a->groups <= S3N_MAX_GROUPS, "s3n_attention: groups 1..4");
  S3_REQUIRE(a->q_stride % 8 == 0 && a->k_stride % 8 == 0 && a->v_stride % 8 == 0,
             "s3n_attention: row strides must be multiples of 8 elements");
  if (a->Nq == 0) return S3_OK;
  AttnP p;
  p.B = a->B; p.Nq = a->Nq; p.Nk = a->Nk; p.H = a->H; p.groups = a->groups;
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    const bool on = g < a->groups;
    p.Q[g] = on ? (const f16*)a->Q[g] : nullptr;
    p.K[g] = on ? (const f16*)a->K[g] : nullptr;
    p.V[g] = on ? (const f16*)a->V[g] : nullptr;
    p.qpos[g] = on ? a->qpos[g] : nullptr;
    p.kpos[g] = on ? a->kpos[g] : nullptr;
    p.O[g] = on ? (f16*)a->O[g] : nullptr;
    if (on) S3_REQUIRE(p.Q[g] && p.K[g] && p.V[g] && p.O[g], "s3n_attention: null operand");
    if (on && (p.qpos[g] || p.kpos[g]))
      S3_REQUIRE(a->rope_cos && a->rope_sin, "s3n_attention: RoPE tables missing");
  }
  p.qs = a->q_stride; p.ks = a->k_stride; p.vs = a->v_stride; p.os = a->o_stride;
  p.cosT = a->rope_cos; p.sinT = a->rope_sin; p.maxpos = a->rope_maxpos;
  p.scale_log2 = a->scale * 1.4426950408889634f;
  p.nqt = (a->Nq + QT - 1) / QT;
  p.xcd = g_attn_xcd;
  dim3 grid((a->Nq + QT - 1) / QT, a->B * a->H, a->groups);
  const unsigned lin = (unsigned)(p.nqt * a->B * a->H * a->groups);
  bool rope = false;
  for (int g = 0; g < a->groups; ++g) rope = rope || p.qpos[g] || p.kpos[g];
  if (rope)
    k_attn<<<grid, kThreads, 0, s3::as_stream(stream)>>>(p);
  else if (g_attn_variant == 1)
    k_attn_dma<<<grid, kThreads, 0, s3::as_stream(stream)>>>(p);
  else if (g_attn_variant == 2)
    k_attn_st<4, 1, kStages><<<lin, kThreads, 0, s3::as_stream(stream)>>>(p);
  else if (g_attn_variant == 3)
    k_attn_st<4, 4, 2><<<lin, kThreads * 4, 0, s3::as_stream(stream)>>>(p);
  else if (g_attn_variant == 4) {
    // 32-query workgroups (2 query waves): twice the workgroups per head
    // (in-graph 0.83 vs 0.75 ms/frame for the default: not used)
    p.nqt = (a->Nq + 31) / 32;
    k_attn_st<2, 2, 2><<<(unsigned)(p.nqt * a->B * a->H * a->groups), 64 * 2 * 2, 0,
                         s3::as_stream(stream)>>>(p);
  } else if (g_attn_variant == 5) {
    // 128-query workgroups (8 query waves x 2 key groups, 1024 threads):
    // half the workgroups, each K / V tile feeds twice the queries
    p.nqt = (a->Nq + 127) / 128;
    k_attn_st<8, 2, 2><<<(unsigned)(p.nqt * a->B * a->H * a->groups), 64 * 8 * 2, 0,
                         s3::as_stream(stream)>>>(p);
  } else
    k_attn_st<4, 2, 2><<<lin, kThreads * 2, 0, s3::as_stream(stream)>>>(p);
  S3_LAUNCH_CHECK();
  return S3_OK;
}
