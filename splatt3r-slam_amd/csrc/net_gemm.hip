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
#include "common.hpp"
#include "s3n.h"

namespace {

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 64;
constexpr int kThreads = 256;

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
};

__device__ __forceinline__ int swz(int row, int kc) { return (kc ^ ((row >> 1) & 7)); }

__device__ __forceinline__ float gelu(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, k = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <int BM, int BN, int AMODE>
__global__ void __launch_bounds__(kThreads) k_gemm(GemmP p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 32, FN = WN / 32;
  constexpr int AC = BM / 32, BC = BN / 32;  // 16-B chunks per thread per tile
  __shared__ __attribute__((aligned(16))) f16 smem[2 * (BM + BN) * BK];

  const int g = blockIdx.z;
  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n, tn = tile % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = p.M, N = p.N, K = p.K;
  const f16* __restrict__ A = p.A[g];
  const f16* __restrict__ B = p.B[g];

  // Per-thread staging rows are fixed across K tiles.
  int a_row[AC], a_kc[AC];
  const f16* a_base[AC];
  int a_iy0[AC], a_ix0[AC];
  bool a_ok[AC];
#pragma unroll
  for (int i = 0; i < AC; ++i) {
    const int c = tid + i * kThreads;
    a_row[i] = c >> 3;
    a_kc[i] = c & 7;
    const int m = m0 + a_row[i];
    a_ok[i] = m < M;
    if constexpr (AMODE == S3N_A_DENSE) {
      a_base[i] = A + (int64_t)(a_ok[i] ? m : 0) * p.lda;
      a_iy0[i] = a_ix0[i] = 0;
    } else {
      const int mm = a_ok[i] ? m : 0;
      const int ox = mm % p.oW, t = mm / p.oW, oy = t % p.oH, b = t / p.oH;
      a_base[i] = A + (int64_t)b * p.cH * p.cW * p.cC;
      a_iy0[i] = oy * p.st - p.pad;
      a_ix0[i] = ox * p.st - p.pad;
    }
  }
  int b_row[BC], b_kc[BC];
  bool b_ok[BC];
#pragma unroll
  for (int i = 0; i < BC; ++i) {
    const int c = tid + i * kThreads;
    b_row[i] = c >> 3;
    b_kc[i] = c & 7;
    b_ok[i] = (n0 + b_row[i]) < N;
  }

  f16x8 ra[AC], rb[BC];
  const f16x8 zero8 = {};

  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < AC; ++i) {
      const int k = k0 + a_kc[i] * 8;
      f16x8 v = zero8;
      if (a_ok[i] && k < K) {
        if constexpr (AMODE == S3N_A_DENSE) {
          v = *reinterpret_cast<const f16x8*>(a_base[i] + k);
        } else {
          const int tap = k / p.cC, ci = k - tap * p.cC;
          const int ky = tap / p.ks, kx = tap - ky * p.ks;
          const int iy = a_iy0[i] + ky, ix = a_ix0[i] + kx;
          if (iy >= 0 && iy < p.cH && ix >= 0 && ix < p.cW) {
            v = *reinterpret_cast<const f16x8*>(a_base[i] + ((int64_t)iy * p.cW + ix) * p.cC + ci);
            if (p.relu_in) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = v[j] > (f16)0 ? v[j] : (f16)0;
            }
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BC; ++i) {
      const int k = k0 + b_kc[i] * 8;
      f16x8 v = zero8;
      if (b_ok[i] && k < K)
        v = *reinterpret_cast<const f16x8*>(B + (int64_t)(n0 + b_row[i]) * p.ldb + k);
      rb[i] = v;
    }
  };
  auto sstore = [&](int buf) {
    f16* As = smem + buf * (BM + BN) * BK;
    f16* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < AC; ++i)
      *reinterpret_cast<f16x8*>(As + a_row[i] * BK + swz(a_row[i], a_kc[i]) * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BC; ++i)
      *reinterpret_cast<f16x8*>(Bs + b_row[i] * BK + swz(b_row[i], b_kc[i]) * 8) = rb[i];
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int KT = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) gload((kt + 1) * BK);
    const f16* As = smem + cur * (BM + BN) * BK;
    const f16* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int kc = 2 * ks + (lane >> 5);
      f16x8 af[FM], bf[FN];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int row = wm * WM + fm * 32 + (lane & 31);
        af[fm] = *reinterpret_cast<const f16x8*>(As + row * BK + swz(row, kc) * 8);
      }
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int row = wn * WN + fn * 32 + (lane & 31);
        bf[fn] = *reinterpret_cast<const f16x8*>(Bs + row * BK + swz(row, kc) * 8);
      }
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    if (kt + 1 < KT) sstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const float* __restrict__ bias = p.bias[g];
  const void* R1 = p.R1[g];
  const void* R2 = p.R2[g];
  void* C = p.C[g];
  f16* C2 = p.C2[g];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int col = n0 + wn * WN + fn * 32 + (lane & 31);
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + fm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        float v = acc[fm][fn][r] + bv;
        if (p.act == S3N_ACT_GELU) v = gelu(v);
        else if (p.act == S3N_ACT_RELU) v = fmaxf(v, 0.0f);
        if (R1) {
          const int64_t o = (int64_t)row * p.ldr1 + col;
          v += p.r1_f16 ? (float)reinterpret_cast<const f16*>(R1)[o] : reinterpret_cast<const float*>(R1)[o];
        }
        if (R2) {
          const int64_t o = (int64_t)row * p.ldr2 + col;
          v += p.r2_f16 ? (float)reinterpret_cast<const f16*>(R2)[o] : reinterpret_cast<const float*>(R2)[o];
        }
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
        if (p.c_f16) reinterpret_cast<f16*>(C)[off] = (f16)v;
        else reinterpret_cast<float*>(C)[off] = v;
        if (C2) C2[(int64_t)row * p.ldc2 + col] = (f16)v;
      }
    }
}

template <int BM, int BN>
int launch(const GemmP& p, hipStream_t st) {
  GemmP q = p;
  q.tiles_m = (p.M + BM - 1) / BM;
  q.tiles_n = (p.N + BN - 1) / BN;
  dim3 grid(q.tiles_m * q.tiles_n, 1, p.groups);
  if (p.a_mode == S3N_A_DENSE)
    k_gemm<BM, BN, S3N_A_DENSE><<<grid, kThreads, 0, st>>>(q);
  else
    k_gemm<BM, BN, S3N_A_CONV><<<grid, kThreads, 0, st>>>(q);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

}  // namespace

extern "C" int s3n_gemm(const s3n_gemm_args* a, void* stream) {
  S3_REQUIRE(a && a->M >= 0 && a->N > 0 && a->K > 0, "s3n_gemm: bad sizes");
  S3_REQUIRE(a->groups >= 1 && a->groups <= S3N_MAX_GROUPS, "s3n_gemm: groups must be 1..4");
  S3_REQUIRE(a->K % 8 == 0, "s3n_gemm: K must be a multiple of 8 (16-B operand chunks)");
  if (a->a_mode == S3N_A_DENSE) S3_REQUIRE(a->lda % 8 == 0, "s3n_gemm: lda %% 8 != 0");
  S3_REQUIRE(a->ldb % 8 == 0, "s3n_gemm: ldb %% 8 != 0");
  if (a->a_mode == S3N_A_CONV) {
    S3_REQUIRE(a->cC % 8 == 0, "s3n_gemm: conv Cin must be a multiple of 8");
    S3_REQUIRE(a->K == a->ksize * a->ksize * a->cC, "s3n_gemm: conv K != ks*ks*Cin");
    S3_REQUIRE(a->oH > 0 && a->oW > 0 && a->M % (a->oH * a->oW) == 0, "s3n_gemm: conv M");
  }
  for (int g = 0; g < a->groups; ++g)
    S3_REQUIRE(a->A[g] && a->B[g] && a->C[g], "s3n_gemm: null operand in group %d", g);
  if (a->M == 0) return S3_OK;
  GemmP p;
  p.M = a->M; p.N = a->N; p.K = a->K; p.groups = a->groups;
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    const bool on = g < a->groups;
    p.A[g] = on ? (const f16*)a->A[g] : nullptr;
    p.B[g] = on ? (const f16*)a->B[g] : nullptr;
    p.bias[g] = on ? a->bias[g] : nullptr;
    p.R1[g] = on ? a->R1[g] : nullptr;
    p.R2[g] = on ? a->R2[g] : nullptr;
    p.C[g] = on ? a->C[g] : nullptr;
    p.C2[g] = on ? (f16*)a->C2[g] : nullptr;
  }
  p.lda = a->lda; p.ldb = a->ldb; p.ldr1 = a->ldr1; p.r1_f16 = a->r1_f16;
  p.ldr2 = a->ldr2; p.r2_f16 = a->r2_f16; p.ldc = a->ldc; p.c_f16 = a->c_f16;
  p.ldc2 = a->ldc2; p.act = a->act; p.store_mode = a->store_mode; p.a_mode = a->a_mode;
  p.cH = a->cH; p.cW = a->cW; p.cC = a->cC; p.ks = a->ksize; p.st = a->stride; p.pad = a->pad;
  p.oH = a->oH; p.oW = a->oW; p.relu_in = a->relu_in;
  p.sH = a->sH; p.sW = a->sW; p.sS = a->sS; p.sCout = a->sCout;
  hipStream_t st = s3::as_stream(stream);
  // Tile choice: fill the 256 CUs before growing the tile.
  auto tiles = [&](int bm, int bn) {
    return (int64_t)a->groups * ((a->M + bm - 1) / bm) * ((a->N + bn - 1) / bn);
  };
  if (tiles(128, 128) >= 240) return launch<128, 128>(p, st);
  if (tiles(64, 128) >= 200 && a->N >= 128) return launch<64, 128>(p, st);
  return launch<64, 64>(p, st);
}
