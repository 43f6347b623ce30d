// GEMM tiles 60, 62-68: the k_gemm tile math (LDS-DMA ring, XOR-swizzled
// fragments, fused epilogues: net_gemm_kernel.hpp) with a K loop whose LDS
// fragment reads overlap the MFMAs of the same wave.
//
// k_gemm reads a whole K tile's fragments, then runs its MFMA chain: with one
// wave per SIMD (the 256 x 128 four-wave tiles, whose 128 x 64 wave tiles
// need the fewest LDS bytes per MFMA) nothing covers the fragment-read
// latency, so the SIMD idles at every K step.  Here each K tile is consumed
// in two halves held in two register sets: the reads of half 1 are issued
// before the MFMAs of half 0, the reads of the NEXT tile's half 0 before the
// MFMAs of half 1.  One barrier per K tile sits between the halves: before
// it every wave has waited for its own reads of the current stage and for
// its own DMA of the next tile, so after it the next tile is visible to all
// and the current stage may be refilled (the ring holds S tiles, all of
// them issued ahead).  Same reduction order as k_gemm with the same MFMA
// shape and K tile (ops.reduction_class: tiles 60-66 share the classes of
// k_gemm tiles).
#include "net_gemm_kernel.hpp"

namespace {

template <int BM, int BN, int NWM, int NWN, int AMODE, int S, int MF>
__global__ void __launch_bounds__(64 * NWM * NWN, lds_waves_per_simd(BM, BN, NWM * NWN, S, 64))
k_gemm_pp(GemmP p) {
  typedef AccT<MF> AT;
  constexpr int BK = 64;
  constexpr int NW = NWM * NWN;
  constexpr int WM = BM / NWM, WN = BN / NWN;
  constexpr int FM = WM / MF, FN = WN / MF;
  constexpr int CPR = BK / 8;          // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;        // tile rows per DMA wave instruction
  constexpr int AW = BM / RPI / NW, BW = BN / RPI / NW;
  static_assert(AW * RPI * NW == BM && BW * RPI * NW == BN, "LDS-DMA rows must split over waves");
  static_assert(WM % MF == 0 && WN % MF == 0, "whole MFMA accumulator blocks per wave");
  static_assert(S >= 2, "ring of at least two stages");
  constexpr int PERW = AW + BW;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int NKS = BK / AT::KS;     // MFMA K steps per K tile (2 or 4)
  constexpr int HK = NKS / 2;          // per half
  __shared__ __attribute__((aligned(1024))) f16 smem[S * STAGE];

  const int g = blockIdx.z;
  const int nwg = p.tiles_m * p.tiles_n;
  int tm, tn;
  if (p.xcd_px > 0) {
    const int px = p.xcd_px, py = 8 / px;
    const int xcd = blockIdx.x % 8, k = blockIdx.x / 8;
    const int rm = p.tiles_m / px, rn = p.tiles_n / py;
    tm = (xcd / py) * rm + k % rm;
    tn = (xcd % py) * rn + k / rm;
  } else {
    const int tile = xcd_remap(blockIdx.x, nwg);
    tm = p.col_major ? tile % p.tiles_m : tile / p.tiles_n;
    tn = p.col_major ? tile / p.tiles_m : tile % p.tiles_n;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  const int M = p.M, N = p.N, K = p.K;
  const f16* __restrict__ A = p.A[g];
  const f16* __restrict__ B = p.B[g];
  const int KT_all = (K + BK - 1) / BK;
  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int kt_end = min(KT_all, kt_begin + p.kt_per_split);

  const int lrow = lane / CPR, lchunk = lane % CPR;
  uint32_t a_off[AW];
  int64_t a_img[AW];
  int a_iy0[AW], a_ix0[AW];
  bool a_ok[AW];
  int a_kc[AW];
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
      const int k = kt_begin * BK + a_kc[j] * 8, tap = k / p.cC;
      c_ci[j] = k - tap * p.cC;
      c_ky[j] = tap / p.ks;
      c_kx[j] = tap - c_ky[j] * p.ks;
    }
  }
  uint32_t b_off[BW];
  int b_kc[BW];
#pragma unroll
  for (int j = 0; j < BW; ++j) {
    const int r = (wave * BW + j) * RPI + lrow;
    b_kc[j] = swz<BK>(r, lchunk);
    b_off[j] = (n0 + r) < N ? (uint32_t)(((int64_t)(n0 + r) * p.ldb + b_kc[j] * 8) * 2) : kOOB;
  }
  const int Bn = AMODE == kDense ? 0 : M / (p.oH * p.oW);
  const __amdgpu_buffer_rsrc_t ra =
      AMODE == kDense ? make_rsrc(A, ((int64_t)(M - 1) * p.lda + K) * 2)
                      : make_rsrc(A, (int64_t)Bn * p.cH * p.cW * p.cC * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, ((int64_t)(N - 1) * p.ldb + K) * 2);
  const bool k_tail = (K % BK) != 0;

  // LDS-DMA of K tile kt into stage st (tiles issued in order: the conv
  // state advances one tile per call)
  auto issue = [&](int kt, int st) {
    f16* As = smem + st * STAGE;
    f16* Bs = As + BM * BK;
    const int k0 = kt * BK;
    const bool tail = k_tail && (k0 + BK > K);
#pragma unroll
    for (int j = 0; j < AW; ++j) {
      uint32_t off;
      if constexpr (AMODE == kDense) {
        off = a_off[j];
        if (tail && k0 + a_kc[j] * 8 >= K) off = kOOB;
        S3_BLDS(ra, As + (wave * AW + j) * 512, off, k0 * 2);
      } else {
        off = kOOB;
        const int iy = a_iy0[j] + c_ky[j], ix = a_ix0[j] + c_kx[j];
        if (a_ok[j] && !(tail && k0 + a_kc[j] * 8 >= K) && iy >= 0 && iy < p.cH && ix >= 0 &&
            ix < p.cW)
          off = (uint32_t)((a_img[j] + ((int64_t)iy * p.cW + ix) * p.cC + c_ci[j]) * 2);
        c_ci[j] += BK;
        while (c_ci[j] >= p.cC) {
          c_ci[j] -= p.cC;
          if (++c_kx[j] == p.ks) { c_kx[j] = 0; ++c_ky[j]; }
        }
        S3_BLDS(ra, As + (wave * AW + j) * 512, off, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BW; ++j) {
      uint32_t off = b_off[j];
      if (tail && k0 + b_kc[j] * 8 >= K) off = kOOB;
      S3_BLDS(rb, Bs + (wave * BW + j) * 512, off, k0 * 2);
    }
  };

  typename AT::T acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < AT::R; ++r) acc[i][j][r] = 0.0f;

  // fragments of one half K tile: MFMA K steps h*HK .. h*HK + HK - 1
  typedef f16x8 FragA[HK][FM];
  typedef f16x8 FragB[HK][FN];
  auto read_half = [&](int st, int h, FragA& a, FragB& b) {
    const f16* As = smem + st * STAGE;
    const f16* Bs = As + BM * BK;
#pragma unroll
    for (int q = 0; q < HK; ++q) {
      const int kc = AT::frag_chunk(h * HK + q, lane);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int row = wm * WM + fm * MF + AT::frag_row(lane);
        a[q][fm] = *reinterpret_cast<const f16x8*>(As + row * BK + swz<BK>(row, kc) * 8);
      }
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int row = wn * WN + fn * MF + AT::frag_row(lane);
        b[q][fn] = *reinterpret_cast<const f16x8*>(Bs + row * BK + swz<BK>(row, kc) * 8);
      }
    }
  };
  auto mma_half = [&](FragA& a, FragB& b) {
#pragma unroll
    for (int q = 0; q < HK; ++q) {
      if constexpr (AMODE == kConvRelu) {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int e = 0; e < 8; ++e) a[q][fm][e] = a[q][fm][e] > (f16)0 ? a[q][fm][e] : (f16)0;
      }
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = AT::mfma(a[q][fm], b[q][fn], acc[fm][fn]);
    }
  };

  const int KT = kt_end - kt_begin;
  FragA ra0, ra1;
  FragB rb0, rb1;
  // prologue: every stage filled, tile 0 landed and visible, its half 0 read
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i < KT) issue(kt_begin + i, i);
  if (KT > 0) {
    wait_tiles<PERW, S - 1>(KT - 1);
    s3::ring_barrier();
    read_half(0, 0, ra0, rb0);
  }
  for (int kt = 0; kt < KT; ++kt) {
    const int st = kt % S;
    read_half(st, 1, ra1, rb1);     // in flight behind the half-0 MFMAs
    mma_half(ra0, rb0);
    if (kt + 1 < KT) {
      // own DMA of tile kt+1 landed (tiles issued after it may stay in
      // flight), own reads of stage st retired; after the barrier everyone's
      // are, so stage st takes tile kt+S and tile kt+1 is readable
      wait_tiles<PERW, S - 2>(KT - 2 - kt);
      s3::ring_barrier();
      if (kt + S < KT) issue(kt_begin + kt + S, st);
      read_half((kt + 1) % S, 0, ra0, rb0);
    }
    mma_half(ra1, rb1);
  }

  // ---- epilogue (same as k_gemm) ----
  constexpr bool kVecFits = BM * BN * 4 <= S * STAGE * 2;
  if constexpr (kVecFits) {
    if (p.vec_epi) {
      constexpr int LDT = BM * (BN + 4) * 4 <= S * STAGE * 2 ? BN + 4 : BN;
      epilogue_vec<BM, BN, NWM, NWN, FM, FN, LDT, S * STAGE * 2, 1, MF>(
          p, g, m0, n0, acc, reinterpret_cast<float*>(smem));
      return;
    }
  }
  if constexpr (MF == 32) {
    epilogue_regs<BM, BN, NWM, NWN, FM, FN>(p, g, m0, n0, acc);
  }
}

template <int BM, int BN, int S, int NWM, int NWN, int MF>
int launch_pp(const GemmP& p, hipStream_t st) {
  constexpr int BK = 64;
  S3_REQUIRE(MF == 32 || p.vec_epi, "s3n_gemm: 16x16 MFMA tiles need the vector epilogue");
  static_assert(MF == 32 || BM * BN * 4 <= S * (BM + BN) * BK * 2,
                "16x16 MFMA tiles stage their fp32 tile in the LDS ring");
  S3_REQUIRE(!p.tail_w[0] || p.N == BN,
             "s3n_gemm: the fused tail needs N == the tile width (%d, N = %d)", BN, p.N);
  S3_REQUIRE(!p.tail_w[0] || BM * BN * 4 <= S * (BM + BN) * BK * 2,
             "s3n_gemm: the fused tail needs a tile whose fp32 image fits its LDS ring");
  constexpr int NT = 64 * NWM * NWN;
  const GemmP q = plan_grid(p, BM, BN, BK);
  dim3 grid(q.tiles_m * q.tiles_n, q.split_k, p.groups);
  if (p.a_mode == S3N_A_DENSE)
    k_gemm_pp<BM, BN, NWM, NWN, kDense, S, MF><<<grid, NT, 0, st>>>(q);
  else if (p.relu_in)
    k_gemm_pp<BM, BN, NWM, NWN, kConvRelu, S, MF><<<grid, NT, 0, st>>>(q);
  else
    k_gemm_pp<BM, BN, NWM, NWN, kConv, S, MF><<<grid, NT, 0, st>>>(q);
  S3_LAUNCH_CHECK();
  return launch_splitk_reduce(q, st);
}

}  // namespace

namespace s3gemm {
int launch_t8(int tile, const GemmP& p, hipStream_t st) {
  if (tile < 60 || tile > 68) return kNotMine;
  if (tile == 61) return kNotMine;   // 256 x 128 with 32x32 MFMAs spills (576 B/lane)
  // the 16x16 tiles stage their fp32 tile through LDS: no silent fallback to
  // another tile (that would change the launch's reduction class)
  S3_REQUIRE(tile == 65 || p.vec_epi, "s3n_gemm: 16x16 MFMA tiles need the vector epilogue");
  switch (tile) {
    case 60: return launch_pp<256, 128, 3, 2, 2, 16>(p, st);   // wave 128 x 64
    case 62: return launch_pp<128, 256, 3, 2, 2, 16>(p, st);   // wave 64 x 128
    case 63: return launch_pp<128, 128, 2, 2, 2, 16>(p, st);   // 64 KiB: 2 workgroups per CU
    case 64: return launch_pp<192, 128, 3, 2, 2, 16>(p, st);   // wave 96 x 64
    case 65: return launch_pp<128, 128, 2, 2, 2, 32>(p, st);
    case 66: return launch_pp<128, 192, 3, 2, 2, 16>(p, st);   // wave 64 x 96
    case 67: return kNotMine;   // 256 x 256: the fp32 tile does not fit the 2-stage ring
    default: return launch_pp<256, 128, 3, 4, 2, 16>(p, st);   // 8 waves, wave 64 x 64
  }
}
int sat_t8(int reset) { return read_sat(reset); }
}  // namespace s3gemm
