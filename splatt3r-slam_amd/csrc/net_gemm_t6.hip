// 3x3 / stride 1 / pad 1 implicit-GEMM convolution with halo reuse of the
// input row segment (tiles 40-42; see net_gemm_kernel.hpp for the shared
// epilogue and LDS-DMA helpers).
//
// The generic conv path (k_gemm AMODE kConv) loads, for every K tile
// (ky, kx, 64 input channels), the BM output pixels' tap pixels by LDS-DMA:
// each input pixel of a tile's row segment crosses the L2 -> LDS path 9 times
// per channel chunk, once per tap.  Here an output tile is one row segment
// of BM pixels (BM divides the output width), and the K tiles run in the
// order (ky, channel chunk, kx): one LDS-DMA brings the BM + 2 input pixels
// (ox0 - 1 .. ox0 + BM) of row oy + ky - 1 and one 64-channel chunk, and the
// three kx taps read it at row offsets 0, 1, 2 (the XOR swizzle stays
// conflict-free at every offset: 16 consecutive rows always hit 16 distinct
// 16-B slots).  A traffic drops 9 -> 3 row segments per channel chunk; the
// weights are read in place (B tile = columns (ky*3 + kx) * Cin + chunk * 64
// of the [Cout, 9 Cin] matrix), so nothing is repacked.  One barrier per
// (ky, chunk) super-step of 3 K tiles; the next super-step's DMA is issued
// right after it and overlaps the current MFMAs.
//
// The K summation order differs from the generic conv path ((ky, chunk, kx)
// instead of (ky, kx, chunk)); ops.reduction_class tells the tuner so, so
// batch-invariant plans never mix the two.
#include "net_gemm_kernel.hpp"

namespace {

template <int BM, int BN, int NWM, int NWN, int MF, bool RELU_IN, bool PIPE, int S>
__global__ void __launch_bounds__(64 * NWM * NWN, S == 1 ? 2 : 1) k_conv3_halo(GemmP p) {
  typedef AccT<MF> AT;
  constexpr int NW = NWM * NWN;
  constexpr int NT = 64 * NW;
  constexpr int BK = 64;
  constexpr int WM = BM / NWM, WN = BN / NWN;
  constexpr int FM = WM / MF, FN = WN / MF;
  static_assert(WM % MF == 0 && WN % MF == 0, "whole MFMA blocks per wave");
  constexpr int AROWS = BM + 2;               // input pixels ox0 - 1 .. ox0 + BM
  constexpr int AINS = (AROWS + 7) / 8;       // LDS-DMA wave instructions (8 rows of 128 B)
  constexpr int AIW = (AINS + NW - 1) / NW;   // per wave (the last ones may idle)
  constexpr int BW = BN / 8 / NW;             // per wave per tap
  static_assert(BW * 8 * NW == BN, "B rows split over waves");
  constexpr int A_EL = AINS * 8 * BK;
  constexpr int B_EL = BN * BK;
  constexpr int STAGE0 = A_EL + 3 * B_EL;
  // S = 1 (one super-stage, two workgroups per CU: one's DMA and epilogue
  // overlap the other's MFMAs): the stage also holds the epilogue's padded
  // fp32 tile and the fused tail's weights
  constexpr int EPI_EL = (BM * (BN + 4) * 4 + 16 * BN * 4) / 2;   // + fp32 tail weights
  constexpr int STAGE = S == 1 ? ((STAGE0 > EPI_EL ? STAGE0 : EPI_EL) + 511) / 512 * 512 : STAGE0;
  static_assert(S == 1 || S == 2, "one or two super-stages");
  __shared__ __attribute__((aligned(1024))) f16 smem[S * STAGE];

  const int g = blockIdx.z;
  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n, tn = tile % p.tiles_n;   // column tiles of a segment adjacent
  const int m0 = tm * BM, n0 = tn * BN;
  const int hw = p.oH * p.oW;
  const int b = m0 / hw, rem = m0 - b * hw;
  const int oy = rem / p.oW, ox0 = rem - oy * p.oW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  const int C = p.cC;
  const f16* __restrict__ A = p.A[g];
  const f16* __restrict__ B = p.B[g];
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A, (int64_t)(p.M / hw) * p.cH * p.cW * C * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, ((int64_t)(p.N - 1) * p.ldb + p.K) * 2);

  // per-lane A offsets (bytes, without the row iy and the channel chunk) of
  // this wave's segment instructions: pixel ox0 - 1 + r of image b
  const int lrow = lane >> 3, lchunk = lane & 7;
  uint32_t a_off[AIW];
#pragma unroll
  for (int j = 0; j < AIW; ++j) {
    const int ins = wave + j * NW;
    const int r = ins * 8 + lrow;
    const int ix = ox0 - 1 + r;
    const bool ok = ins < AINS && r < AROWS && ix >= 0 && ix < p.cW;
    a_off[j] = ok ? (uint32_t)((((int64_t)b * p.cH * p.cW + ix) * C + swz<BK>(r, lchunk) * 8) * 2)
                  : kOOB;
  }
  uint32_t b_off[BW];
#pragma unroll
  for (int j = 0; j < BW; ++j) {
    const int r = (wave * BW + j) * 8 + lrow;
    b_off[j] = (n0 + r) < p.N ? (uint32_t)(((int64_t)(n0 + r) * p.ldb + swz<BK>(r, lchunk) * 8) * 2)
                              : kOOB;
  }
  const int CC = C / BK;            // channel chunks
  const int SS = 3 * CC;            // super-steps (ky, chunk)
  auto issue = [&](int ss, int st) {
    const int ky = ss / CC, cc = ss - ky * CC;
    f16* As = smem + st * STAGE;
    f16* Bs = As + A_EL;
    const int iy = oy + ky - 1;
    const bool row_ok = iy >= 0 && iy < p.cH;   // wave-uniform
    const int a_soff = row_ok ? (iy * p.cW * C + cc * BK) * 2 : 0;
#pragma unroll
    for (int j = 0; j < AIW; ++j) {
      const int ins = wave + j * NW;
      if (ins < AINS && !(p.debug & 2))
        S3_BLDS(ra, As + ins * 512, row_ok ? a_off[j] : kOOB, a_soff);
    }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int k0 = (ky * 3 + kx) * C + cc * BK;
#pragma unroll
      for (int j = 0; j < BW; ++j)
        if (!(p.debug & 2)) S3_BLDS(rb, Bs + kx * B_EL + (wave * BW + j) * 512, b_off[j], k0 * 2);
    }
  };

  typename AT::T acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < AT::R; ++r) acc[i][j][r] = 0.0f;

  const int SSn = (p.debug & 8) ? 0 : SS;
  if (SSn > 0) issue(0, 0);
  for (int ss = 0; ss < SSn; ++ss) {
    if constexpr (S == 1) {
      if (ss > 0) {
        s3::ring_barrier();   // every wave is done reading the stage
        issue(ss, 0);
      }
    }
    // this super-step's DMA (the only one outstanding) has landed, and every
    // wave is done reading the stage the next one overwrites
    wait_vmcnt<0>();
    s3::ring_barrier();
    if constexpr (S == 2)
      if (ss + 1 < SSn) issue(ss + 1, (ss + 1) & 1);
    const f16* As = smem + (S == 2 ? (ss & 1) : 0) * STAGE;
    const f16* Bs = As + A_EL;
    constexpr int NKS = BK / AT::KS;
    // fragments of tap kx: A rows shifted by kx (the halo), B tile kx
    auto frags = [&](int kx, f16x8 (&af)[NKS][FM], f16x8 (&bf)[NKS][FN]) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int kc = AT::frag_chunk(ks, lane);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int row = wm * WM + fm * MF + AT::frag_row(lane) + kx;
          af[ks][fm] = *reinterpret_cast<const f16x8*>(As + row * BK + swz<BK>(row, kc) * 8);
        }
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int row = wn * WN + fn * MF + AT::frag_row(lane);
          bf[ks][fn] =
              *reinterpret_cast<const f16x8*>(Bs + kx * B_EL + row * BK + swz<BK>(row, kc) * 8);
        }
      }
    };
    auto mfmas = [&](f16x8 (&af)[NKS][FM], f16x8 (&bf)[NKS][FN]) {
      if (p.debug & 1) return;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if constexpr (RELU_IN) {
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
    };
    if constexpr (PIPE) {
      // tap kx + 1's fragments are read while tap kx's MFMAs run (one wave
      // per SIMD: nothing else hides the LDS latency)
      f16x8 a0[NKS][FM], b0[NKS][FN], a1[NKS][FM], b1[NKS][FN];
      frags(0, a0, b0);
      frags(1, a1, b1);
      mfmas(a0, b0);
      frags(2, a0, b0);
      mfmas(a1, b1);
      mfmas(a0, b0);
    } else {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        f16x8 af[NKS][FM], bf[NKS][FN];
        frags(kx, af, bf);
        mfmas(af, bf);
      }
    }
  }
  if (p.debug & 4) return;
  constexpr int RING = S * STAGE * 2;
  constexpr int LDT = BM * (BN + 4) * 4 <= RING ? BN + 4 : BN;
  static_assert(BM * LDT * 4 <= RING, "fp32 tile staged in the LDS ring");
  epilogue_vec<BM, BN, NWM, NWN, FM, FN, LDT, RING, 1, MF>(p, g, m0, n0, acc,
                                                           reinterpret_cast<float*>(smem));
}

template <int BM, int BN, int NWM, int NWN, int MF, bool PIPE, int S = 2>
int launch_halo(const GemmP& p, hipStream_t st) {
  S3_REQUIRE(p.a_mode != S3N_A_DENSE && p.ks == 3 && p.st == 1 && p.pad == 1 &&
                 p.cH == p.oH && p.cW == p.oW,
             "s3n_gemm: halo tiles need a 3x3 / stride 1 / pad 1 conv");
  S3_REQUIRE(p.cC % 64 == 0 && p.oW % BM == 0, "s3n_gemm: halo tiles need Cin %% 64 == 0 and "
                                               "BM (%d) dividing the output width (%d)", BM, p.oW);
  S3_REQUIRE(p.split_k <= 1 && p.vec_epi && p.store_mode == S3N_STORE_PLAIN,
             "s3n_gemm: halo tiles need split_k 1, the vector epilogue and a plain store");
  S3_REQUIRE(!p.tail_w[0] || p.N == BN, "s3n_gemm: the fused tail needs N == BN (%d)", BN);
  GemmP q = p;
  q.tiles_m = p.M / BM;
  q.tiles_n = (p.N + BN - 1) / BN;
  q.split_k = 1;
  dim3 grid(q.tiles_m * q.tiles_n, 1, p.groups);
  if (p.relu_in)
    k_conv3_halo<BM, BN, NWM, NWN, MF, true, PIPE, S><<<grid, 64 * NWM * NWN, 0, st>>>(q);
  else
    k_conv3_halo<BM, BN, NWM, NWN, MF, false, PIPE, S><<<grid, 64 * NWM * NWN, 0, st>>>(q);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

}  // namespace

namespace s3gemm {
// halo conv tiles: 128x128 (16x16x32 MFMA, 4 waves of 64x64), 256x64
// (16x16x32, 4 waves of 128x32), 128x128 (32x32x16, 4 waves of 64x64);
// 43, 45: 40 / 42 with the taps' fragment reads software-pipelined (the
// 256x64 form would spill with them)
int launch_t6(int tile, const GemmP& p, hipStream_t st) {
  if (tile == 40) return launch_halo<128, 128, 2, 2, 16, false>(p, st);
  if (tile == 41) return launch_halo<256, 64, 2, 2, 16, false>(p, st);
  if (tile == 42) return launch_halo<128, 128, 2, 2, 32, false>(p, st);
  if (tile == 43) return launch_halo<128, 128, 2, 2, 16, true>(p, st);
  if (tile == 45) return launch_halo<128, 128, 2, 2, 32, true>(p, st);
  // 8 waves (two per SIMD: one wave's LDS reads hide behind the other's MFMAs)
  if (tile == 46) return launch_halo<128, 128, 2, 4, 16, false>(p, st);
  if (tile == 47) return launch_halo<256, 64, 4, 2, 16, false>(p, st);
  if (tile == 48) return launch_halo<128, 128, 2, 4, 32, false>(p, st);
  if (tile == 49) return launch_halo<128, 128, 2, 4, 16, true>(p, st);
  if (tile == 50) return launch_halo<256, 64, 4, 2, 16, true>(p, st);
  // one super-stage, two workgroups per CU
  if (tile == 51) return launch_halo<128, 128, 2, 2, 16, false, 1>(p, st);
  if (tile == 52) return launch_halo<128, 128, 2, 2, 32, false, 1>(p, st);
  if (tile == 53) return launch_halo<256, 64, 2, 2, 16, false, 1>(p, st);
  return kNotMine;
}
int sat_t6(int reset) { return read_sat(reset); }
}  // namespace s3gemm
