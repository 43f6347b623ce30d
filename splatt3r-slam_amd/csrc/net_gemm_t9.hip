// Dense fp16 GEMM with the B operand (the weights) read straight from a
// fragment-major packed copy into registers: no LDS stage, no LDS reads and
// no barrier dependency for B.  A (the activations, shared by the waves of a
// row of the tile) keeps the LDS-DMA ring and XOR-swizzled fragment reads of
// k_gemm (net_gemm_kernel.hpp).
//
// Packed layout (s3n_gemm_args.Bp, ops.packed_b): Bp[nb][ks][lane][8] for nb = n / 16,
// ks = k / 32, lane = 16 * ((k % 32) / 8) + n % 16, element k % 8 -- one
// v_mfma_f32_16x16x32_f16 B fragment is 1 KiB contiguous, so a wave loads
// it with one fully coalesced 16-B-per-lane buffer load.  N is padded to a
// multiple of 16 with zeros; K must be a multiple of 32.
//
// Reduction order: the K tiles of the workgroup's split run in order, each
// as two 16x16x32 steps in k order, into one accumulator chain per element
// -- the order of every other 16x16x32 tile without K-groups
// (ops.reduction_class (16, 1, 0, bound, ...)); with split-K each split's
// fp32 plane goes through the shared k_splitk_reduce, which adds the planes
// in split order, and without it the same LDS-staged vector epilogue: these
// tiles compute the same bits as the LDS-staged tiles of their class.
//
// The A tile and the B fragments of K tile kt are issued together (one
// "tile" of AW + 2 FN vector-memory operations per wave), S - 1 tiles ahead,
// so the one vmcnt counter orders both: when tile kt has landed, so has its
// B.  B lives in an S-deep register ring indexed by kt % S (the K loop is
// unrolled by S so the indices are static).
#include "net_gemm_kernel.hpp"

#include <type_traits>
#include <utility>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int BM, int BN, int NWM, int NWN, int S>
constexpr int bd_min_waves() {
  // waves per SIMD the register budget allows: ~ acc + A frags + B ring
  constexpr int NW = NWM * NWN;
  constexpr int FM = BM / NWM / 16, FN = BN / NWN / 16;
  constexpr int regs = FM * FN * 4 + 2 * FM * 4 + S * 2 * FN * 4 + 40;
  constexpr int per_simd = regs <= 128 ? 4 : (regs <= 168 ? 3 : (regs <= 256 ? 2 : 1));
  // workgroups of NW waves: NW / 4 waves per SIMD each
  constexpr int wg = per_simd * 4 / NW;
  return (wg < 1 ? 1 : wg) * NW / 4;
}

template <int BM, int BN, int NWM, int NWN, int S>
__global__ void __launch_bounds__(64 * NWM * NWN, (bd_min_waves<BM, BN, NWM, NWN, S>()))
k_gemm_bd(GemmP p) {
  typedef AccT<16> AT;
  constexpr int BK = 64;
  constexpr int NW = NWM * NWN;
  constexpr int WM = BM / NWM, WN = BN / NWN;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int CPR = BK / 8;       // 16-B chunks per A row
  constexpr int RPI = 64 / CPR;     // A rows per DMA wave instruction
  constexpr int AW = BM / RPI / NW;
  static_assert(AW * RPI * NW == BM, "A rows split over the waves");
  static_assert(WM % 16 == 0 && WN % 16 == 0, "16x16 blocks per wave");
  constexpr int NKS = 2;            // 16x16x32 steps per K tile
  constexpr int PERW = AW + NKS * FN;
  constexpr int AHEAD = S - 1;
  constexpr int STAGE = BM * BK;    // fp16 elements of one A stage
  constexpr int RING = S * STAGE * 2;
  constexpr int LDT = BN + 4;
  constexpr int EPI = BM * LDT * 4;
  constexpr int SMEM = RING > EPI ? RING : EPI;
  __shared__ __attribute__((aligned(1024))) char smem_raw[SMEM];
  f16* const ring = reinterpret_cast<f16*>(smem_raw);

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
  const f16* __restrict__ Bp = p.Bp[g];
  // this workgroup's K tiles: split blockIdx.y of plan_grid's partition
  const int KT_all = (K + BK - 1) / BK;
  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int KT = min(KT_all, kt_begin + p.kt_per_split) - kt_begin;
  const int KS = K / 32;            // packed K steps (host: K % 32 == 0)
  const int Npad = (N + 15) & ~15;

  // A: lane -> (row within its 8-row group, swizzled chunk)
  const int lrow = lane / CPR, lchunk = lane % CPR;
  uint32_t a_off[AW];
  int a_kc[AW];
#pragma unroll
  for (int j = 0; j < AW; ++j) {
    const int r = (wave * AW + j) * RPI + lrow;
    a_kc[j] = swz<BK>(r, lchunk);
    const int m = m0 + r;
    a_off[j] = m < M ? (uint32_t)(((int64_t)m * p.lda + a_kc[j] * 8) * 2) : kOOB;
  }
  // B: this wave's 16-column blocks, byte offset of (nb, ks = 0, lane)
  uint32_t b_off[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int nb = (n0 + wn * WN) / 16 + fn;
    b_off[fn] = nb * 16 < N ? (uint32_t)(((int64_t)nb * KS * 64 + lane) * 16) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A, ((int64_t)(M - 1) * p.lda + K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bp, (int64_t)Npad * K * 2);

  f16x8 bq[S][NKS][FN];
  typename AT::T acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < AT::R; ++r) acc[i][j][r] = 0.0f;

  // Every step issues a tile (tiles past KT read zeros: out-of-range buffer
  // offsets), so the number of vector-memory operations behind any tile is
  // always AHEAD - 1 tiles' worth and the waits are constants.
  auto issue = [&](int kt, auto stc) {
    constexpr int st = decltype(stc)::value;
    f16* As = ring + st * STAGE;
    const int k0 = (kt_begin + kt) * BK;
    const bool live = kt < KT;
#pragma unroll
    for (int j = 0; j < AW; ++j) {
      uint32_t off = a_off[j];
      if (!live || k0 + a_kc[j] * 8 >= K) off = kOOB;
      S3_BLDS(ra, As + (wave * AW + j) * 512, off, live ? k0 * 2 : 0);
    }
#pragma unroll
    for (int q = 0; q < NKS; ++q) {
      const int ks = 2 * (kt_begin + kt) + q;
      const bool ok = live && ks < KS;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
            rb, ok ? b_off[fn] : kOOB, ok ? ks * 1024 : 0, 0);
        bq[st][q][fn] = __builtin_bit_cast(f16x8, v);
      }
    }
  };

  auto step = [&](int kt, auto stc) {
    constexpr int st = decltype(stc)::value;
    // own A DMA + B loads of tile kt landed (the AHEAD - 1 later tiles may
    // stay in flight); after the barrier every wave's A of tile kt is
    // visible and the stage tile kt + AHEAD refills is no longer read
    wait_vmcnt<PERW * (AHEAD - 1)>();
    s3::ring_barrier();
    const bool live = kt < KT;
    f16x8 af[NKS][FM];
    if (live) {
      const f16* As = ring + st * STAGE;
#pragma unroll
      for (int q = 0; q < NKS; ++q) {
        const int kc = AT::frag_chunk(q, lane);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int row = wm * WM + fm * 16 + AT::frag_row(lane);
          af[q][fm] = *reinterpret_cast<const f16x8*>(As + row * BK + swz<BK>(row, kc) * 8);
        }
      }
    }
    issue(kt + AHEAD, std::integral_constant<int, (st + AHEAD) % S>{});
    if (live) {
#pragma unroll
      for (int q = 0; q < NKS; ++q)
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] = AT::mfma(af[q][fm], bq[st][q][fn], acc[fm][fn]);
    }
  };

  // prologue: tiles 0 .. AHEAD-1 into stages 0 .. AHEAD-1
  static_for<0, AHEAD>([&](auto ic) { issue(decltype(ic)::value, ic); });
  for (int kt = 0; kt < KT; kt += S)
    static_for<0, S>([&](auto ic) { step(kt + decltype(ic)::value, ic); });
  // the phantom tiles' DMA must land before the ring becomes the epilogue's
  // staging area
  wait_vmcnt<0>();
  epilogue_vec<BM, BN, NWM, NWN, FM, FN, LDT, SMEM, 1, 16>(
      p, g, m0, n0, acc, reinterpret_cast<float*>(smem_raw));
}

template <int BM, int BN, int NWM, int NWN, int S>
int launch_bd(const GemmP& p, hipStream_t st) {
  S3_REQUIRE(p.a_mode == S3N_A_DENSE && p.Bp[0] && p.vec_epi && !p.tail_w[0] && p.K % 32 == 0,
             "s3n_gemm: B-direct tiles need dense A, the packed B (s3n_gemm_args.Bp), the vector "
             "epilogue, no fused tail and K %% 32 == 0");
  const GemmP q = plan_grid(p, BM, BN, 64);
  dim3 grid(q.tiles_m * q.tiles_n, q.split_k, p.groups);
  k_gemm_bd<BM, BN, NWM, NWN, S><<<grid, 64 * NWM * NWN, 0, st>>>(q);
  S3_LAUNCH_CHECK();
  return launch_splitk_reduce(q, st);
}

}  // namespace

namespace s3gemm {
// tiles 70-79 (ops._BDIRECT); launch configurations measured against the
// LDS-staged tiles of the same reduction class on the network's dense shapes
// (tools/bench_gemm_bd.py, profiles/r06b_gemm_bdirect.log)
int launch_t9(int tile, const GemmP& p, hipStream_t st) {
  switch (tile) {
    case 70: return launch_bd<64, 128, 1, 4, 3>(p, st);    // wave 64 x 32
    case 71: return launch_bd<64, 128, 1, 4, 2>(p, st);    // double-buffered
    case 72: return launch_bd<64, 64, 1, 4, 3>(p, st);     // wave 64 x 16
    case 73: return launch_bd<64, 64, 1, 4, 4>(p, st);
    case 74: return launch_bd<128, 128, 1, 4, 4>(p, st);   // wave 128 x 32
    case 75: return launch_bd<128, 128, 1, 4, 3>(p, st);
    case 76: return launch_bd<128, 128, 2, 4, 3>(p, st);   // 8 waves, wave 64 x 32
    case 77: return launch_bd<64, 128, 1, 4, 4>(p, st);
    // 6-stage rings (5 K tiles in flight) for the latency-bound decoder
    // launches: B needs no LDS, so a stage is only the A tile (8 KiB at BM 64)
    case 78: return launch_bd<64, 64, 1, 4, 6>(p, st);
    case 79: return launch_bd<64, 128, 1, 4, 6>(p, st);
    default: return kNotMine;
  }
}
int sat_t9(int reset) { return read_sat(reset); }
}  // namespace s3gemm
