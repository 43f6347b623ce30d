// GEMM tile family instantiations (see net_gemm_kernel.hpp); one
// translation unit per family so hipcc compiles them in parallel.
#include "net_gemm_kernel.hpp"

namespace s3gemm {
// v_mfma_f32_16x16x32 tiles: 4 waves (2 x 2), one large tile per CU (wave
// tiles 32x80, 48x32, 64x48, 80x64, 128x64): the decomposition hipBLASLt
// picks for the network's M = 768 shapes on gfx950.  A 16x16 tile without
// the vector epilogue (unaligned operands) falls back to tile 1.
int launch_t4(int tile, const GemmP& p, hipStream_t st) {
  if (tile < 21 || tile > 25) return kNotMine;
  if (!p.vec_epi) return launch_t1(1, p, st);
  if (tile == 21) return launch<64, 160, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 22) return launch<96, 64, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 23) return launch<128, 96, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 24) return launch<160, 128, 3, 2, 2, 64, 1, 16>(p, st);
  return launch<256, 128, 3, 2, 2, 64, 1, 16>(p, st);
}
int sat_t4(int reset) { return read_sat(reset); }
}  // namespace s3gemm
