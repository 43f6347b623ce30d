// GEMM tile family instantiations (see net_gemm_kernel.hpp); one
// translation unit per family so hipcc compiles them in parallel.
#include "net_gemm_kernel.hpp"

namespace s3gemm {
// v_mfma_f32_16x16x32 tiles: 4 waves (2 x 2), one large tile per CU (wave
// tiles 32x80, 48x32, 64x48, 80x64, 128x64): the decomposition hipBLASLt
// picks for the network's M = 768 shapes on gfx950.  A 16x16 tile needs the vector
// epilogue (aligned operands).
int launch_t4(int tile, const GemmP& p, hipStream_t st) {
  if (tile < 21 || tile > 25) return kNotMine;
  // no silent fallback to another tile: that would change the launch's
  // reduction class (ops.reduction_class); the tuner skips the error
  S3_REQUIRE(p.vec_epi, "s3n_gemm: 16x16 MFMA tiles need the vector epilogue");
  if (tile == 21) return launch<64, 160, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 22) return launch<96, 64, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 23) return launch<128, 96, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 24) return launch<160, 128, 3, 2, 2, 64, 1, 16>(p, st);
  return launch<256, 128, 3, 2, 2, 64, 1, 16>(p, st);
}
int sat_t4(int reset) { return read_sat(reset); }
}  // namespace s3gemm
