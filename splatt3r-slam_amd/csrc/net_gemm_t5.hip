// GEMM tile family instantiations (see net_gemm_kernel.hpp); one
// translation unit per family so hipcc compiles them in parallel.
#include "net_gemm_kernel.hpp"

namespace s3gemm {
// v_mfma_f32_16x16x32 tiles, continued
int launch_t5(int tile, const GemmP& p, hipStream_t st) {
  if (tile < 26 || tile > 31) return kNotMine;
  // no silent fallback to another tile: that would change the launch's
  // reduction class (ops.reduction_class); the tuner skips the error
  S3_REQUIRE(p.vec_epi, "s3n_gemm: 16x16 MFMA tiles need the vector epilogue");
  if (tile == 26) return launch<64, 64, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 27) return launch<128, 128, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 28) return launch<64, 128, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 29) return launch<96, 128, 3, 2, 2, 64, 1, 16>(p, st);
  if (tile == 30) return launch<64, 192, 3, 2, 2, 64, 1, 16>(p, st);
  return launch<64, 64, 4, 2, 2, 128, 1, 16>(p, st);
}
int sat_t5(int reset) { return read_sat(reset); }
}  // namespace s3gemm
