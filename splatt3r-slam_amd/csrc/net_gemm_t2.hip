// GEMM tile family instantiations (see net_gemm_kernel.hpp); one
// translation unit per family so hipcc compiles them in parallel.
#include "net_gemm_kernel.hpp"

namespace s3gemm {
// 32x32x16 MFMA: large tiles and K tile 128
int launch_t2(int tile, const GemmP& p, hipStream_t st) {
  if (tile == 4) return launch<256, 128, 3, 4, 2>(p, st);
  if (tile == 5) return launch<128, 128, 3, 2, 4>(p, st);
  // K tile 128: half the K iterations (and barriers) per output tile
  if (tile == 9) return launch<64, 64, 3, 2, 2, 128>(p, st);
  if (tile == 10) return launch<64, 64, 2, 2, 2, 128>(p, st);
  if (tile == 11) return launch<64, 128, 2, 2, 2, 128>(p, st);
  if (tile == 12) return launch<128, 128, 2, 2, 2, 128>(p, st);
  // 256x256 output tiles, 8 waves of 128x64 (half the operand bytes per MFMA
  // of 128x128; only 2 stages fit, so it wins only on some large shapes)
  if (tile == 14) return launch<256, 256, 2, 2, 4>(p, st);
  return kNotMine;
}
int sat_t2(int reset) { return read_sat(reset); }
}  // namespace s3gemm
