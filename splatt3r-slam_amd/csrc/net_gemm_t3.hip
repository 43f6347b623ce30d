// GEMM tile family instantiations (see net_gemm_kernel.hpp); one
// translation unit per family so hipcc compiles them in parallel.
#include "net_gemm_kernel.hpp"

namespace s3gemm {
// in-workgroup split-K: KG groups of 4 waves on one output tile
int launch_t3(int tile, const GemmP& p, hipStream_t st) {
  if (tile == 15) return launch<64, 64, 3, 2, 2, 64, 2>(p, st);
  if (tile == 16) return launch<64, 64, 2, 2, 2, 64, 4>(p, st);
  if (tile == 17) return launch<64, 128, 2, 2, 2, 64, 2>(p, st);
  if (tile == 18) return launch<128, 128, 2, 2, 2, 64, 2>(p, st);
  if (tile == 19) return launch<64, 64, 2, 2, 2, 128, 2>(p, st);
  if (tile == 20) return launch<64, 128, 2, 2, 2, 64, 3>(p, st);
  return kNotMine;
}
int sat_t3(int reset) { return read_sat(reset); }
}  // namespace s3gemm
