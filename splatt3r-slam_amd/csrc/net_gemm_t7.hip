// GEMM tile family instantiations (see net_gemm_kernel.hpp): 8- and 16-wave
// dense / conv tiles.  The halo-conv measurements (net_gemm_t6.hip) showed
// that at one big-LDS workgroup per CU nothing hides a wave's LDS fragment
// reads and epilogue; these tiles put two waves on every SIMD (8 waves per
// workgroup) or two workgroups on every CU (128x128, 2 stages = 64 KiB).
// (An 8-wave 128x128 32x32x16 tile and a 16-wave 256x256 tile spill at
// these occupancies and are not built.)
#include "net_gemm_kernel.hpp"

namespace s3gemm {
int launch_t7(int tile, const GemmP& p, hipStream_t st) {
  if (tile < 32 || tile > 37 || tile == 33) return kNotMine;
  const bool mf16 = tile == 32 || tile == 36 || tile == 37;
  // no silent fallback to another tile (it would change the reduction class)
  S3_REQUIRE(!mf16 || p.vec_epi, "s3n_gemm: 16x16 MFMA tiles need the vector epilogue");
  if (tile == 32) return launch<128, 128, 2, 2, 4, 64, 1, 16>(p, st);
  if (tile == 34) return launch<256, 128, 2, 4, 2, 64, 1, 32>(p, st);
  if (tile == 35) return launch<128, 256, 2, 2, 4, 64, 1, 32>(p, st);
  if (tile == 36) return launch<256, 128, 3, 4, 2, 64, 1, 16>(p, st);
  // (deep rings of 4-6 stages for the small 1536-row decoder grids were
  // slower on every decoder shape: fewer workgroups per CU hide less of the
  // per-step latency than the extra tiles in flight, profiles/r05c)
  return launch<128, 128, 3, 2, 4, 64, 1, 16>(p, st);
}
int sat_t7(int reset) { return read_sat(reset); }
}  // namespace s3gemm
