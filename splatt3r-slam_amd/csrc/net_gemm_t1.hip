// GEMM tile family instantiations (see net_gemm_kernel.hpp); one
// translation unit per family so hipcc compiles them in parallel.
#include "net_gemm_kernel.hpp"

namespace s3gemm {
// 32x32x16 MFMA tiles with one K-group, and the default / fused-tail choice
int launch_t1(int tile, const GemmP& p, hipStream_t st) {
  if (tile == 1) return launch<64, 64, 3>(p, st);
  if (tile == 2) return launch<64, 128, 3>(p, st);
  if (tile == 3) return launch<128, 128, 2>(p, st);
  if (tile == 6) return launch<64, 64, 4>(p, st);
  if (tile == 7) return launch<64, 64, 5>(p, st);
  if (tile == 8) return launch<64, 128, 4>(p, st);
  if (tile != 0) return kNotMine;
  // the fused tail needs one column tile per row block
  if (p.tail_w[0]) {
    S3_REQUIRE(p.N == 64 || p.N == 128, "s3n_gemm: the fused tail needs N of 64 or 128");
    if (p.N == 128) return launch<64, 128, 3>(p, st);
    return launch<64, 64, 3>(p, st);
  }
  // Tile choice: fill the 256 CUs before growing the tile.
  auto tiles = [&](int bm, int bn) {
    return (int64_t)p.groups * ((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn);
  };
  // LDS: 64x64 x 3 stages = 48 KB (3 WG/CU), 64x128 x 3 = 72 KB (2),
  // 128x128 x 2 = 64 KB (2).  Measured on the network's shapes
  // (tools/bench_gemm.py): 64x64 wins up to ~2k tiles (the 768-token
  // GEMMs), 64x128 beyond (head MLP, DPT convs).
  if (tiles(64, 64) > 2048 && p.N >= 128) return launch<64, 128, 3>(p, st);
  return launch<64, 64, 3>(p, st);
}
int sat_t1(int reset) { return read_sat(reset); }
}  // namespace s3gemm
