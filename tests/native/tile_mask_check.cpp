// Host check of raster_math.hpp tile_mask_rows against the per-tile test
// tile_hit (tests/test_raster.py test_tile_mask_rows_keeps_every_hit):
// random ellipses and rects of <= 64 tiles; every tile tile_hit keeps must
// be in the row mask.  Prints "<cases> <hit tiles> <row-mask tiles> <misses>".
#include <cstdint>
#include <cstdio>
#include <random>

#include "raster_math.hpp"

using namespace gsr;

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 200000;
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(0.0f, 1.0f);
  const int W = 960, H = 540, gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
  long hits = 0, kept = 0, miss = 0, n = 0;
  while (n < cases) {
    // 2-D covariance from random axes / angle, conic = inverse (+0.3 dilation as the kernel)
    const float s1 = 0.3f + 60.0f * U(rng) * U(rng), s2 = 0.3f + 60.0f * U(rng) * U(rng);
    const float th = 6.2831853f * U(rng), cs = cosf(th), sn = sinf(th);
    const float a = s1 * s1 * cs * cs + s2 * s2 * sn * sn + 0.3f;
    const float b = (s1 * s1 - s2 * s2) * cs * sn;
    const float c = s1 * s1 * sn * sn + s2 * s2 * cs * cs + 0.3f;
    const float det = a * c - b * b;
    if (det == 0.0f) continue;
    const float di = 1.0f / det;
    const float A = c * di, B = -b * di, C = a * di;
    const float o = U(rng) < 0.1f ? 0.004f * U(rng) : U(rng);
    const float mx = -20.0f + (W + 40.0f) * U(rng), my = -20.0f + (H + 40.0f) * U(rng);
    const float mid = 0.5f * (a + c);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const int r = (int)ceilf(3.0f * sqrtf(l1));
    int x0, y0, x1, y1;
    get_rect(mx, my, r, gx, gy, &x0, &y0, &x1, &y1);
    const int rw = x1 - x0, rh = y1 - y0;
    if (rw * rh <= 1 || rw * rh > 64) continue;
    ++n;
    const TileCull tc = tile_cull(mx, my, A, B, C, o, x0, y0, x1, y1);
    uint64_t ref = 0;
    for (int y = tc.y0; y < tc.y1; ++y)
      for (int x = tc.x0; x < tc.x1; ++x)
        if (tile_hit(tc, mx, my, A, B, C, x, y, W, H)) ref |= 1ull << ((y - y0) * rw + (x - x0));
    const uint64_t got = tile_mask_rows(tc, mx, my, A, B, C, x0, y0, rw, rh, H);
    hits += __builtin_popcountll(ref);
    kept += __builtin_popcountll(got);
    miss += __builtin_popcountll(ref & ~got);
  }
  printf("%ld %ld %ld %ld\n", n, hits, kept, miss);
  return 0;
}
