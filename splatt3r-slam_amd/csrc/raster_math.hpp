// Per-Gaussian math of the tile rasterizer, shared by the forward and the
// backward kernels (raster.hip).  Canonical graphdeco 3DGS formulas written
// in explicit row-major form; compiled with -ffp-contract=off and with a
// fixed-sequence exponential so the forward is reproducible operation by
// operation by the CPU oracle (oracle/raster_ref.c).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#define GSR_HD __host__ __device__ __forceinline__

namespace gsr {

constexpr int BX = 16, BY = 16, BS = BX * BY;  // 16x16 pixel tiles, 256 threads

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f,
                SH_C2_2 = 0.31539156525252005f, SH_C2_3 = -1.0925484305920792f,
                SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f,
                SH_C3_2 = -0.4570457994644658f, SH_C3_3 = 0.3731763325901154f,
                SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;

// exp(x) by Cody-Waite reduction + degree-6 Taylor/Horner, <= 3 ulp from the
// correctly rounded exp on the blend's domain [-87, 0] (measured by
// tests/test_raster.py test_oracle_fexp_ulp_bound).  A fixed operation sequence (no libm / ocml) so
// the GPU forward and the CPU oracle agree bit for bit.
GSR_HD float fexp(float x) {
  if (x < -87.0f) return 0.0f;
  float k = rintf(x * 1.44269504088896341f);
  float r = x - k * 0.693145751953125f;
  r = r - k * 1.42860682030941723e-06f;
  float p = 0.00138888888888889f;
  p = p * r + 0.00833333333333333f;
  p = p * r + 0.0416666666666667f;
  p = p * r + 0.166666666666667f;
  p = p * r + 0.5f;
  p = p * r + 1.0f;
  p = p * r + 1.0f;
  return ldexpf(p, (int)k);
}

GSR_HD float ndc2pix(float v, int S) { return ((v + 1.0f) * S - 1.0f) * 0.5f; }

// Tile rectangle of a splat (reference getRect, int radius).
GSR_HD void get_rect(float px, float py, int r, int gx, int gy, int* xmin, int* ymin,
                     int* xmax, int* ymax) {
  int a = (int)((px - r) / BX), b = (int)((py - r) / BY);
  int c = (int)((px + r + BX - 1) / BX), d = (int)((py + r + BY - 1) / BY);
  *xmin = a < 0 ? 0 : (a > gx ? gx : a);
  *ymin = b < 0 ? 0 : (b > gy ? gy : b);
  *xmax = c < 0 ? 0 : (c > gx ? gx : c);
  *ymax = d < 0 ? 0 : (d > gy ? gy : d);
}

// Conservative tile culling.  A (Gaussian, tile) pair may be dropped only
// when the blend skips the Gaussian at EVERY pixel of the tile, i.e.
// o * exp(power) < 1/255 there (the reference's own per-pixel skip), with
// power = -q/2, q = A dx^2 + 2B dx dy + C dy^2 (conic A, B, C).  Keeping a
// pair is always safe, so every approximation below errs towards keeping:
//  * thr = 2 ln(255 o) + 0.05: keep iff q_min <= thr (0.05 = 5 % in alpha,
//    far above fexp's 2 ulp);
//  * the blend's fp32 q is off by at most ~1e-6 (A dx^2 + C dy^2) <=
//    1e-6 q / (1 - rho), rho = |B| / sqrt(AC); this test's own fp32 q_min
//    has the same order of error, so q_min is scaled down by
//    1e-4 / (1 - rho) (50x the sum) before comparing; rho >= 0.99 keeps all;
//  * q_min is taken over the continuous pixel rectangle of the tile (a
//    superset of its pixel centres): 0 if the mean lies inside, else the
//    least of the four clamped edge minima;
//  * the tiles tested are those of the reference rect that meet the
//    ellipse's bounding box q <= thr / shrink (half-widths
//    sqrt(t C / det), sqrt(t A / det)).
// A dropped pair therefore contributes nothing at any pixel: image, final_T
// and gradients stay bit-identical; only num_rendered shrinks.
struct TileCull {
  float thr, shrink, inv_a, inv_c;
  int mode;   // 0 = test tiles, 1 = keep every rect tile, 2 = drop all
  int x0, y0, x1, y1;   // candidate tile rect (subset of the reference rect)
};

GSR_HD TileCull tile_cull(float mx, float my, float A, float B, float C, float o, int rx0,
                          int ry0, int rx1, int ry1) {
  TileCull t;
  t.x0 = rx0; t.y0 = ry0; t.x1 = rx1; t.y1 = ry1;
  t.thr = 0.0f; t.shrink = 1.0f; t.mode = 1;
  t.inv_a = 0.0f; t.inv_c = 0.0f;
  if (!(A > 0.0f) || !(C > 0.0f) || !(o > 0.0f)) return t;
  const float rho = fabsf(B) / sqrtf(A * C);
  if (!(rho < 0.99f)) return t;
  const float thr = 2.0f * logf(255.0f * o) + 0.05f;
  if (thr < 0.0f) { t.mode = 2; return t; }   // o < ~1/262: never blended
  t.mode = 0;
  t.thr = thr;
  // reciprocals for the edge minimisers: an inexact minimiser location
  // changes q only to second order (C dv^2), far inside the 0.05 margin
  t.inv_a = 1.0f / A;
  t.inv_c = 1.0f / C;
  t.shrink = 1.0f - 1e-4f / (1.0f - rho);
  const float det = A * C - B * B;
  const float tt = thr / t.shrink * 1.001f;
  const float hx = sqrtf(tt * C / det) + 1.0f, hy = sqrtf(tt * A / det) + 1.0f;
  const int bx0 = (int)floorf((mx - hx) / BX), bx1 = (int)floorf((mx + hx) / BX) + 1;
  const int by0 = (int)floorf((my - hy) / BY), by1 = (int)floorf((my + hy) / BY) + 1;
  t.x0 = bx0 > rx0 ? bx0 : rx0;
  t.x1 = bx1 < rx1 ? bx1 : rx1;
  t.y0 = by0 > ry0 ? by0 : ry0;
  t.y1 = by1 < ry1 ? by1 : ry1;
  if (t.x1 < t.x0) t.x1 = t.x0;
  if (t.y1 < t.y0) t.y1 = t.y0;
  return t;
}

GSR_HD bool tile_hit(const TileCull& t, float mx, float my, float A, float B, float C, int tx,
                     int ty, int W, int H) {
  if (t.mode != 0) return t.mode == 1;
  const float x0 = (float)(tx * BX), y0 = (float)(ty * BY);
  const float x1 = fminf(x0 + (BX - 1), (float)(W - 1)), y1 = fminf(y0 + (BY - 1), (float)(H - 1));
  // d = mean - pixel over [mx - x1, mx - x0] x [my - y1, my - y0]
  const float ux0 = mx - x1, ux1 = mx - x0, vy0 = my - y1, vy1 = my - y0;
  if (ux0 <= 0.0f && ux1 >= 0.0f && vy0 <= 0.0f && vy1 >= 0.0f) return true;
  float qmin = 3.0e38f;
  const float ux[2] = {ux0, ux1}, vy[2] = {vy0, vy1};
  for (int e = 0; e < 2; ++e) {
    const float u = ux[e];
    const float v = fminf(fmaxf(-B * u * t.inv_c, vy0), vy1);
    qmin = fminf(qmin, A * u * u + 2.0f * B * u * v + C * v * v);
    const float w = vy[e];
    const float x = fminf(fmaxf(-B * w * t.inv_a, ux0), ux1);
    qmin = fminf(qmin, A * x * x + 2.0f * B * x * w + C * w * w);
  }
  return qmin * t.shrink <= t.thr;
}

// Kept-tile mask of a reference rect of <= 64 tiles (bit (ty - ry0) * rw +
// (tx - rx0)), one tile row at a time instead of tile_hit per tile.  Over
// a row's v band (v = my - y, y in the row's continuous pixel range) the
// ellipse q <= T covers one u interval [umin, umax] (u = mx - x): the slice
// at v spans u = (-B v -+ sqrt(A T - det v^2)) / A, the right end concave
// and the left end convex in v, so their extremes over the band sit at the
// tangent points v = -/+ B sqrt(T / (C det)) clamped into it.  A tile of
// the row meets the ellipse iff its u range meets [umin, umax], i.e. its
// columns form one run.  Same criterion as tile_hit (q_min over the tile's
// continuous rect <= thr / shrink), with T inflated by 1e-3 and the run
// widened by 0.01 px against rounding (keeping a tile is always safe; the
// last column is not clipped to W - 1, which only keeps more).
// tests/test_raster.py checks the mask holds every tile tile_hit keeps.
GSR_HD uint64_t tile_mask_rows(const TileCull& t, float mx, float my, float A, float B, float C,
                               int rx0, int ry0, int rw, int rh, int H) {
  const int area = rw * rh;
  const uint64_t all = area >= 64 ? ~0ull : (1ull << area) - 1ull;
  if (t.mode == 1) return all;
  if (t.mode == 2) return 0ull;
  const float T = t.thr / t.shrink * 1.001f;
  const float det = A * C - B * B;   // > 0: rho < 0.99 in mode 0
  const float vm = sqrtf(T * A / det);          // |v| reach of the ellipse
  const float vs = B * sqrtf(T / (C * det));    // v of the leftmost point
  const float AT = A * T;
  uint64_t mask = 0ull;
  for (int ty = t.y0; ty < t.y1; ++ty) {
    const float yt0 = (float)(ty * BY), yt1 = fminf(yt0 + (BY - 1), (float)(H - 1));
    const float vb0 = fmaxf(my - yt1, -vm), vb1 = fminf(my - yt0, vm);
    if (vb0 > vb1) continue;
    const float vr = fminf(fmaxf(-vs, vb0), vb1), vl = fminf(fmaxf(vs, vb0), vb1);
    const float umax = (-B * vr + sqrtf(fmaxf(AT - det * vr * vr, 0.0f))) * t.inv_a;
    const float umin = (-B * vl - sqrtf(fmaxf(AT - det * vl * vl, 0.0f))) * t.inv_a;
    // tiles tx with 16 tx <= mx - umin and 16 tx + 15 >= mx - umax
    int c0 = (int)ceilf((mx - umax - 0.01f - (float)(BX - 1)) * (1.0f / BX));
    int c1 = (int)floorf((mx - umin + 0.01f) * (1.0f / BX));
    c0 = c0 > t.x0 ? c0 : t.x0;
    c1 = c1 < t.x1 - 1 ? c1 : t.x1 - 1;
    if (c0 > c1) continue;
    const int n = c1 - c0 + 1;
    mask |= (n >= 64 ? ~0ull : (1ull << n) - 1ull) << ((ty - ry0) * rw + (c0 - rx0));
  }
  return mask;
}

// p (3) through a column-major 4x4 stored as the reference passes it.
GSR_HD void xform43(const float* m, float x, float y, float z, float* o) {
  o[0] = m[0] * x + m[4] * y + m[8] * z + m[12];
  o[1] = m[1] * x + m[5] * y + m[9] * z + m[13];
  o[2] = m[2] * x + m[6] * y + m[10] * z + m[14];
}
GSR_HD void xform44(const float* m, float x, float y, float z, float* o) {
  xform43(m, x, y, z, o);
  o[3] = m[3] * x + m[7] * y + m[11] * z + m[15];
}

// 3-D covariance from scale (x modifier) and unit quaternion (r, x, y, z):
// Sigma = R S S^T R^T, upper triangle (xx, xy, xz, yy, yz, zz).
GSR_HD void cov3d_from_scale_rot(const float* s3, float mod, const float* q, float* cov) {
  float r = q[0], x = q[1], y = q[2], z = q[3];
  float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
  float s[3] = {mod * s3[0], mod * s3[1], mod * s3[2]};
  // M = R diag(s); Sigma = M M^T
  float M[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[3 * i + j] = R[3 * i + j] * s[j];
  int k = 0;
  for (int i = 0; i < 3; ++i)
    for (int j = i; j < 3; ++j)
      cov[k++] = M[3 * i + 0] * M[3 * j + 0] + M[3 * i + 1] * M[3 * j + 1] +
                 M[3 * i + 2] * M[3 * j + 2];
}

// Jacobian-clamped EWA projection: returns T = J Wv (2x3) and the 2-D
// covariance (a, b, c) before the 0.3 low-pass, plus the clamped view point.
struct Ewa {
  float T[6];
  float a, b, c;
  float tx, ty, tz;
  float xmul, ymul;
};

GSR_HD Ewa ewa_project(float mx, float my, float mz, const float* cov3, const float* vm,
                       float fx, float fy, float tanfx, float tanfy) {
  Ewa e;
  float t[3];
  xform43(vm, mx, my, mz, t);
  const float limx = 1.3f * tanfx, limy = 1.3f * tanfy;
  const float txtz = t[0] / t[2], tytz = t[1] / t[2];
  e.xmul = (txtz < -limx || txtz > limx) ? 0.0f : 1.0f;
  e.ymul = (tytz < -limy || tytz > limy) ? 0.0f : 1.0f;
  e.tx = fminf(limx, fmaxf(-limx, txtz)) * t[2];
  e.ty = fminf(limy, fmaxf(-limy, tytz)) * t[2];
  e.tz = t[2];
  const float J00 = fx / e.tz, J02 = -(fx * e.tx) / (e.tz * e.tz);
  const float J11 = fy / e.tz, J12 = -(fy * e.ty) / (e.tz * e.tz);
  // Wv[r][c] = vm[r + 4c]
  for (int c = 0; c < 3; ++c) {
    e.T[c] = J00 * vm[0 + 4 * c] + J02 * vm[2 + 4 * c];
    e.T[3 + c] = J11 * vm[1 + 4 * c] + J12 * vm[2 + 4 * c];
  }
  const float V[9] = {cov3[0], cov3[1], cov3[2], cov3[1], cov3[3], cov3[4],
                      cov3[2], cov3[4], cov3[5]};
  float TV0[3], TV1[3];  // rows of T V
  for (int c = 0; c < 3; ++c) {
    TV0[c] = e.T[0] * V[c] + e.T[1] * V[3 + c] + e.T[2] * V[6 + c];
    TV1[c] = e.T[3] * V[c] + e.T[4] * V[3 + c] + e.T[5] * V[6 + c];
  }
  e.a = TV0[0] * e.T[0] + TV0[1] * e.T[1] + TV0[2] * e.T[2];
  e.b = TV0[0] * e.T[3] + TV0[1] * e.T[4] + TV0[2] * e.T[5];
  e.c = TV1[0] * e.T[3] + TV1[1] * e.T[4] + TV1[2] * e.T[5];
  return e;
}

// View-dependent colour from SH (degree <= 3).  sh points at the M x 3
// coefficients of one Gaussian; dir is the unit view direction.
GSR_HD void sh_basis(int deg, float x, float y, float z, float* B /*16*/) {
  B[0] = SH_C0;
  if (deg > 0) {
    B[1] = -SH_C1 * y; B[2] = SH_C1 * z; B[3] = -SH_C1 * x;
    if (deg > 1) {
      float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      B[4] = SH_C2_0 * xy;
      B[5] = SH_C2_1 * yz;
      B[6] = SH_C2_2 * (2.0f * zz - xx - yy);
      B[7] = SH_C2_3 * xz;
      B[8] = SH_C2_4 * (xx - yy);
      if (deg > 2) {
        B[9] = SH_C3_0 * y * (3.0f * xx - yy);
        B[10] = SH_C3_1 * xy * z;
        B[11] = SH_C3_2 * y * (4.0f * zz - xx - yy);
        B[12] = SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
        B[13] = SH_C3_4 * x * (4.0f * zz - xx - yy);
        B[14] = SH_C3_5 * z * (xx - yy);
        B[15] = SH_C3_6 * x * (xx - 3.0f * yy);
      }
    }
  }
}

// d(basis)/d(x,y,z) for the direction backward (degree <= 3).
GSR_HD void sh_basis_grad(int deg, float x, float y, float z, float* dX, float* dY, float* dZ) {
  for (int i = 0; i < 16; ++i) { dX[i] = 0.f; dY[i] = 0.f; dZ[i] = 0.f; }
  if (deg < 1) return;
  dY[1] = -SH_C1; dZ[2] = SH_C1; dX[3] = -SH_C1;
  if (deg < 2) return;
  float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
  dX[4] = SH_C2_0 * y; dY[4] = SH_C2_0 * x;
  dY[5] = SH_C2_1 * z; dZ[5] = SH_C2_1 * y;
  dX[6] = SH_C2_2 * -2.0f * x; dY[6] = SH_C2_2 * -2.0f * y; dZ[6] = SH_C2_2 * 4.0f * z;
  dX[7] = SH_C2_3 * z; dZ[7] = SH_C2_3 * x;
  dX[8] = SH_C2_4 * 2.0f * x; dY[8] = SH_C2_4 * -2.0f * y;
  if (deg < 3) return;
  dX[9] = SH_C3_0 * 6.0f * xy; dY[9] = SH_C3_0 * 3.0f * (xx - yy);
  dX[10] = SH_C3_1 * yz; dY[10] = SH_C3_1 * xz; dZ[10] = SH_C3_1 * xy;
  dX[11] = SH_C3_2 * -2.0f * xy; dY[11] = SH_C3_2 * (4.0f * zz - xx - 3.0f * yy);
  dZ[11] = SH_C3_2 * 8.0f * yz;
  dX[12] = SH_C3_3 * -6.0f * xz; dY[12] = SH_C3_3 * -6.0f * yz;
  dZ[12] = SH_C3_3 * (6.0f * zz - 3.0f * xx - 3.0f * yy);
  dX[13] = SH_C3_4 * (4.0f * zz - 3.0f * xx - yy); dY[13] = SH_C3_4 * -2.0f * xy;
  dZ[13] = SH_C3_4 * 8.0f * xz;
  dX[14] = SH_C3_5 * 2.0f * xz; dY[14] = SH_C3_5 * -2.0f * yz; dZ[14] = SH_C3_5 * (xx - yy);
  dX[15] = SH_C3_6 * 3.0f * (xx - yy); dY[15] = SH_C3_6 * -6.0f * xy;
}

}  // namespace gsr
