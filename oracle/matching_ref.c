/*
 * ORACLE — test infrastructure only (see oracle/README.md).  CPU restatement
 * of the dense-matching path, used as the parity checker for include/s3m.h.
 *
 * Sources restated:
 *   iter_proj_kernel       splatt3r_slam/backend/src/matching_kernels.cu:118-274
 *   refine_matches_kernel  matching_kernels.cu:24-80
 *   prep_for_iter_proj     splatt3r_slam/matching.py:25-49
 *   img_gradient           splatt3r_slam/image.py:5-38 (Scharr/32, reflect pad)
 *   occlusion check        matching.py:68-76 ; pixel_to_lin matching.py:13-15
 *
 * Arithmetic: strict evaluation of the .cu text (compile with
 * -ffp-contract=off): float ops stay float, sub-expressions written with
 * double literals are evaluated in double.  refine_matches follows c10::Half
 * semantics: product and running sum are each rounded to fp16 (RNE).
 * Initial best score = 0 (cuda::std::numeric_limits<c10::Half>::min() of the
 * unspecialised primary template).
 * Parity vs the CUDA reference binary: UNPINNED (no nvcc here, no reference
 * tests); pinned by the reference-importable img_gradient fixture and by
 * planted-shift / self-match known answers in tests/.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

/* ---- fp16 <-> fp32 (IEEE binary16, round to nearest even) ------------- */
static float h2f(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t man = h & 0x3ff;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else { /* subnormal: value = man * 2^-24 */
      float v = (float)man * 5.9604644775390625e-08f;
      memcpy(&bits, &v, 4);
      bits |= sign;
    }
  } else if (exp == 31) {
    bits = sign | 0x7f800000u | (man << 13);
  } else {
    bits = sign | ((exp + 112) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

static uint16_t f2h(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint32_t sign = (x >> 16) & 0x8000;
  uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00 | (ax > 0x7f800000u ? 0x200 : 0));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00); /* rounds to inf */
  if (ax < 0x38800000u) {                                   /* subnormal or zero */
    /* value / 2^-24 rounded to nearest even integer */
    float af;
    memcpy(&af, &ax, 4);
    double m = (double)af * 16777216.0;
    double r = nearbyint(m); /* default rounding mode: nearest-even */
    return (uint16_t)(sign | (uint32_t)r);
  }
  uint32_t e = ((ax >> 23) - 112) << 10;
  uint32_t m = (ax >> 13) & 0x3ff;
  uint32_t base = e | m;
  uint32_t rem = ax & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (base & 1))) base += 1;
  return (uint16_t)(sign | base);
}

uint16_t oracle_f32_to_f16(float f) { return f2h(f); }
float oracle_f16_to_f32(uint16_t h) { return h2f(h); }

/* ---- iter_proj ---------------------------------------------------------- */
typedef struct {
  const float *r11, *r12, *r21, *r22;
  float w11, w12, w21, w22;
} taps_t;

static taps_t make_taps(const float* img, int w, float u, float v) {
  taps_t t;
  int u11 = (int)floorf(u);
  int v11 = (int)floorf(v);
  float du = u - (float)u11;
  float dv = v - (float)v11;
  t.w11 = du * dv;
  t.w12 = (1.0 - du) * dv;
  t.w21 = du * (1.0 - dv);
  t.w22 = (1.0 - du) * (1.0 - dv);
  t.r11 = &img[((int64_t)(v11 + 1) * w + (u11 + 1)) * 9];
  t.r12 = &img[((int64_t)(v11 + 1) * w + u11) * 9];
  t.r21 = &img[((int64_t)v11 * w + (u11 + 1)) * 9];
  t.r22 = &img[((int64_t)v11 * w + u11) * 9];
  return t;
}

static float lerp_ch(const taps_t* t, int c) {
  return t->w11 * t->r11[c] + t->w12 * t->r12[c] + t->w21 * t->r21[c] + t->w22 * t->r22[c];
}

void oracle_iter_proj(const float* rays_img, const float* pts, const float* p_init,
                      float* p_new, uint8_t* converged_out, int b, int h, int w, int n,
                      int max_iter, float lambda_init, float cost_thresh) {
  /* pixels are independent: OpenMP over them changes no result */
#pragma omp parallel for collapse(2) schedule(static)
  for (int bi = 0; bi < b; ++bi) {
    for (int i = 0; i < n; ++i) {
      const float* img = rays_img + (int64_t)bi * h * w * 9;
      int64_t pi = (int64_t)bi * n + i;
      float u = p_init[pi * 2 + 0], v = p_init[pi * 2 + 1];
      u = clampf(u, 1, w - 2);
      v = clampf(v, 1, h - 2);
      const float* P = pts + pi * 3;
      float lambda = lambda_init;
      uint8_t converged = 0;
      for (int it = 0; it < max_iter; ++it) {
        taps_t t = make_taps(img, w, u, v);
        float r[3], gx[3], gy[3], err[3];
        for (int j = 0; j < 3; ++j) r[j] = lerp_ch(&t, j);
        for (int j = 3; j < 6; ++j) gx[j - 3] = lerp_ch(&t, j);
        for (int j = 6; j < 9; ++j) gy[j - 6] = lerp_ch(&t, j);
        float r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
        float r_norm_inv = 1.0 / r_norm;
        for (int j = 0; j < 3; ++j) r[j] *= r_norm_inv;
        for (int j = 0; j < 3; ++j) err[j] = r[j] - P[j];
        float cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
        float A00 = gx[0] * gx[0] + gx[1] * gx[1] + gx[2] * gx[2];
        float A01 = gx[0] * gy[0] + gx[1] * gy[1] + gx[2] * gy[2];
        float A11 = gy[0] * gy[0] + gy[1] * gy[1] + gy[2] * gy[2];
        float b0 = -(err[0] * gx[0] + err[1] * gx[1] + err[2] * gx[2]);
        float b1 = -(err[0] * gy[0] + err[1] * gy[1] + err[2] * gy[2]);
        A00 += lambda;
        A11 += lambda;
        float det_inv = 1.0 / (A00 * A11 - A01 * A01);
        float delta_u = det_inv * (A11 * b0 - A01 * b1);
        float delta_v = det_inv * (-A01 * b0 + A00 * b1);
        float u_new = u + delta_u;
        float v_new = v + delta_v;
        u_new = clampf(u_new, 1, w - 2);
        v_new = clampf(v_new, 1, h - 2);
        taps_t t2 = make_taps(img, w, u_new, v_new);
        for (int j = 0; j < 3; ++j) r[j] = lerp_ch(&t2, j);
        r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
        r_norm_inv = 1.0 / r_norm;
        for (int j = 0; j < 3; ++j) r[j] *= r_norm_inv;
        for (int j = 0; j < 3; ++j) err[j] = r[j] - P[j];
        float new_cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
        if (new_cost < cost) {
          u = u_new;
          v = v_new;
          lambda *= 0.1;
          converged = new_cost < cost_thresh;
        } else {
          lambda *= 10.0;
          converged = cost < cost_thresh;
        }
      }
      p_new[pi * 2 + 0] = u;
      p_new[pi * 2 + 1] = v;
      converged_out[pi] = converged;
    }
  }
}

/* ---- refine_matches ----------------------------------------------------- */
void oracle_refine_matches(const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                           int64_t* p1_new, int b, int h, int w, int n, int fdim,
                           int radius, int dilation_max) {
#pragma omp parallel for collapse(2) schedule(dynamic, 256)
  for (int bi = 0; bi < b; ++bi) {
    for (int i = 0; i < n; ++i) {
      int64_t pi = (int64_t)bi * n + i;
      int64_t u0 = p1[pi * 2 + 0], v0 = p1[pi * 2 + 1];
      uint16_t max_score = 0; /* Half() == +0 */
      int64_t u_new = u0, v_new = v0;
      for (int d = dilation_max; d > 0; d--) {
        const int rd = radius * d;
        const int diam = 2 * rd + 1;
        for (int ii = 0; ii < diam; ii += d) {
          for (int jj = 0; jj < diam; jj += d) {
            const int64_t u = u0 - rd + ii;
            const int64_t v = v0 - rd + jj;
            if (v >= 0 && v < h && u >= 0 && u < w) {
              uint16_t score = 0;
              const uint16_t* a = D21 + pi * fdim;
              const uint16_t* c = D11 + (((int64_t)bi * h + v) * w + u) * fdim;
              for (int k = 0; k < fdim; k++) {
                uint16_t prod = f2h(h2f(a[k]) * h2f(c[k]));
                score = f2h(h2f(score) + h2f(prod));
              }
              if (h2f(score) > h2f(max_score)) {
                max_score = score;
                u_new = u;
                v_new = v;
              }
            }
          }
        }
        u0 = u_new;
        v0 = v_new;
      }
      p1_new[pi * 2 + 0] = u_new;
      p1_new[pi * 2 + 1] = v_new;
    }
  }
}

/* ---- prep_for_iter_proj + img_gradient ---------------------------------- */
static void normalize3(const float* x, float* o) {
  float nrm = sqrtf(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  float d = fmaxf(nrm, 1e-12f);
  o[0] = x[0] / d; o[1] = x[1] / d; o[2] = x[2] / d;
}

static int reflect(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

void oracle_prep_iter_proj(const float* X11, const float* X21, const int64_t* idx_init,
                           float* rays_out, float* pts_out, float* p_init, int b, int h,
                           int w) {
  const int64_t hw = (int64_t)h * w;
  const float k3 = 3.0f / 32.0f, k10 = 10.0f / 32.0f;
  for (int bi = 0; bi < b; ++bi) {
    const float* X = X11 + (int64_t)bi * hw * 3;
    for (int y = 0; y < h; ++y) {
      for (int x = 0; x < w; ++x) {
        float r[3][3][3];
        for (int dy = 0; dy < 3; ++dy)
          for (int dx = 0; dx < 3; ++dx)
            normalize3(X + ((int64_t)reflect(y + dy - 1, h) * w + reflect(x + dx - 1, w)) * 3,
                       r[dy][dx]);
        int64_t i = (int64_t)y * w + x;
        float* o = rays_out + ((int64_t)bi * hw + i) * 9;
        for (int c = 0; c < 3; ++c) {
          o[c] = r[1][1][c];
          o[3 + c] = -k3 * r[0][0][c] + k3 * r[0][2][c] - k10 * r[1][0][c] +
                     k10 * r[1][2][c] - k3 * r[2][0][c] + k3 * r[2][2][c];
          o[6 + c] = -k3 * r[0][0][c] - k10 * r[0][1][c] - k3 * r[0][2][c] +
                     k3 * r[2][0][c] + k10 * r[2][1][c] + k3 * r[2][2][c];
        }
        normalize3(X21 + ((int64_t)bi * hw + i) * 3, pts_out + ((int64_t)bi * hw + i) * 3);
        int64_t lin = idx_init ? idx_init[(int64_t)bi * hw + i] : i;
        p_init[((int64_t)bi * hw + i) * 2 + 0] = (float)(lin % w);
        p_init[((int64_t)bi * hw + i) * 2 + 1] = (float)(lin / w);
      }
    }
  }
}

void oracle_occlusion(const float* p, const uint8_t* conv, const float* X11, const float* X21,
                      int64_t* p1, uint8_t* valid, int b, int h, int w, float dist_thresh) {
  const int64_t hw = (int64_t)h * w;
  for (int bi = 0; bi < b; ++bi)
    for (int64_t i = 0; i < hw; ++i) {
      int64_t pi = (int64_t)bi * hw + i;
      int64_t u = (int64_t)p[pi * 2 + 0], v = (int64_t)p[pi * 2 + 1];
      p1[pi * 2 + 0] = u;
      p1[pi * 2 + 1] = v;
      const float* a = X11 + ((int64_t)bi * hw + v * w + u) * 3;
      const float* c = X21 + pi * 3;
      float d0 = a[0] - c[0], d1 = a[1] - c[1], d2 = a[2] - c[2];
      float dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
      valid[pi] = (conv[pi] && dist < dist_thresh) ? 1 : 0;
    }
}
