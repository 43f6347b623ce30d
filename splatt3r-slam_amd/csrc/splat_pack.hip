// Fused per-view splat packing (include/s3r.h): one lane per splat reads the
// head outputs once (means, scales, rotations, SH residual, opacity, pixel
// colour: 56 B) and writes the rasterizer inputs once (52 B).
#include "common.hpp"
#include "s3r.h"
#include "sim3_math.hpp"

namespace {

constexpr int kThreads = 256;
constexpr float kC0 = 0.28209479177387814f;

__global__ void __launch_bounds__(kThreads)
k_pack(const float* __restrict__ means, const float* __restrict__ scales,
       const float* __restrict__ rots, const float* __restrict__ sh,
       const float* __restrict__ opac, const float* __restrict__ img, int64_t n,
       float s, int chw, float* __restrict__ mo, float* __restrict__ co,
       float* __restrict__ so, float* __restrict__ oo) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  mo[p * 3 + 0] = means[p * 3 + 0] * s;
  mo[p * 3 + 1] = means[p * 3 + 1] * s;
  mo[p * 3 + 2] = means[p * 3 + 2] * s;
  // quaternion_to_matrix (xyzw as (i, j, k, r))
  const float i = rots[p * 4 + 0], j = rots[p * 4 + 1], k = rots[p * 4 + 2], r = rots[p * 4 + 3];
  const float two_s = 2.0f / ((i * i + j * j + k * k + r * r) + 1e-8f);
  const float R[9] = {1.0f - two_s * (j * j + k * k), two_s * (i * j - k * r),
                      two_s * (i * k + j * r),        two_s * (i * j + k * r),
                      1.0f - two_s * (i * i + k * k), two_s * (j * k - i * r),
                      two_s * (i * k - j * r),        two_s * (j * k + i * r),
                      1.0f - two_s * (i * i + j * j)};
  const float sx = scales[p * 3 + 0], sy = scales[p * 3 + 1], sz = scales[p * 3 + 2];
  const float d[3] = {sx * sx, sy * sy, sz * sz};
  const float s2 = s * s;
  int q = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = a; b < 3; ++b) {
      const float v = R[3 * a + 0] * d[0] * R[3 * b + 0] + R[3 * a + 1] * d[1] * R[3 * b + 1] +
                      R[3 * a + 2] * d[2] * R[3 * b + 2];
      co[p * 6 + q++] = v * s2;
    }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float px = chw ? img[(int64_t)c * n + p] : img[p * 3 + c];
    if (chw) px = fminf(fmaxf(px * 0.5f + 0.5f, 0.0f), 1.0f);
    so[p * 3 + c] = sh[p * 3 + c] + (px - 0.5f) / kC0;
  }
  oo[p] = opac[p];
}

__device__ void sim3_mat(const float* T, double* M) {
  float R[9];
  const float q[4] = {T[3], T[4], T[5], T[6]};
  s3lie::quat_to_rot(q, R);
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) M[4 * r + c] = (double)(R[3 * r + c] * T[7]);
    M[4 * r + 3] = (double)T[r];
  }
  M[12] = M[13] = M[14] = 0.0;
  M[15] = 1.0;
}

// Gauss-Jordan inverse with partial pivoting (4x4, fp64).
__device__ void inv4(const double* A, double* out) {
  double m[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      m[r][c] = A[4 * r + c];
      m[r][4 + c] = r == c ? 1.0 : 0.0;
    }
  for (int c = 0; c < 4; ++c) {
    int p = c;
    for (int r = c + 1; r < 4; ++r)
      if (fabs(m[r][c]) > fabs(m[p][c])) p = r;
    if (p != c)
      for (int k = 0; k < 8; ++k) { const double t = m[c][k]; m[c][k] = m[p][k]; m[p][k] = t; }
    const double d = 1.0 / m[c][c];
    for (int k = 0; k < 8; ++k) m[c][k] *= d;
    for (int r = 0; r < 4; ++r)
      if (r != c) {
        const double f = m[r][c];
        for (int k = 0; k < 8; ++k) m[r][k] -= f * m[c][k];
      }
  }
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) out[4 * r + c] = m[r][4 + c];
}

__device__ void mul4(const double* A, const double* B, double* C) {
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s += A[4 * r + k] * B[4 * k + c];
      C[4 * r + c] = s;
    }
}

__global__ void k_camera(const float* __restrict__ Tc, const float* __restrict__ Tt,
                         const float* __restrict__ proj_t, float scale, float* __restrict__ view,
                         float* __restrict__ full, float* __restrict__ campos) {
  if (threadIdx.x != 0) return;
  double Mc[16], Mt[16], Ic[16], E[16], Ie[16], V[16], P[16], F[16];
  sim3_mat(Tc, Mc);
  sim3_mat(Tt, Mt);
  inv4(Mc, Ic);
  mul4(Ic, Mt, E);
  for (int r = 0; r < 3; ++r) E[4 * r + 3] *= (double)scale;
  inv4(E, Ie);
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) V[4 * r + c] = Ie[4 * c + r];
  for (int k = 0; k < 16; ++k) P[k] = (double)proj_t[k];
  mul4(V, P, F);
  for (int k = 0; k < 16; ++k) {
    view[k] = (float)V[k];
    full[k] = (float)F[k];
  }
  for (int r = 0; r < 3; ++r) campos[r] = (float)E[4 * r + 3];
}

}  // namespace

extern "C" int s3r_camera(const float* T_context, const float* T_target, const float* proj_t,
                          float scale, float* view, float* full, float* campos, void* stream) {
  S3_REQUIRE(T_context && T_target && proj_t && view && full && campos, "s3r_camera: null");
  k_camera<<<1, 64, 0, s3::as_stream(stream)>>>(T_context, T_target, proj_t, scale, view, full,
                                                campos);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3r_pack_splats(const float* means, const float* scales, const float* rotations,
                               const float* sh, const float* opacities, const float* img,
                               int64_t n, int d_sh, float scale, int img_chw_normalized,
                               float* means_out, float* cov6_out, float* shs_out,
                               float* opac_out, void* stream) {
  S3_REQUIRE(n >= 0, "s3r_pack_splats: n < 0");
  S3_REQUIRE(d_sh == 1, "s3r_pack_splats: only d_sh == 1 (sh_degree 0) is supported");
  if (n == 0) return S3_OK;
  k_pack<<<(unsigned)s3::cdiv(n, kThreads), kThreads, 0, s3::as_stream(stream)>>>(
      means, scales, rotations, sh, opacities, img, n, scale, img_chw_normalized, means_out,
      cov6_out, shs_out, opac_out);
  S3_LAUNCH_CHECK();
  return S3_OK;
}
