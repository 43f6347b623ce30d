// Sim3 / SO3 math shared by the device kernels (sim3.hip, tracker.hip) and
// the host single-pose helpers.  Restated from
// splatt3r_slam/backend/src/gn_kernels.cu:171-412 (itself DROID-SLAM /
// lietorch derived).  Element layout: t(3) q(xyzw,4) s(1).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#define S3_HD __host__ __device__ __forceinline__

namespace s3lie {

constexpr float kEps = 1e-6f;  // gn_kernels.cu:33 (#define EPS 1e-6)

// out = qi * qj  (gn_kernels.cu:177-184 quat_comp)
S3_HD void quat_comp(const float* qi, const float* qj, float* out) {
  float o0 = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  float o1 = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  float o2 = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  float o3 = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
  out[0] = o0; out[1] = o1; out[2] = o2; out[3] = o3;
}

// gn_kernels.cu:187-193 quat_inv
S3_HD void quat_inv(const float* q, float* out) {
  out[0] = -q[0]; out[1] = -q[1]; out[2] = -q[2]; out[3] = q[3];
}

// Y = R(q) X  (gn_kernels.cu:195-205 actSO3; Eigen _transformVector form).
// Safe for Y == X.
S3_HD void act_so3(const float* q, const float* X, float* Y) {
  float uv0 = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  float uv1 = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  float uv2 = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  float y0 = X[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  float y1 = X[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  float y2 = X[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
  Y[0] = y0; Y[1] = y1; Y[2] = y2;
}

// Y = s R X + t  (gn_kernels.cu:207-220 actSim3)
S3_HD void act_sim3(const float* T, const float* X, float* Y) {
  act_so3(T + 3, X, Y);
  Y[0] = Y[0] * T[7] + T[0];
  Y[1] = Y[1] * T[7] + T[1];
  Y[2] = Y[2] * T[7] + T[2];
}

// Normalise a quaternion in place (lietorch SO3/RxSO3 constructors normalise).
S3_HD void quat_normalize(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  float inv = 1.0f / n;
  q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
}

// out = a * b  ((t1,q1,s1)(t2,q2,s2) = (t1 + s1 R1 t2, q1 q2, s1 s2))
S3_HD void mul_sim3(const float* a, const float* b, float* out) {
  float t[3], q[4];
  act_so3(a + 3, b, t);
  t[0] = t[0] * a[7] + a[0];
  t[1] = t[1] * a[7] + a[1];
  t[2] = t[2] * a[7] + a[2];
  quat_comp(a + 3, b + 3, q);
  quat_normalize(q);
  float s = a[7] * b[7];
  out[0] = t[0]; out[1] = t[1]; out[2] = t[2];
  out[3] = q[0]; out[4] = q[1]; out[5] = q[2]; out[6] = q[3];
  out[7] = s;
}

// out = a^-1 = (-(1/s) R^T t, q^-1, 1/s)
S3_HD void inv_sim3(const float* a, float* out) {
  float qi[4], t[3];
  quat_inv(a + 3, qi);
  float sinv = 1.0f / a[7];
  act_so3(qi, a, t);
  out[0] = -sinv * t[0]; out[1] = -sinv * t[1]; out[2] = -sinv * t[2];
  out[3] = qi[0]; out[4] = qi[1]; out[5] = qi[2]; out[6] = qi[3];
  out[7] = sinv;
}

// gn_kernels.cu:297-317 expSO3
S3_HD void exp_so3(const float* phi, float* q) {
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float imag, real;
  if (theta_sq < kEps) {
    float theta_p4 = theta_sq * theta_sq;
    imag = (float)(0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4);
    real = (float)(1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4);
  } else {
    float theta = sqrtf(theta_sq);
    imag = sinf(0.5f * theta) / theta;
    real = cosf(0.5f * theta);
  }
  q[0] = imag * phi[0]; q[1] = imag * phi[1]; q[2] = imag * phi[2]; q[3] = real;
}

// Coefficients of W = C I + A [phi]x + B [phi]x^2 (gn_kernels.cu:339-371).
S3_HD void sim3_w_coeffs(float theta_sq, float sigma, float scale, float* A,
                         float* B, float* C) {
  float theta = sqrtf(theta_sq);
  const float one = 1.0f, half = 0.5f;
  if (fabsf(sigma) < kEps) {
    *C = one;
    if (fabsf(theta) < kEps) {
      *A = half;
      *B = (float)(1.0 / 6.0);
    } else {
      *A = (one - cosf(theta)) / theta_sq;
      *B = (theta - sinf(theta)) / (theta_sq * theta);
    }
  } else {
    *C = (scale - one) / sigma;
    if (fabsf(theta) < kEps) {
      float sigma_sq = sigma * sigma;
      *A = ((sigma - one) * scale + one) / sigma_sq;
      *B = (scale * half * sigma_sq + scale - one - sigma * scale) / (sigma_sq * sigma);
    } else {
      float a = scale * sinf(theta);
      float b = scale * cosf(theta);
      float c = theta_sq + sigma * sigma;
      *A = (a * sigma + (one - b) * theta) / (theta * c);
      *B = (*C - ((b - one) * sigma + a * theta) / c) / theta_sq;
    }
  }
}

S3_HD void cross3(const float* a, const float* b, float* o) {
  float x = a[1] * b[2] - a[2] * b[1];
  float y = a[2] * b[0] - a[0] * b[2];
  float z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

// out = Exp(xi), xi = (tau, phi, sigma)  (gn_kernels.cu:319-391 expSim3)
S3_HD void exp_sim3(const float* xi, float* out) {
  float tau[3] = {xi[0], xi[1], xi[2]};
  float phi[3] = {xi[3], xi[4], xi[5]};
  float sigma = xi[6];
  float scale = expf(sigma);
  float q[4];
  exp_so3(phi, q);
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float A, B, C;
  sim3_w_coeffs(theta_sq, sigma, scale, &A, &B, &C);
  float t[3] = {C * tau[0], C * tau[1], C * tau[2]};
  cross3(phi, tau, tau);
  t[0] += A * tau[0]; t[1] += A * tau[1]; t[2] += A * tau[2];
  cross3(phi, tau, tau);
  t[0] += B * tau[0]; t[1] += B * tau[1]; t[2] += B * tau[2];
  out[0] = t[0]; out[1] = t[1]; out[2] = t[2];
  out[3] = q[0]; out[4] = q[1]; out[5] = q[2]; out[6] = q[3];
  out[7] = scale;
}

// out = Exp(xi) * T  (gn_kernels.cu:393-412 retrSim3; left composition).
// The quaternion is not re-normalised, as in the source.
S3_HD void retr_sim3(const float* T, const float* xi, float* out) {
  float d[8];
  exp_sim3(xi, d);
  float q1[4], t1[3];
  quat_comp(d + 3, T + 3, q1);
  act_so3(d + 3, T, t1);
  t1[0] = t1[0] * d[7] + d[0];
  t1[1] = t1[1] * d[7] + d[1];
  t1[2] = t1[2] * d[7] + d[2];
  out[0] = t1[0]; out[1] = t1[1]; out[2] = t1[2];
  out[3] = q1[0]; out[4] = q1[1]; out[5] = q1[2]; out[6] = q1[3];
  out[7] = d[7] * T[7];
}

// lietorch SO3::Log (two_atan_nbyw_by_n form).
S3_HD void log_so3(const float* q, float* phi) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  float w = q[3];
  float f;
  if (n < kEps) {
    f = 2.0f / w - (2.0f / 3.0f) * (n * n) / (w * w * w);
  } else if (fabsf(w) < kEps) {
    f = (w > 0.0f ? 3.14159265358979323846f : -3.14159265358979323846f) / n;
  } else {
    f = 2.0f * atanf(n / w) / n;
  }
  phi[0] = f * q[0]; phi[1] = f * q[1]; phi[2] = f * q[2];
}

// xi = Log(T): phi = Log(q), sigma = log(s), tau = W(phi, sigma)^-1 t.
S3_HD void log_sim3(const float* T, float* xi) {
  float phi[3];
  log_so3(T + 3, phi);
  float sigma = logf(T[7]);
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float A, B, C;
  sim3_w_coeffs(theta_sq, sigma, T[7], &A, &B, &C);
  // W = C I + A K + B K^2, K = [phi]x ; K^2 = phi phi^T - theta^2 I
  float K[9] = {0.f, -phi[2], phi[1], phi[2], 0.f, -phi[0], -phi[1], phi[0], 0.f};
  float W[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      float k2 = phi[r] * phi[c] - (r == c ? theta_sq : 0.0f);
      W[3 * r + c] = (r == c ? C : 0.0f) + A * K[3 * r + c] + B * k2;
    }
  // Solve W tau = t by the adjugate (W is well conditioned: det > 0).
  float c00 = W[4] * W[8] - W[5] * W[7];
  float c01 = W[5] * W[6] - W[3] * W[8];
  float c02 = W[3] * W[7] - W[4] * W[6];
  float det = W[0] * c00 + W[1] * c01 + W[2] * c02;
  float idet = 1.0f / det;
  float inv[9] = {c00 * idet, (W[2] * W[7] - W[1] * W[8]) * idet, (W[1] * W[5] - W[2] * W[4]) * idet,
                  c01 * idet, (W[0] * W[8] - W[2] * W[6]) * idet, (W[2] * W[3] - W[0] * W[5]) * idet,
                  c02 * idet, (W[1] * W[6] - W[0] * W[7]) * idet, (W[0] * W[4] - W[1] * W[3]) * idet};
  for (int r = 0; r < 3; ++r)
    xi[r] = inv[3 * r] * T[0] + inv[3 * r + 1] * T[1] + inv[3 * r + 2] * T[2];
  xi[3] = phi[0]; xi[4] = phi[1]; xi[5] = phi[2]; xi[6] = sigma;
}

// Row-major 3x3 rotation of a unit quaternion (Eigen toRotationMatrix form).
S3_HD void quat_to_rot(const float* q, float* R) {
  float tx = 2.0f * q[0], ty = 2.0f * q[1], tz = 2.0f * q[2];
  float twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
  float txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
  float tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
  R[0] = 1.0f - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1.0f - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1.0f - (txx + tyy);
}

}  // namespace s3lie
