/*
 * ORACLE — test infrastructure only.  CPU restatement of the Sim3 group math
 * used as the parity checker for include/s3lie.h.  Nothing in the product
 * path links or calls this file; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load oracle/_build/liboracle.so.
 *
 * Source restated: splatt3r_slam/backend/src/gn_kernels.cu
 *   quat_comp :177-184, quat_inv :187-193, actSO3 :195-205, actSim3 :207-220,
 *   expSO3 :297-317, expSim3 :319-391, retrSim3 :393-412,
 *   pose_retr_kernel :414-452.
 * Group product / inverse follow lietorch's Sim3 (t, q, s) composition rule
 * (external lietorch, unpinned; quaternion re-normalised after products as
 * lietorch's SO3 constructor does).  Parity vs lietorch itself: UNPINNED
 * (submodule absent); pinned instead by group identities in tests/.
 * Compile with -ffp-contract=off (strict evaluation of the source text).
 */
#include <math.h>
#include <stdint.h>

#define EPS 1e-6f

static void quat_comp(const float* qi, const float* qj, float* out) {
  float o0 = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  float o1 = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  float o2 = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  float o3 = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
  out[0] = o0; out[1] = o1; out[2] = o2; out[3] = o3;
}

static void actSO3(const float* q, const float* X, float* Y) {
  float uv[3];
  uv[0] = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  uv[1] = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  uv[2] = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  float y0 = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  float y1 = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  float y2 = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
  Y[0] = y0; Y[1] = y1; Y[2] = y2;
}

void oracle_sim3_act(const float* T, const float* X, float* Y) {
  actSO3(T + 3, X, Y);
  Y[0] *= T[7]; Y[1] *= T[7]; Y[2] *= T[7];
  Y[0] += T[0]; Y[1] += T[1]; Y[2] += T[2];
}

static void normalize_q(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  float inv = 1.0f / n;
  for (int i = 0; i < 4; ++i) q[i] *= inv;
}

void oracle_sim3_mul(const float* a, const float* b, float* out) {
  float t[3], q[4];
  actSO3(a + 3, b, t);
  for (int i = 0; i < 3; ++i) { t[i] *= a[7]; t[i] += a[i]; }
  quat_comp(a + 3, b + 3, q);
  normalize_q(q);
  float s = a[7] * b[7];
  for (int i = 0; i < 3; ++i) out[i] = t[i];
  for (int i = 0; i < 4; ++i) out[3 + i] = q[i];
  out[7] = s;
}

void oracle_sim3_inv(const float* a, float* out) {
  float qi[4] = {-a[3], -a[4], -a[5], a[6]};
  float t[3];
  float sinv = 1.0f / a[7];
  actSO3(qi, a, t);
  for (int i = 0; i < 3; ++i) out[i] = -sinv * t[i];
  for (int i = 0; i < 4; ++i) out[3 + i] = qi[i];
  out[7] = sinv;
}

static void expSO3(const float* phi, float* q) {
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float imag, real;
  if (theta_sq < EPS) {
    float theta_p4 = theta_sq * theta_sq;
    imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4;
    real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4;
  } else {
    float theta = sqrtf(theta_sq);
    imag = sinf(0.5f * theta) / theta;
    real = cosf(0.5f * theta);
  }
  q[0] = imag * phi[0]; q[1] = imag * phi[1]; q[2] = imag * phi[2]; q[3] = real;
}

static void cross_inplace(const float* a, float* b) {
  float x0 = a[1] * b[2] - a[2] * b[1];
  float x1 = a[2] * b[0] - a[0] * b[2];
  float x2 = a[0] * b[1] - a[1] * b[0];
  b[0] = x0; b[1] = x1; b[2] = x2;
}

void oracle_sim3_exp(const float* xi, float* out) {
  float tau[3] = {xi[0], xi[1], xi[2]};
  float phi[3] = {xi[3], xi[4], xi[5]};
  float sigma = xi[6];
  float scale = expf(sigma);
  float q[4];
  expSO3(phi, q);
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta = sqrtf(theta_sq);
  float A, B, C;
  const float one = 1.0f, half = 0.5f;
  if (fabsf(sigma) < EPS) {
    C = one;
    if (fabsf(theta) < EPS) {
      A = half;
      B = 1.0 / 6.0;
    } else {
      A = (one - cosf(theta)) / theta_sq;
      B = (theta - sinf(theta)) / (theta_sq * theta);
    }
  } else {
    C = (scale - one) / sigma;
    if (fabsf(theta) < EPS) {
      float sigma_sq = sigma * sigma;
      A = ((sigma - one) * scale + one) / sigma_sq;
      B = (scale * half * sigma_sq + scale - one - sigma * scale) / (sigma_sq * sigma);
    } else {
      float a = scale * sinf(theta);
      float b = scale * cosf(theta);
      float c = theta_sq + sigma * sigma;
      A = (a * sigma + (one - b) * theta) / (theta * c);
      B = (C - ((b - one) * sigma + a * theta) / (c)) / (theta_sq);
    }
  }
  float t[3] = {C * tau[0], C * tau[1], C * tau[2]};
  cross_inplace(phi, tau);
  t[0] += A * tau[0]; t[1] += A * tau[1]; t[2] += A * tau[2];
  cross_inplace(phi, tau);
  t[0] += B * tau[0]; t[1] += B * tau[1]; t[2] += B * tau[2];
  for (int i = 0; i < 3; ++i) out[i] = t[i];
  for (int i = 0; i < 4; ++i) out[3 + i] = q[i];
  out[7] = scale;
}

void oracle_sim3_retr(const float* T, const float* xi, float* out) {
  float d[8];
  oracle_sim3_exp(xi, d);
  float q1[4], t1[3];
  quat_comp(d + 3, T + 3, q1);
  actSO3(d + 3, T, t1);
  for (int i = 0; i < 3; ++i) { t1[i] *= d[7]; t1[i] += d[i]; }
  for (int i = 0; i < 3; ++i) out[i] = t1[i];
  for (int i = 0; i < 4; ++i) out[3 + i] = q1[i];
  out[7] = d[7] * T[7];
}

/* Batched entry points (n elements, group element broadcast when nT == 1). */
void oracle_sim3_act_batch(const float* T, int64_t nT, const float* X, float* Y, int64_t n) {
  for (int64_t i = 0; i < n; ++i) oracle_sim3_act(T + (nT == 1 ? 0 : i) * 8, X + i * 3, Y + i * 3);
}
void oracle_sim3_mul_batch(const float* a, const float* b, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) oracle_sim3_mul(a + i * 8, b + i * 8, out + i * 8);
}
void oracle_sim3_inv_batch(const float* a, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) oracle_sim3_inv(a + i * 8, out + i * 8);
}
void oracle_sim3_exp_batch(const float* xi, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) oracle_sim3_exp(xi + i * 7, out + i * 8);
}
void oracle_sim3_retr_batch(const float* T, const float* xi, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) oracle_sim3_retr(T + i * 8, xi + i * 7, out + i * 8);
}
void oracle_pose_retr(float* poses, const float* dx, int64_t num_poses, int64_t num_fix) {
  for (int64_t k = num_fix; k < num_poses; ++k) {
    float o[8];
    oracle_sim3_retr(poses + k * 8, dx + (k - num_fix) * 7, o);
    for (int j = 0; j < 8; ++j) poses[k * 8 + j] = o[j];
  }
}
