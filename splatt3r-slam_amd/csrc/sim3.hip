// Sim3 / SE3 group kernels behind include/s3lie.h (lietorch replacement).
// One thread per group element; all element math lives in sim3_math.hpp.
#include "common.hpp"
#include "s3lie.h"
#include "sim3_math.hpp"

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n) { return (int)s3::cdiv(n, kBlock); }

__global__ void k_mul(const float* __restrict__ a, int64_t n_a,
                      const float* __restrict__ b, int64_t n_b,
                      float* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float A[8], B[8], O[8];
  const float* pa = a + (n_a == 1 ? 0 : i) * 8;
  const float* pb = b + (n_b == 1 ? 0 : i) * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) { A[k] = pa[k]; B[k] = pb[k]; }
  s3lie::mul_sim3(A, B, O);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = O[k];
}

__global__ void k_inv(const float* __restrict__ a, float* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float A[8], O[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) A[k] = a[i * 8 + k];
  s3lie::inv_sim3(A, O);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = O[k];
}

// Point action: the group element is broadcast when n_T == 1 (the tracker
// case: one pose acting on h*w points), so it is loaded once per thread from
// a uniform address (scalar cache).
__global__ void k_act(const float* __restrict__ T, int64_t n_T,
                      const float* __restrict__ X, float* __restrict__ Y, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float G[8];
  const float* pt = T + (n_T == 1 ? 0 : i) * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) G[k] = pt[k];
  float x[3] = {X[i * 3 + 0], X[i * 3 + 1], X[i * 3 + 2]};
  float y[3];
  s3lie::act_sim3(G, x, y);
  Y[i * 3 + 0] = y[0]; Y[i * 3 + 1] = y[1]; Y[i * 3 + 2] = y[2];
}

__global__ void k_exp(const float* __restrict__ xi, float* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[7], O[8];
#pragma unroll
  for (int k = 0; k < 7; ++k) x[k] = xi[i * 7 + k];
  s3lie::exp_sim3(x, O);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = O[k];
}

__global__ void k_log(const float* __restrict__ T, float* __restrict__ xi, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float G[8], x[7];
#pragma unroll
  for (int k = 0; k < 8; ++k) G[k] = T[i * 8 + k];
  s3lie::log_sim3(G, x);
#pragma unroll
  for (int k = 0; k < 7; ++k) xi[i * 7 + k] = x[k];
}

__global__ void k_retr(const float* __restrict__ T, int64_t n_T,
                       const float* __restrict__ xi, int64_t n_xi,
                       float* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float G[8], x[7], O[8];
  const float* pt = T + (n_T == 1 ? 0 : i) * 8;
  const float* px = xi + (n_xi == 1 ? 0 : i) * 7;
#pragma unroll
  for (int k = 0; k < 8; ++k) G[k] = pt[k];
#pragma unroll
  for (int k = 0; k < 7; ++k) x[k] = px[k];
  s3lie::retr_sim3(G, x, O);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = O[k];
}

template <bool kSim3>
__global__ void k_matrix(const float* __restrict__ T, float* __restrict__ M, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int D = kSim3 ? 8 : 7;
  const float* p = T + i * D;
  float q[4] = {p[3], p[4], p[5], p[6]};
  float R[9];
  s3lie::quat_to_rot(q, R);
  float s = kSim3 ? p[7] : 1.0f;
  float* m = M + i * 16;
  for (int r = 0; r < 3; ++r) {
    m[4 * r + 0] = R[3 * r + 0] * s;
    m[4 * r + 1] = R[3 * r + 1] * s;
    m[4 * r + 2] = R[3 * r + 2] * s;
    m[4 * r + 3] = p[r];
  }
  m[12] = 0.f; m[13] = 0.f; m[14] = 0.f; m[15] = 1.f;
}

// gn_kernels.cu:414-452: one block walks the poses; dx is indexed k-num_fix.
__global__ void k_pose_retr(float* __restrict__ poses, const float* __restrict__ dx,
                            int64_t num_poses, int64_t num_fix) {
  for (int64_t k = num_fix + threadIdx.x; k < num_poses; k += blockDim.x) {
    float G[8], x[7], O[8];
    for (int j = 0; j < 8; ++j) G[j] = poses[k * 8 + j];
    for (int j = 0; j < 7; ++j) x[j] = dx[(k - num_fix) * 7 + j];
    s3lie::retr_sim3(G, x, O);
    for (int j = 0; j < 8; ++j) poses[k * 8 + j] = O[j];
  }
}

}  // namespace

extern "C" {

int s3lie_sim3_mul(const float* a, int64_t n_a, const float* b, int64_t n_b,
                   float* out, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0 && (n_a == 1 || n_a == n) && (n_b == 1 || n_b == n),
             "s3lie_sim3_mul: bad broadcast n=%lld n_a=%lld n_b=%lld",
             (long long)n, (long long)n_a, (long long)n_b);
  if (n == 0) return S3_OK;
  k_mul<<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(a, n_a, b, n_b, out, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_sim3_inv(const float* a, float* out, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0, "s3lie_sim3_inv: n < 0");
  if (n == 0) return S3_OK;
  k_inv<<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(a, out, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_sim3_act(const float* T, int64_t n_T, const float* X, float* Y,
                   int64_t n, void* stream) {
  S3_REQUIRE(n >= 0 && (n_T == 1 || n_T == n), "s3lie_sim3_act: bad broadcast");
  if (n == 0) return S3_OK;
  k_act<<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(T, n_T, X, Y, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_sim3_exp(const float* xi, float* out, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0, "s3lie_sim3_exp: n < 0");
  if (n == 0) return S3_OK;
  k_exp<<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(xi, out, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_sim3_log(const float* T, float* xi, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0, "s3lie_sim3_log: n < 0");
  if (n == 0) return S3_OK;
  k_log<<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(T, xi, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_sim3_retr(const float* T, int64_t n_T, const float* xi, int64_t n_xi,
                    float* out, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0 && (n_T == 1 || n_T == n) && (n_xi == 1 || n_xi == n),
             "s3lie_sim3_retr: bad broadcast");
  if (n == 0) return S3_OK;
  k_retr<<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(T, n_T, xi, n_xi, out, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_sim3_matrix(const float* T, float* M, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0, "s3lie_sim3_matrix: n < 0");
  if (n == 0) return S3_OK;
  k_matrix<true><<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(T, M, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_se3_matrix(const float* T, float* M, int64_t n, void* stream) {
  S3_REQUIRE(n >= 0, "s3lie_se3_matrix: n < 0");
  if (n == 0) return S3_OK;
  k_matrix<false><<<grid_for(n), kBlock, 0, s3::as_stream(stream)>>>(T, M, n);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

int s3lie_pose_retr(float* poses, const float* dx, int64_t num_poses,
                    int64_t num_fix, void* stream) {
  S3_REQUIRE(num_poses >= 0 && num_fix >= 0, "s3lie_pose_retr: bad sizes");
  if (num_poses <= num_fix) return S3_OK;
  k_pose_retr<<<1, kBlock, 0, s3::as_stream(stream)>>>(poses, dx, num_poses, num_fix);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

void s3lie_sim3_retr_host(const float T[8], const float xi[7], float out[8]) {
  s3lie::retr_sim3(T, xi, out);
}
void s3lie_sim3_mul_host(const float a[8], const float b[8], float out[8]) {
  s3lie::mul_sim3(a, b, out);
}
void s3lie_sim3_inv_host(const float a[8], float out[8]) { s3lie::inv_sim3(a, out); }

}  // extern "C"
