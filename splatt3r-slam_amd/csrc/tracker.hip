// Fused Gauss-Newton normal equations of the tracker (include/s3t.h).
// One pass over the h*w correspondences per GN iteration: residuals, Huber
// weights, Jacobians and the 7x7 / 7 / 1 reduction all stay in registers;
// block partials are summed in a fixed order in fp64 by a second one-block
// kernel (deterministic).  Replaces ~30 torch kernels plus a cuBLAS A^T A
// per iteration in the reference (tracker.py:156-214).
#include "common.hpp"
#include "s3t.h"
#include "sim3_math.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 1024;
constexpr int NV = 36;  // 28 (H upper) + 7 (g) + 1 (cost)

// Calibrated variant parameters (tracker.py:216-270, geometry.project_calib
// :63-104): K row-major 3x3, image size, pixel border, z_eps (projection
// and keyframe-measurement validity both use it, tracker.py:148-151).
struct CalibP {
  float K[9];
  int h, w;
  float border, z_eps;
};

constexpr int kRayDist = 0, kCalib = 1;

// Per-row accumulation of one whitened residual row into the 36 sums.
__device__ __forceinline__ void accum_row(float* acc, const float* J, float r, float si,
                                          float hk) {
  const float wr = si * r;
  const float aw = fabsf(wr);
  const float hw = aw < hk ? 1.0f : hk / aw;
  const float rob = si * sqrtf(hw);
  const float bb = rob * r;
  float A[7];
#pragma unroll
  for (int c = 0; c < 7; ++c) A[c] = rob * J[c];
  int q = 0;
#pragma unroll
  for (int a = 0; a < 7; ++a)
#pragma unroll
    for (int b = a; b < 7; ++b) acc[q++] += A[a] * A[b];
#pragma unroll
  for (int a = 0; a < 7; ++a) acc[28 + a] -= A[a] * bb;
  acc[35] += 0.5f * bb * bb;
}

// J row = -D [I, -[p]x, p] for one row D (3) of the measurement Jacobian.
__device__ __forceinline__ void jac_row(const float* D, const float* p, float* J) {
  const float nsk[3][3] = {{0.f, p[2], -p[1]}, {-p[2], 0.f, p[0]}, {p[1], -p[0], 0.f}};
#pragma unroll
  for (int c = 0; c < 3; ++c) J[c] = -D[c];
#pragma unroll
  for (int c = 0; c < 3; ++c) J[3 + c] = -(D[0] * nsk[0][c] + D[1] * nsk[1][c] + D[2] * nsk[2][c]);
  J[6] = -(D[0] * p[0] + D[1] * p[1] + D[2] * p[2]);
}

// MODE kRayDist: inv_a = 1/sigma_ray, inv_b = 1/sigma_dist (4 rows / point).
// MODE kCalib:   inv_a = 1/sigma_pixel, inv_b = 1/sigma_depth (3 rows:
// u, v, log z); Xk is the ray-constrained keyframe pointmap, its pixel grid
// and log depth are the measurement (tracker.py:143-151).
template <int MODE>
__global__ void __launch_bounds__(kThreads)
k_normal_eqs(const double* __restrict__ state, const float* __restrict__ Tdev,
             const float* __restrict__ Xf, const float* __restrict__ Xk,
             const float* __restrict__ Q, const uint8_t* __restrict__ valid, int64_t n,
             float inv_a, float inv_b, float hk, CalibP cp, float* __restrict__ partial) {
  if (state && state[2] != 0.0) return;   // the device-side GN loop has finished
  float T[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) T[k] = Tdev[k];
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float x[3] = {Xf[i * 3 + 0], Xf[i * 3 + 1], Xf[i * 3 + 2]};
    float p[3];
    s3lie::act_sim3(T, x, p);
    const float sq = sqrtf(Q[i]);
    const float vv = valid[i] ? 1.0f : 0.0f;
    if constexpr (MODE == kRayDist) {
      const float d = sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
      const float di = 1.0f / d;
      const float rf[3] = {di * p[0], di * p[1], di * p[2]};
      const float xk[3] = {Xk[i * 3 + 0], Xk[i * 3 + 1], Xk[i * 3 + 2]};
      const float dk = sqrtf(xk[0] * xk[0] + xk[1] * xk[1] + xk[2] * xk[2]);
      const float dki = 1.0f / dk;
      float r[4] = {dki * xk[0] - rf[0], dki * xk[1] - rf[1], dki * xk[2] - rf[2], dk - d};
      // drd/dp: rows 0..2 = di (I - di^2 p p^T), row 3 = rf^T
      const float di2 = di * di;
      float Dm[4][3];
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) Dm[a][b] = di * ((a == b ? 1.0f : 0.0f) - di2 * p[a] * p[b]);
      Dm[3][0] = rf[0]; Dm[3][1] = rf[1]; Dm[3][2] = rf[2];
      const float si_r = inv_a * vv * sq, si_d = inv_b * vv * sq;
#pragma unroll
      for (int row = 0; row < 4; ++row) {
        float J[7];
        jac_row(Dm[row], p, J);
        accum_row(acc, J, r[row], row < 3 ? si_r : si_d, hk);
      }
    } else {
      // project_calib: p' = K p, (u, v) = p'.xy / p'.z
      const float* K = cp.K;
      const float q0 = K[0] * p[0] + K[1] * p[1] + K[2] * p[2];
      const float q1 = K[3] * p[0] + K[4] * p[1] + K[5] * p[2];
      const float q2 = K[6] * p[0] + K[7] * p[1] + K[8] * p[2];
      const float u = q0 / q2, v = q1 / q2;
      const bool vz = p[2] > cp.z_eps;
      const bool vproj = (u > cp.border) && (u < (float)(cp.w - 1) - cp.border) &&
                         (v > cp.border) && (v < (float)(cp.h - 1) - cp.border) && vz;
      const float logz = vz ? logf(p[2]) : 0.0f;
      // keyframe measurement: pixel grid + log depth, zeroed where invalid
      const float zk = Xk[i * 3 + 2];
      const bool vmeas = zk > cp.z_eps;
      const int64_t pix_v = i / cp.w, pix_u = i - pix_v * cp.w;
      const float mu = vmeas ? (float)pix_u : 0.f, mv = vmeas ? (float)pix_v : 0.f;
      const float mz = vmeas ? logf(zk) : 0.f;
      const float r[3] = {mu - u, mv - v, mz - logz};
      const float fx = K[0], fy = K[4];
      const float zi = 1.0f / p[2];
      const float Dm[3][3] = {{fx * zi, 0.f, -fx * p[0] * zi * zi},
                              {0.f, fy * zi, -fy * p[1] * zi * zi},
                              {0.f, 0.f, zi}};
      const float v2 = (vproj && vmeas) ? 1.0f : 0.0f;
      const float si_p = v2 * (inv_a * vv * sq), si_z = v2 * (inv_b * vv * sq);
#pragma unroll
      for (int row = 0; row < 3; ++row) {
        float J[7];
        jac_row(Dm[row], p, J);
        accum_row(acc, J, r[row], row < 2 ? si_p : si_z, hk);
      }
    }
  }
  // block reduction: a reduce-scatter across the wave (lane k gets the wave
  // total of sum k), then the 4 wave partials through LDS
  __shared__ float red[4][NV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float wsum = s3::wave_reduce_scatter(acc);
  if (lane < NV) red[wave][lane] = wsum;
  __syncthreads();
  if (threadIdx.x < NV)
    partial[blockIdx.x * NV + threadIdx.x] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// One workgroup per output value; fixed-order fp64 tree (deterministic).
__global__ void __launch_bounds__(kThreads)
k_finalize(const double* __restrict__ state, const float* __restrict__ partial, int nblocks,
           float* __restrict__ out) {
  if (state && state[2] != 0.0) return;
  const int k = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kThreads) s += (double)partial[b * NV + k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double red[kThreads / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[k] = (float)((red[0] + red[1]) + (red[2] + red[3]));
}

// One Gauss-Newton update on the device (tracker.py:156-171 + retr +
// nonlinear_optimizer.check_convergence): fp64 Cholesky of the 7x7 normal
// equations, tau = H^-1 g, T <- Exp(tau) * T, convergence flags.
// state: [0] previous cost (starts +inf), [1] iterations done, [2] flag
// (0 running, 1 converged, 2 Cholesky failed, 3 max iterations), [3] cost.
__global__ void k_gn_solve(const float* __restrict__ out36, float* __restrict__ T,
                           double* __restrict__ state, int max_iters, float rel_error,
                           float delta_norm) {
  if (threadIdx.x != 0 || state[2] != 0.0) return;
  double H[7][7], g[7];
  int q = 0;
  for (int a = 0; a < 7; ++a)
    for (int b = a; b < 7; ++b) H[a][b] = H[b][a] = (double)out36[q++];
  for (int a = 0; a < 7; ++a) g[a] = (double)out36[28 + a];
  const double cost = (double)out36[35];
  // Cholesky H = L L^T (in place, lower)
  for (int j = 0; j < 7; ++j) {
    double d = H[j][j];
    for (int k = 0; k < j; ++k) d -= H[j][k] * H[j][k];
    if (!(d > 0.0) || !isfinite(d)) { state[2] = 2.0; return; }
    const double l = sqrt(d);
    H[j][j] = l;
    for (int i = j + 1; i < 7; ++i) {
      double v = H[i][j];
      for (int k = 0; k < j; ++k) v -= H[i][k] * H[j][k];
      H[i][j] = v / l;
    }
  }
  double y[7], x[7];
  for (int i = 0; i < 7; ++i) {
    double v = g[i];
    for (int k = 0; k < i; ++k) v -= H[i][k] * y[k];
    y[i] = v / H[i][i];
  }
  for (int i = 6; i >= 0; --i) {
    double v = y[i];
    for (int k = i + 1; k < 7; ++k) v -= H[k][i] * x[k];
    x[i] = v / H[i][i];
  }
  float tau[7], Tn[8], Tc[8];
  double nrm = 0.0;
  for (int i = 0; i < 7; ++i) {
    tau[i] = (float)x[i];
    nrm += (double)tau[i] * tau[i];
  }
  for (int k = 0; k < 8; ++k) Tc[k] = T[k];
  s3lie::retr_sim3(Tc, tau, Tn);
  for (int k = 0; k < 8; ++k) T[k] = Tn[k];
  const double old = state[0];
  const double rel = fabs((old - cost) / old);   // nan at the first step, like math.fabs(inf/inf)
  const int it = (int)state[1] + 1;
  state[1] = it;
  state[3] = cost;
  state[0] = cost;
  if (rel < rel_error || sqrt(nrm) < delta_norm) state[2] = 1.0;
  else if (it >= max_iters) state[2] = 3.0;
}

int blocks_for(int64_t n) {
  int64_t b = s3::cdiv(n, kThreads);
  return (int)(b < kMaxBlocks ? (b > 0 ? b : 1) : kMaxBlocks);
}

}  // namespace

extern "C" size_t s3t_workspace_bytes(int64_t n) {
  return sizeof(float) * NV * (size_t)blocks_for(n);
}

extern "C" int s3t_ray_dist_normal_eqs(const float* T, const float* Xf, const float* Xk,
                                       const float* Q, const uint8_t* valid, int64_t n,
                                       float sigma_ray, float sigma_dist, float huber_k,
                                       void* workspace, float* out36, void* stream) {
  S3_REQUIRE(T && n >= 0 && workspace && out36, "s3t_ray_dist_normal_eqs: bad arguments");
  hipStream_t st = s3::as_stream(stream);
  const int nb = blocks_for(n);
  float* partial = static_cast<float*>(workspace);
  // reference: sqrt_info = 1 / sigma * valid * sqrt(Q)  (tracker.py:175-176)
  k_normal_eqs<kRayDist><<<nb, kThreads, 0, st>>>(nullptr, T, Xf, Xk, Q, valid, n,
                                                 1.0f / sigma_ray, 1.0f / sigma_dist, huber_k,
                                                 CalibP{}, partial);
  S3_LAUNCH_CHECK();
  k_finalize<<<NV, kThreads, 0, st>>>(nullptr, partial, nb, out36);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3t_gn_iterations(const float* Xf, const float* Xk, const float* Q,
                                 const uint8_t* valid, int64_t n, float sigma_ray,
                                 float sigma_dist, float huber_k, int iters, int max_iters,
                                 float rel_error, float delta_norm, float* T, double* state,
                                 void* workspace, float* out36, void* stream) {
  S3_REQUIRE(T && state && n >= 0 && workspace && out36 && iters >= 0,
             "s3t_gn_iterations: bad arguments");
  hipStream_t st = s3::as_stream(stream);
  const int nb = blocks_for(n);
  float* partial = static_cast<float*>(workspace);
  for (int i = 0; i < iters; ++i) {
    k_normal_eqs<kRayDist><<<nb, kThreads, 0, st>>>(state, T, Xf, Xk, Q, valid, n,
                                                   1.0f / sigma_ray, 1.0f / sigma_dist, huber_k,
                                                   CalibP{}, partial);
    S3_LAUNCH_CHECK();
    k_finalize<<<NV, kThreads, 0, st>>>(state, partial, nb, out36);
    S3_LAUNCH_CHECK();
    k_gn_solve<<<1, 64, 0, st>>>(out36, T, state, max_iters, rel_error, delta_norm);
    S3_LAUNCH_CHECK();
  }
  return S3_OK;
}

namespace {

int make_calib(const float* K, int h, int w, float pixel_border, float depth_eps, CalibP* cp) {
  S3_REQUIRE(K && h > 0 && w > 0, "s3t calib: K, h > 0, w > 0 required");
  for (int k = 0; k < 9; ++k) cp->K[k] = K[k];
  cp->h = h;
  cp->w = w;
  cp->border = pixel_border;
  cp->z_eps = depth_eps;
  return S3_OK;
}

}  // namespace

extern "C" int s3t_calib_normal_eqs(const float* T, const float* Xf, const float* Xk,
                                    const float* Q, const uint8_t* valid, int64_t n,
                                    const float* K, int h, int w, float pixel_border,
                                    float depth_eps, float sigma_pixel, float sigma_depth,
                                    float huber_k, void* workspace, float* out36, void* stream) {
  S3_REQUIRE(T && n >= 0 && workspace && out36, "s3t_calib_normal_eqs: bad arguments");
  S3_REQUIRE(n == (int64_t)h * w, "s3t_calib_normal_eqs: n must equal h*w (keyframe pixels)");
  CalibP cp;
  if (int e = make_calib(K, h, w, pixel_border, depth_eps, &cp)) return e;
  hipStream_t st = s3::as_stream(stream);
  const int nb = blocks_for(n);
  float* partial = static_cast<float*>(workspace);
  // sqrt_info = 1 / sigma * valid * sqrt(Q), masked by valid_proj & valid_meas (tracker.py:219-240)
  k_normal_eqs<kCalib><<<nb, kThreads, 0, st>>>(nullptr, T, Xf, Xk, Q, valid, n,
                                               1.0f / sigma_pixel, 1.0f / sigma_depth, huber_k,
                                               cp, partial);
  S3_LAUNCH_CHECK();
  k_finalize<<<NV, kThreads, 0, st>>>(nullptr, partial, nb, out36);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

extern "C" int s3t_gn_iterations_calib(const float* Xf, const float* Xk, const float* Q,
                                       const uint8_t* valid, int64_t n, const float* K, int h,
                                       int w, float pixel_border, float depth_eps,
                                       float sigma_pixel, float sigma_depth, float huber_k,
                                       int iters, int max_iters, float rel_error,
                                       float delta_norm, float* T, double* state,
                                       void* workspace, float* out36, void* stream) {
  S3_REQUIRE(T && state && n >= 0 && workspace && out36 && iters >= 0,
             "s3t_gn_iterations_calib: bad arguments");
  S3_REQUIRE(n == (int64_t)h * w, "s3t_gn_iterations_calib: n must equal h*w (keyframe pixels)");
  CalibP cp;
  if (int e = make_calib(K, h, w, pixel_border, depth_eps, &cp)) return e;
  hipStream_t st = s3::as_stream(stream);
  const int nb = blocks_for(n);
  float* partial = static_cast<float*>(workspace);
  for (int i = 0; i < iters; ++i) {
    k_normal_eqs<kCalib><<<nb, kThreads, 0, st>>>(state, T, Xf, Xk, Q, valid, n,
                                                 1.0f / sigma_pixel, 1.0f / sigma_depth,
                                                 huber_k, cp, partial);
    S3_LAUNCH_CHECK();
    k_finalize<<<NV, kThreads, 0, st>>>(state, partial, nb, out36);
    S3_LAUNCH_CHECK();
    k_gn_solve<<<1, 64, 0, st>>>(out36, T, state, max_iters, rel_error, delta_norm);
    S3_LAUNCH_CHECK();
  }
  return S3_OK;
}

// ------------------------------------------------------------ track prep --
// FrameTracker.track's correspondence filter (include/s3t.h s3t_track_prep):
// gathers, the three validity masks and the decision counts in one pass.
// Counts: wave ballots summed over the workgroup in LDS, then one atomic per
// workgroup and count into one of 64 spread slots (slot = workgroup mod 64:
// one address per count took ~9k serialised atomics per frame, ~110 us), and
// k_track_count sums the slots (exact integers, so the result does not depend
// on the order).  Unique hits: the first writer of hit[j] (atomicExch returns
// 0) counts it.  The slots live behind the n hit words.
namespace {

constexpr int kTrackSlots = 64;

__global__ void __launch_bounds__(kThreads)
k_track_prep(const int64_t* __restrict__ idx, const uint8_t* __restrict__ vm,
             const float* __restrict__ Xf, const float* __restrict__ Cf,
             const float* __restrict__ Ck, const float* __restrict__ Qff,
             const float* __restrict__ Qkf, int64_t n, float C_conf, float Q_conf,
             float* __restrict__ Xf_out, float* __restrict__ Q_out,
             uint8_t* __restrict__ valid_opt, uint32_t* __restrict__ hit) {
  __shared__ uint32_t s_cnt[kThreads / 64][3];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool vopt = false, vkf = false, uniq = false;
  if (i < n) {
    const int64_t j = idx[i];
    const bool m = vm[i] != 0;
    Xf_out[i * 3 + 0] = Xf[j * 3 + 0];
    Xf_out[i * 3 + 1] = Xf[j * 3 + 1];
    Xf_out[i * 3 + 2] = Xf[j * 3 + 2];
    const float prod = Qff[j] * Qkf[i];
    const float q = sqrtf(prod);
    Q_out[i] = q;
    const bool vq = q > Q_conf;
    vopt = m && Cf[j] > C_conf && Ck[i] > C_conf && vq;
    vkf = m && vq;
    valid_opt[i] = vopt ? 1 : 0;
    if (m) uniq = atomicExch(&hit[j], 1u) == 0u;
  }
  const int w = threadIdx.x >> 6;
  const unsigned long long b0 = __ballot(vopt), b1 = __ballot(vkf), b2 = __ballot(uniq);
  if ((threadIdx.x & 63) == 0) {
    s_cnt[w][0] = (uint32_t)__popcll(b0);
    s_cnt[w][1] = (uint32_t)__popcll(b1);
    s_cnt[w][2] = (uint32_t)__popcll(b2);
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) t += s_cnt[k][threadIdx.x];
    if (t) atomicAdd(&hit[n + (blockIdx.x % kTrackSlots) * 3 + threadIdx.x], t);
  }
}

// counts[c] = sum of the spread slots of count c (one wave)
__global__ void __launch_bounds__(64)
k_track_count(const uint32_t* __restrict__ slots, int64_t* __restrict__ counts) {
  const int lane = threadIdx.x;
  for (int c = 0; c < 3; ++c) {
    unsigned long long v = slots[lane * 3 + c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) counts[c] = (int64_t)v;
  }
}

}  // namespace

extern "C" int s3t_track_prep(const int64_t* idx, const uint8_t* vm, const float* Xf,
                              const float* Cf, const float* Ck, const float* Qff,
                              const float* Qkf, int64_t n, float C_conf, float Q_conf,
                              float* Xf_out, float* Q_out, uint8_t* valid_opt, uint32_t* hit,
                              int64_t* counts, void* stream) {
  S3_REQUIRE(n >= 0, "s3t_track_prep: bad n");
  S3_REQUIRE(hit && counts, "s3t_track_prep: null scratch / counts");
  S3_REQUIRE(n == 0 || (idx && vm && Xf && Cf && Ck && Qff && Qkf && Xf_out && Q_out &&
                        valid_opt),
             "s3t_track_prep: null operand");
  hipStream_t st = s3::as_stream(stream);
  // the hit flags and the count slots behind them, zeroed in one fill
  S3_HIP(hipMemsetAsync(hit, 0, ((size_t)n + kTrackSlots * 3) * sizeof(uint32_t), st));
  if (n > 0) {
    k_track_prep<<<(unsigned)s3::cdiv(n, kThreads), kThreads, 0, st>>>(
        idx, vm, Xf, Cf, Ck, Qff, Qkf, n, C_conf, Q_conf, Xf_out, Q_out, valid_opt, hit);
    S3_LAUNCH_CHECK();
  }
  k_track_count<<<1, 64, 0, st>>>(hit + n, counts);
  S3_LAUNCH_CHECK();
  return S3_OK;
}
