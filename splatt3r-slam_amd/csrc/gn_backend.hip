// Backend pose-graph Gauss-Newton on rays and on calibrated pixel/log-depth
// residuals (include/s3g.h), restating splatt3r_slam/backend/src/
// gn_kernels.cu:812-1227 (ray_align_kernel + gauss_newton_rays_cuda) and
// :1230-1637 (calib_proj_kernel + gauss_newton_calib_cuda) MI355X-first:
//  * an edge's h*w correspondences are split over many workgroups (the
//    reference runs ONE 256-thread block per edge, i.e. a handful of CUs);
//  * the 14-dof Jacobian of an edge is [-Jj, Jj] (ray_align_kernel sets
//    Ji = -Jj after apply_Sim3_adj_inv), so H_e = [[A, -A], [-A, A]] and
//    g_e = [-u, u] with A = sum w Jj^T Jj (28 upper values) and u = sum w r
//    Jj: 35 accumulators per thread instead of 119, same products (a sign
//    flip is exact);
//  * slices are reduced in a fixed order in fp64, the dense 7(N - fix)
//    system is assembled and Cholesky-solved on the device in fp64
//    (replacing the host Eigen SimplicialLLT and the per-iteration
//    device->host copies), then the poses are retracted; a device flag ends
//    the queued iterations once |dx| < delta_thresh.
#include "common.hpp"
#include "s3g.h"
#include "sim3_math.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int NA = 35;   // 28 (A upper, row-major) + 7 (u)

__device__ __forceinline__ float huber_w(float r) {
  const float a = fabsf(r);
  return a < 1.345f ? 1.0f : 1.345f / a;
}

// gn_kernels.cu:251-271 relSim3: T_ij = T_i^-1 T_j
__device__ __forceinline__ void rel_sim3(const float* Ti, const float* Tj, float* Tij) {
  const float si_inv = 1.0f / Ti[7];
  Tij[7] = si_inv * Tj[7];
  float qi_inv[4];
  s3lie::quat_inv(Ti + 3, qi_inv);
  s3lie::quat_comp(qi_inv, Tj + 3, Tij + 3);
  float d[3] = {Tj[0] - Ti[0], Tj[1] - Ti[1], Tj[2] - Ti[2]};
  s3lie::act_so3(qi_inv, d, Tij);
  Tij[0] *= si_inv; Tij[1] *= si_inv; Tij[2] *= si_inv;
}

// gn_kernels.cu:276-296 apply_Sim3_adj_inv (row vector X times Adj^-1)
__device__ __forceinline__ void adj_inv(const float* T, const float* X, float* Y) {
  const float s_inv = 1.0f / T[7];
  float Ra[3];
  s3lie::act_so3(T + 3, X, Ra);
  Y[0] = s_inv * Ra[0];
  Y[1] = s_inv * Ra[1];
  Y[2] = s_inv * Ra[2];
  s3lie::act_so3(T + 3, X + 3, Y + 3);
  const float* t = T;
  Y[3] += s_inv * (t[1] * Ra[2] - t[2] * Ra[1]);
  Y[4] += s_inv * (t[2] * Ra[0] - t[0] * Ra[2]);
  Y[5] += s_inv * (t[0] * Ra[1] - t[1] * Ra[0]);
  Y[6] = X[6] + s_inv * (t[0] * Ra[0] + t[1] * Ra[1] + t[2] * Ra[2]);
}

enum { kRays = 0, kCalib = 1 };

struct EdgeP {
  const float* Twc;
  const float* Xs;
  const float* Cs;
  int64_t n;
  const int32_t* ii;
  const int32_t* jj;
  const int64_t* idx;
  const uint8_t* valid;
  const float* Q;
  float inv_sr, inv_sd, C_thresh, Q_thresh;
  float* partial;   // [E, S, NA]
  const double* state;
  // calib (calib_proj_kernel): K [3,3] row-major on the device, image size,
  // border and depth floor; inv_sr / inv_sd are then 1/sigma_pixel, 1/sigma_depth
  const float* K;
  int height, width, pixel_border;
  float z_eps;
};

// Accumulate one residual row: A += w Jj^T Jj (upper), u += w r Jj.
__device__ __forceinline__ void accum_row(const float* Ti, const float* Jl, float w, float r,
                                          float* acc) {
  float Jj[7];
  adj_inv(Ti, Jl, Jj);
  int c = 0;
#pragma unroll
  for (int a = 0; a < 7; ++a)
#pragma unroll
    for (int b = a; b < 7; ++b) acc[c++] += w * Jj[a] * Jj[b];
#pragma unroll
  for (int a = 0; a < 7; ++a) acc[28 + a] += w * r * Jj[a];
}

// grid (S, E): slice s of edge e.  MODE kRays: ray_align_kernel
// (gn_kernels.cu:812-1137, 4 rows: ray direction + distance); kCalib:
// calib_proj_kernel (:1230-1542, 3 rows: pixel u, v + log depth).  Both set
// Ji = -Jj, so both reduce to the same 35 accumulators.
template <int MODE>
__global__ void __launch_bounds__(kThreads) k_edge_align(EdgeP p) {
  if (p.state && p.state[0] != 0.0) return;
  const int s = blockIdx.x, S = gridDim.x, e = blockIdx.y;
  const int ix = p.ii[e], jx = p.jj[e];
  float Ti[8], Tj[8], Tij[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { Ti[k] = p.Twc[ix * 8 + k]; Tj[k] = p.Twc[jx * 8 + k]; }
  rel_sim3(Ti, Tj, Tij);
  float acc[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) acc[k] = 0.f;
  const int64_t n = p.n;
  const int64_t chunk = (n + S - 1) / S;
  const int64_t k0 = (int64_t)s * chunk, k1 = min(n, k0 + chunk);
  const float* Xi_all = p.Xs + (int64_t)ix * n * 3;
  const float* Xj_all = p.Xs + (int64_t)jx * n * 3;
  const float* Ci_all = p.Cs + (int64_t)ix * n;
  const float* Cj_all = p.Cs + (int64_t)jx * n;
  const int64_t* idx = p.idx + (int64_t)e * n;
  const uint8_t* vm = p.valid + (int64_t)e * n;
  const float* Qe = p.Q + (int64_t)e * n;
  float fx = 0.f, fy = 0.f, cx = 0.f, cy = 0.f;
  if constexpr (MODE == kCalib) { fx = p.K[0]; fy = p.K[4]; cx = p.K[2]; cy = p.K[5]; }
  for (int64_t k = k0 + threadIdx.x; k < k1; k += kThreads) {
    const bool vmk = vm[k] != 0;
    const int64_t ind = vmk ? idx[k] : 0;
    const float Xi[3] = {Xi_all[ind * 3], Xi_all[ind * 3 + 1], Xi_all[ind * 3 + 2]};
    const float Xj[3] = {Xj_all[k * 3], Xj_all[k * 3 + 1], Xj_all[k * 3 + 2]};
    if constexpr (MODE == kRays) {
      const float n2i = Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2];
      const float n1i = sqrtf(n2i);
      const float n1i_inv = 1.0f / n1i;
      const float ri[3] = {n1i_inv * Xi[0], n1i_inv * Xi[1], n1i_inv * Xi[2]};
      float P[3];
      s3lie::act_sim3(Tij, Xj, P);
      const float n2j = P[0] * P[0] + P[1] * P[1] + P[2] * P[2];
      const float n1j = sqrtf(n2j);
      const float n1j_inv = 1.0f / n1j;
      const float rj[3] = {n1j_inv * P[0], n1j_inv * P[1], n1j_inv * P[2]};
      const float err[4] = {rj[0] - ri[0], rj[1] - ri[1], rj[2] - ri[2], n1j - n1i};
      const float q = Qe[k];
      const float ci = Ci_all[ind], cj = Cj_all[k];
      const bool valid = vmk & (q > p.Q_thresh) & (ci > p.C_thresh) & (cj > p.C_thresh);
      const float sq = sqrtf(q);
      const float swr = valid ? p.inv_sr * sq : 0.f;
      const float swd = valid ? p.inv_sd * sq : 0.f;
      float w[4];
      w[0] = huber_w(swr * err[0]) * (swr * swr);
      w[1] = huber_w(swr * err[1]) * (swr * swr);
      w[2] = huber_w(swr * err[2]) * (swr * swr);
      w[3] = huber_w(swd * err[3]) * (swd * swd);
      const float n3 = n1j_inv / n2j;
      const float dxx = n1j_inv - P[0] * P[0] * n3, dyy = n1j_inv - P[1] * P[1] * n3;
      const float dzz = n1j_inv - P[2] * P[2] * n3;
      const float dxy = -P[0] * P[1] * n3, dxz = -P[0] * P[2] * n3, dyz = -P[1] * P[2] * n3;
      const float Jl[4][7] = {{dxx, dxy, dxz, 0.f, rj[2], -rj[1], 0.f},
                              {dxy, dyy, dyz, -rj[2], 0.f, rj[0], 0.f},
                              {dxz, dyz, dzz, rj[1], -rj[0], 0.f, 0.f},
                              {rj[0], rj[1], rj[2], 0.f, 0.f, 0.f, n1j}};
  #pragma unroll
      for (int r = 0; r < 4; ++r) accum_row(Ti, Jl[r], w[r], err[r], acc);
    } else {
      // calib_proj_kernel:1359-1495
      const int u_target = (int)(ind % p.width), v_target = (int)(ind / p.width);
      float P[3];
      s3lie::act_sim3(Tij, Xj, P);
      const bool valid_z = (P[2] > p.z_eps) && (Xi[2] > p.z_eps);
      const float zj_inv = valid_z ? 1.0f / P[2] : 0.f;
      const float zj_log = valid_z ? logf(P[2]) : 0.f;
      const float zi_log = valid_z ? logf(Xi[2]) : 0.f;
      const float xz = P[0] * zj_inv, yz = P[1] * zj_inv;
      const float u = fx * xz + cx, v = fy * yz + cy;
      const bool valid_u = (u > (float)p.pixel_border) && (u < (float)(p.width - 1 - p.pixel_border));
      const bool valid_v = (v > (float)p.pixel_border) && (v < (float)(p.height - 1 - p.pixel_border));
      const float err[3] = {u - (float)u_target, v - (float)v_target, zj_log - zi_log};
      const float q = Qe[k];
      const float ci = Ci_all[ind], cj = Cj_all[k];
      const bool valid = vmk & (q > p.Q_thresh) & (ci > p.C_thresh) & (cj > p.C_thresh) &
                         valid_u & valid_v & valid_z;
      const float sq = sqrtf(q);
      const float swp = valid ? p.inv_sr * sq : 0.f;
      const float swd = valid ? p.inv_sd * sq : 0.f;
      const float w[3] = {huber_w(swp * err[0]) * (swp * swp), huber_w(swp * err[1]) * (swp * swp),
                          huber_w(swd * err[2]) * (swd * swd)};
      const float Jl[3][7] = {
          {fx * zj_inv, 0.f, -fx * xz * zj_inv, -fx * xz * yz, fx * (1 + xz * xz), -fx * yz, 0.f},
          {0.f, fy * zj_inv, -fy * yz * zj_inv, -fy * (1 + yz * yz), fy * xz * yz, fy * xz, 0.f},
          {0.f, 0.f, zj_inv, yz, -xz, 0.f, 1.0f}};
#pragma unroll
      for (int r = 0; r < 3; ++r) accum_row(Ti, Jl[r], w[r], err[r], acc);
    }
  }
  // wave reduce-scatter (lane k gets the wave total of sum k), then the
  // wave partials through LDS
  __shared__ float red[kThreads / 64][NA];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float wsum = s3::wave_reduce_scatter(acc);
  if (lane < NA) red[wave][lane] = wsum;
  __syncthreads();
  if (threadIdx.x < NA)
    p.partial[((int64_t)e * S + s) * NA + threadIdx.x] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// Per edge, fixed-order fp64 sum of the slices: esum [E, NA].
__global__ void k_edge_sum(const float* __restrict__ partial, int S, int E,
                           double* __restrict__ esum, const double* state) {
  if (state && state[0] != 0.0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * NA) return;
  const int e = t / NA, k = t % NA;
  double s = 0.0;
  for (int i = 0; i < S; ++i) s += (double)partial[((int64_t)e * S + i) * NA + k];
  esum[t] = s;
}

__device__ __forceinline__ double a_elem(const double* A, int a, int b) {
  // upper-triangle row-major index of (min, max)
  const int r = a < b ? a : b, c = a < b ? b : a;
  return A[r * 7 - r * (r - 1) / 2 + (c - r)];
}

// Edges incident to every unfixed pose (CSR, edge ids ascending): one
// workgroup counts, scans, fills with atomic cursors and sorts each list, so
// the assembly below visits only a pose's own edges, in edge order.
constexpr int kCsrThreads = 1024;

__global__ void __launch_bounds__(kCsrThreads)
k_edge_csr(const int32_t* __restrict__ ii, const int32_t* __restrict__ jj, int E, int num_fix,
           int np, int32_t* __restrict__ off, int32_t* __restrict__ list) {
  __shared__ int cnt[4097];
  const int tid = threadIdx.x;
  for (int i = tid; i <= np; i += kCsrThreads) cnt[i] = 0;
  __syncthreads();
  for (int e = tid; e < E; e += kCsrThreads) {
    const int io = ii[e] - num_fix, jo = jj[e] - num_fix;
    if (io >= 0) atomicAdd(&cnt[io], 1);
    if (jo >= 0) atomicAdd(&cnt[jo], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int i = 0; i < np; ++i) {
      const int c = cnt[i];
      off[i] = acc;
      cnt[i] = acc;       // becomes the fill cursor
      acc += c;
    }
    off[np] = acc;
  }
  __syncthreads();
  for (int e = tid; e < E; e += kCsrThreads) {
    const int io = ii[e] - num_fix, jo = jj[e] - num_fix;
    if (io >= 0) list[atomicAdd(&cnt[io], 1)] = e;
    if (jo >= 0) list[atomicAdd(&cnt[jo], 1)] = e;
  }
  __syncthreads();
  // ascending edge ids per pose (insertion sort; lists are short)
  for (int pz = tid; pz < np; pz += kCsrThreads) {
    const int a = off[pz], z = off[pz + 1];
    for (int i = a + 1; i < z; ++i) {
      const int v = list[i];
      int j = i - 1;
      while (j >= a && list[j] > v) {
        list[j + 1] = list[j];
        --j;
      }
      list[j + 1] = v;
    }
  }
}

// Dense H [n x n], b [n] over the unfixed poses: edge blocks (io,io)+A,
// (io,jo)-A, (jo,io)-A, (jo,jo)+A and b(io) -u, b(jo) +u (SparseBlock
// update_lhs/update_rhs with Hs = {A, -A, -A, A}, gs = {-u, u}).  Element
// (r, c) of block (pr, pc) sums over pr's incident edges in edge order: the
// same terms in the same order as a sweep over all edges (the others add
// nothing), at O(degree) instead of O(E) per element.
__global__ void k_assemble(const double* __restrict__ esum, const int32_t* __restrict__ ii,
                           const int32_t* __restrict__ jj, const int32_t* __restrict__ off,
                           const int32_t* __restrict__ list, int num_fix, int n,
                           double* __restrict__ H, double* __restrict__ b, const double* state) {
  if (state && state[0] != 0.0) return;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * n + n) return;
  if (t < (int64_t)n * n) {
    const int r = (int)(t / n), c = (int)(t % n);
    const int pr = r / 7, a = r % 7, pc = c / 7, bb = c % 7;
    double h = 0.0;
    for (int q = off[pr]; q < off[pr + 1]; ++q) {
      const int e = list[q];
      const int io = ii[e] - num_fix, jo = jj[e] - num_fix;
      const double* A = esum + (int64_t)e * NA;
      double sgn = 0.0;
      if (pr == io && pc == io) sgn += 1.0;
      if (pr == io && pc == jo) sgn -= 1.0;
      if (pr == jo && pc == io) sgn -= 1.0;
      if (pr == jo && pc == jo) sgn += 1.0;
      if (sgn != 0.0) h += sgn * a_elem(A, a, bb);
    }
    H[t] = h;
  } else {
    const int r = (int)(t - (int64_t)n * n);
    const int pr = r / 7, a = r % 7;
    double v = 0.0;
    for (int q = off[pr]; q < off[pr + 1]; ++q) {
      const int e = list[q];
      const int io = ii[e] - num_fix, jo = jj[e] - num_fix;
      const double u = esum[(int64_t)e * NA + 28 + a];
      if (pr == io) v -= u;
      if (pr == jo) v += u;
    }
    b[r] = v;
  }
}

// ---- blocked right-looking Cholesky (multi-workgroup) ------------------
// H = L L^T in place (lower), 64-wide panels, three launches per panel:
// the diagonal block in one workgroup (LDS), the panel below it (one
// workgroup per 64 rows, triangular solve against the LDS diagonal block),
// and the trailing lower triangle (one workgroup per 64x64 block,
// H_ij -= L_i L_j^T with the two panel slices in LDS).  Replaces the
// O(n^3)-in-one-workgroup factorisation for long keyframe sequences.  A
// non-positive pivot sets ctl[0]; later launches then skip and the solve
// writes dx = 0 (SimplicialLLT failure in the reference).
constexpr int kNB = 64;
// systems up to this size keep the single-workgroup factorisation (the
// small pose graphs of the first keyframes: one launch instead of 3 per panel)
constexpr int kSmallChol = 7 * 24;

__global__ void __launch_bounds__(kThreads)
k_potrf_diag(double* __restrict__ H, int n, int k0, int* __restrict__ ctl, const double* state) {
  if ((state && state[0] != 0.0) || ctl[0]) return;
  __shared__ double A[kNB][kNB + 1];
  __shared__ int fail;
  const int nb = min(kNB, n - k0), tid = threadIdx.x;
  for (int t = tid; t < nb * nb; t += kThreads) {
    const int i = t / nb, j = t % nb;
    A[i][j] = H[(int64_t)(k0 + i) * n + k0 + j];
  }
  if (tid == 0) fail = 0;
  __syncthreads();
  for (int k = 0; k < nb; ++k) {
    if (tid == 0) {
      const double d = A[k][k];
      if (!(d > 0.0)) fail = 1;
      A[k][k] = fail ? 1.0 : sqrt(d);
    }
    __syncthreads();
    if (fail) break;
    for (int i = k + 1 + tid; i < nb; i += kThreads) A[i][k] /= A[k][k];
    __syncthreads();
    const int m = nb - k - 1;
    for (int t = tid; t < m * m; t += kThreads) {
      const int i = k + 1 + t / m, j = k + 1 + t % m;
      if (j <= i) A[i][j] -= A[i][k] * A[j][k];
    }
    __syncthreads();
  }
  if (fail) {
    if (tid == 0) ctl[0] = 1;
    return;
  }
  for (int t = tid; t < nb * nb; t += kThreads) {
    const int i = t / nb, j = t % nb;
    if (j <= i) H[(int64_t)(k0 + i) * n + k0 + j] = A[i][j];
  }
}

// L21 = A21 L11^-T: one thread per row of the panel, columns in order.
__global__ void __launch_bounds__(kThreads)
k_trsm_panel(double* __restrict__ H, int n, int k0, const int* __restrict__ ctl,
             const double* state) {
  if ((state && state[0] != 0.0) || ctl[0]) return;
  __shared__ double L[kNB][kNB + 1];
  const int nb = min(kNB, n - k0), tid = threadIdx.x;
  for (int t = tid; t < nb * nb; t += kThreads) {
    const int i = t / nb, j = t % nb;
    L[i][j] = j <= i ? H[(int64_t)(k0 + i) * n + k0 + j] : 0.0;
  }
  __syncthreads();
  const int r = k0 + nb + blockIdx.x * kThreads + tid;
  if (r >= n) return;
  // in place along the row (the solved prefix stays in the row, L1-resident)
  double* row = H + (int64_t)r * n + k0;
  for (int c = 0; c < nb; ++c) {
    double v = row[c];
    for (int j = 0; j < c; ++j) v -= row[j] * L[c][j];
    row[c] = v / L[c][c];
  }
}

// Trailing update of the lower triangle: block (bi, bj), bi >= bj, of the
// rows/cols after the panel: H_ij -= L_i L_j^T (L_* = panel columns).
__global__ void __launch_bounds__(kThreads)
k_syrk_trailing(double* __restrict__ H, int n, int k0, const int* __restrict__ ctl,
                const double* state) {
  if ((state && state[0] != 0.0) || ctl[0]) return;
  const int nb = min(kNB, n - k0);
  const int base = k0 + nb;
  // linear block index -> (bi, bj), bj <= bi
  const int t = blockIdx.x;
  int bi = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
  while (bi * (bi + 1) / 2 > t) --bi;
  const int bj = t - bi * (bi + 1) / 2;
  const int r0 = base + bi * kNB, c0 = base + bj * kNB;
  if (r0 >= n || c0 >= n) return;
  __shared__ double Li[kNB][kNB + 1];
  __shared__ double Lj[kNB][kNB + 1];
  const int tid = threadIdx.x;
  for (int q = tid; q < kNB * nb; q += kThreads) {
    const int i = q / nb, k = q % nb;
    Li[i][k] = r0 + i < n ? H[(int64_t)(r0 + i) * n + k0 + k] : 0.0;
    Lj[i][k] = c0 + i < n ? H[(int64_t)(c0 + i) * n + k0 + k] : 0.0;
  }
  __syncthreads();
  // 256 threads x 16 outputs: thread (ty, tx) owns rows ty*4..+4, cols tx*4..+4
  const int ty = tid / 16, tx = tid % 16;
  double acc[4][4] = {};
  for (int k = 0; k < nb; ++k) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { a[u] = Li[ty * 4 + u][k]; b[u] = Lj[tx * 4 + u][k]; }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[u][v] += a[u] * b[v];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = r0 + ty * 4 + u, j = c0 + tx * 4 + v;
      if (i < n && j < n && j <= i) H[(int64_t)i * n + j] -= acc[u][v];
    }
}

// L L^T x = b after the blocked factorisation (one workgroup), dx = -x;
// a failed factorisation (ctl[0]) gives dx = 0.
__global__ void __launch_bounds__(kThreads)
k_chol_subst(const double* __restrict__ H, double* __restrict__ b, int n,
             float* __restrict__ dx, const int* __restrict__ ctl, const double* state) {
  if (state && state[0] != 0.0) return;
  const int tid = threadIdx.x;
  if (ctl[0]) {
    for (int i = tid; i < n; i += kThreads) dx[i] = 0.f;
    return;
  }
  for (int k = 0; k < n; ++k) {
    if (tid == 0) b[k] /= H[(int64_t)k * n + k];
    __syncthreads();
    const double yk = b[k];
    for (int i = k + 1 + tid; i < n; i += kThreads) b[i] -= H[(int64_t)i * n + k] * yk;
    __syncthreads();
  }
  for (int k = n - 1; k >= 0; --k) {
    if (tid == 0) b[k] /= H[(int64_t)k * n + k];
    __syncthreads();
    const double xk = b[k];
    for (int i = tid; i < k; i += kThreads) b[i] -= H[(int64_t)k * n + i] * xk;
    __syncthreads();
  }
  for (int i = tid; i < n; i += kThreads) dx[i] = (float)(-b[i]);
}

// One workgroup: in-place fp64 Cholesky H = L L^T (lower), then L L^T x = b,
// dx = -x (fp32).  Not positive definite -> dx = 0 (the reference returns
// zeros when SimplicialLLT fails), which then ends the iterations.
__global__ void __launch_bounds__(kThreads)
k_chol_solve(double* __restrict__ H, double* __restrict__ b, int n, float* __restrict__ dx,
             double* state) {
  if (state && state[0] != 0.0) return;
  __shared__ int fail;
  __shared__ double piv;
  const int tid = threadIdx.x;
  if (tid == 0) fail = 0;
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    if (tid == 0) {
      const double d = H[(int64_t)k * n + k];
      if (!(d > 0.0)) fail = 1;
      piv = fail ? 1.0 : sqrt(d);
      H[(int64_t)k * n + k] = piv;
    }
    __syncthreads();
    if (fail) break;
    const double pv = piv;
    for (int i = k + 1 + tid; i < n; i += kThreads) H[(int64_t)i * n + k] /= pv;
    __syncthreads();
    const int m = n - k - 1;
    for (int64_t t = tid; t < (int64_t)m * m; t += kThreads) {
      const int i = k + 1 + (int)(t / m), j = k + 1 + (int)(t % m);
      if (j <= i) H[(int64_t)i * n + j] -= H[(int64_t)i * n + k] * H[(int64_t)j * n + k];
    }
    __syncthreads();
  }
  if (fail) {
    for (int i = tid; i < n; i += kThreads) dx[i] = 0.f;
    return;
  }
  // forward: L y = b (y overwrites b)
  for (int k = 0; k < n; ++k) {
    if (tid == 0) b[k] /= H[(int64_t)k * n + k];
    __syncthreads();
    const double yk = b[k];
    for (int i = k + 1 + tid; i < n; i += kThreads) b[i] -= H[(int64_t)i * n + k] * yk;
    __syncthreads();
  }
  // backward: L^T x = y
  for (int k = n - 1; k >= 0; --k) {
    if (tid == 0) b[k] /= H[(int64_t)k * n + k];
    __syncthreads();
    const double xk = b[k];
    for (int i = tid; i < k; i += kThreads) b[i] -= H[(int64_t)k * n + i] * xk;
    __syncthreads();
  }
  for (int i = tid; i < n; i += kThreads) dx[i] = (float)(-b[i]);
}

// pose_retr_kernel (gn_kernels.cu:414-454): T_k <- Exp(dx_k) T_k for the
// unfixed poses, |dx|, iteration count and the termination flag.
// state: [0] flag (1 = |dx| < delta_thresh), [1] iterations, [2] |dx|.
__global__ void __launch_bounds__(kThreads)
k_retr(float* __restrict__ Twc, int n_poses, int num_fix, const float* __restrict__ dx,
       float delta_thresh, double* state) {
  if (state[0] != 0.0) return;
  const int tid = threadIdx.x;
  for (int k = num_fix + tid; k < n_poses; k += kThreads) {
    float T[8], out[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) T[c] = Twc[k * 8 + c];
    s3lie::retr_sim3(T, dx + (k - num_fix) * 7, out);
#pragma unroll
    for (int c = 0; c < 8; ++c) Twc[k * 8 + c] = out[c];
  }
  const int m = (n_poses - num_fix) * 7;
  double s = 0.0;
  for (int i = tid; i < m; i += kThreads) s += (double)dx[i] * (double)dx[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double red[kThreads / 64];
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    const float nrm = (float)sqrt((red[0] + red[1]) + (red[2] + red[3]));
    state[1] += 1.0;
    state[2] = nrm;
    if (nrm < delta_thresh) state[0] = 1.0;
  }
}

struct Ws {
  float* partial;
  double* esum;
  double* H;
  double* b;
  double* state;
  int32_t* off;    // [free poses + 1] CSR offsets of the incident edges
  int32_t* list;   // [2 E] incident edge ids
  int* ctl;        // [0]: blocked Cholesky failed (non-positive pivot)
  int S;
};

int slices(int n_edges, int64_t n_points) {
  int S = (int)s3::cdiv(1024, n_edges > 0 ? n_edges : 1);
  const int64_t maxs = s3::cdiv(n_points, 1024);
  if (S > maxs) S = (int)maxs;
  return S < 1 ? 1 : S;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

Ws carve(void* ws, int n_poses, int n_edges, int64_t n_points, int num_fix) {
  Ws w;
  w.S = slices(n_edges, n_points);
  const int n = 7 * (n_poses - num_fix);
  char* p = static_cast<char*>(ws);
  w.partial = reinterpret_cast<float*>(p);
  p += align256(sizeof(float) * (size_t)n_edges * w.S * NA);
  w.esum = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * (size_t)n_edges * NA);
  w.H = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * (size_t)n * n);
  w.b = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * (size_t)n);
  w.state = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * 4);
  w.off = reinterpret_cast<int32_t*>(p);
  p += align256(sizeof(int32_t) * (size_t)(n / 7 + 1));
  w.list = reinterpret_cast<int32_t*>(p);
  p += align256(sizeof(int32_t) * 2 * (size_t)n_edges);
  w.ctl = reinterpret_cast<int*>(p);
  return w;
}

int check_args(int n_poses, int n_edges, int64_t n_points, int num_fix) {
  S3_REQUIRE(n_poses > num_fix && num_fix >= 0 && n_edges >= 0 && n_points > 0,
             "s3g: bad sizes (poses %d, fixed %d, edges %d)", n_poses, num_fix, n_edges);
  S3_REQUIRE(7LL * (n_poses - num_fix) <= 7 * 4096, "s3g: at most 4096 free poses");
  return S3_OK;
}

// Calib extras of EdgeP (null K = rays).
struct CalibArgs {
  const float* K = nullptr;
  int height = 0, width = 0, pixel_border = 0;
  float z_eps = 0.f;
};

int queue_system(const float* Twc, const float* Xs, const float* Cs, int64_t n_points,
                 const int32_t* ii, const int32_t* jj, int n_edges, const int64_t* idx,
                 const uint8_t* valid, const float* Q, float sigma_a, float sigma_b,
                 float C_thresh, float Q_thresh, int num_fix, int n, const Ws& w,
                 const double* state, hipStream_t st, const CalibArgs& cal = CalibArgs()) {
  if (n_edges > 0) {
    EdgeP p{Twc, Xs, Cs, n_points, ii, jj, idx, valid, Q, 1.0f / sigma_a, 1.0f / sigma_b,
            C_thresh, Q_thresh, w.partial, state, cal.K, cal.height, cal.width,
            cal.pixel_border, cal.z_eps};
    if (cal.K)
      k_edge_align<kCalib><<<dim3(w.S, n_edges), kThreads, 0, st>>>(p);
    else
      k_edge_align<kRays><<<dim3(w.S, n_edges), kThreads, 0, st>>>(p);
    S3_LAUNCH_CHECK();
    k_edge_sum<<<(unsigned)s3::cdiv((int64_t)n_edges * NA, kThreads), kThreads, 0, st>>>(
        w.partial, w.S, n_edges, w.esum, state);
    S3_LAUNCH_CHECK();
  }
  k_assemble<<<(unsigned)s3::cdiv((int64_t)n * n + n, kThreads), kThreads, 0, st>>>(
      w.esum, ii, jj, w.off, w.list, num_fix, n, w.H, w.b, state);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

// The incident-edge CSR of the (constant) edge set, once per solve.
int queue_csr(const int32_t* ii, const int32_t* jj, int n_edges, int num_fix, int n, const Ws& w,
              hipStream_t st) {
  k_edge_csr<<<1, kCsrThreads, 0, st>>>(ii, jj, n_edges, num_fix, n / 7, w.off, w.list);
  S3_LAUNCH_CHECK();
  return S3_OK;
}

}  // namespace

extern "C" size_t s3g_workspace_bytes(int n_poses, int n_edges, int64_t n_points, int num_fix) {
  const int S = slices(n_edges, n_points);
  const size_t n = 7 * (size_t)(n_poses > num_fix ? n_poses - num_fix : 0);
  return align256(sizeof(float) * (size_t)n_edges * S * NA) +
         align256(sizeof(double) * (size_t)n_edges * NA) + align256(sizeof(double) * n * n) +
         align256(sizeof(double) * n) + align256(sizeof(double) * 4) +
         align256(sizeof(int32_t) * (n / 7 + 1)) + align256(sizeof(int32_t) * 2 * (size_t)n_edges) +
         align256(sizeof(int) * 4);
}

extern "C" int s3g_ray_system(const float* Twc, int n_poses, const float* Xs, const float* Cs,
                              int64_t n_points, const int32_t* ii, const int32_t* jj, int n_edges,
                              const int64_t* idx_ii2jj, const uint8_t* valid_match,
                              const float* Q, float sigma_ray, float sigma_dist, float C_thresh,
                              float Q_thresh, int num_fix, void* workspace, double* H, double* b,
                              void* stream) {
  if (int r = check_args(n_poses, n_edges, n_points, num_fix)) return r;
  S3_REQUIRE(workspace && H && b, "s3g_ray_system: null workspace/output");
  hipStream_t st = s3::as_stream(stream);
  Ws w = carve(workspace, n_poses, n_edges, n_points, num_fix);
  w.H = H;
  w.b = b;
  const int n = 7 * (n_poses - num_fix);
  if (int r = queue_csr(ii, jj, n_edges, num_fix, n, w, st)) return r;
  return queue_system(Twc, Xs, Cs, n_points, ii, jj, n_edges, idx_ii2jj, valid_match, Q,
                      sigma_ray, sigma_dist, C_thresh, Q_thresh, num_fix, n, w, nullptr, st);
}

namespace {
int solve(float* Twc, int n_poses, const float* Xs, const float* Cs, int64_t n_points,
          const int32_t* ii, const int32_t* jj, int n_edges, const int64_t* idx_ii2jj,
          const uint8_t* valid_match, const float* Q, float sigma_a, float sigma_b,
          float C_thresh, float Q_thresh, int max_iter, float delta_thresh, int num_fix,
          void* workspace, float* dx, float* stats, hipStream_t st, const CalibArgs& cal) {
  Ws w = carve(workspace, n_poses, n_edges, n_points, num_fix);
  const int n = 7 * (n_poses - num_fix);
  S3_HIP(hipMemsetAsync(w.state, 0, sizeof(double) * 4, st));
  S3_HIP(hipMemsetAsync(dx, 0, sizeof(float) * n, st));
  if (int r = queue_csr(ii, jj, n_edges, num_fix, n, w, st)) return r;
  for (int it = 0; it < max_iter; ++it) {
    if (int r = queue_system(Twc, Xs, Cs, n_points, ii, jj, n_edges, idx_ii2jj, valid_match, Q,
                             sigma_a, sigma_b, C_thresh, Q_thresh, num_fix, n, w, w.state, st,
                             cal))
      return r;
    if (n <= kSmallChol) {
      k_chol_solve<<<1, kThreads, 0, st>>>(w.H, w.b, n, dx, w.state);
      S3_LAUNCH_CHECK();
    } else {
      S3_HIP(hipMemsetAsync(w.ctl, 0, sizeof(int), st));
      for (int k0 = 0; k0 < n; k0 += kNB) {
        k_potrf_diag<<<1, kThreads, 0, st>>>(w.H, n, k0, w.ctl, w.state);
        S3_LAUNCH_CHECK();
        const int rest = n - k0 - kNB;
        if (rest > 0) {
          k_trsm_panel<<<(unsigned)s3::cdiv(rest, kThreads), kThreads, 0, st>>>(w.H, n, k0, w.ctl,
                                                                               w.state);
          S3_LAUNCH_CHECK();
          const int T = (int)s3::cdiv(rest, kNB);
          k_syrk_trailing<<<(unsigned)(T * (T + 1) / 2), kThreads, 0, st>>>(w.H, n, k0, w.ctl,
                                                                            w.state);
          S3_LAUNCH_CHECK();
        }
      }
      k_chol_subst<<<1, kThreads, 0, st>>>(w.H, w.b, n, dx, w.ctl, w.state);
      S3_LAUNCH_CHECK();
    }
    k_retr<<<1, kThreads, 0, st>>>(Twc, n_poses, num_fix, dx, delta_thresh, w.state);
    S3_LAUNCH_CHECK();
  }
  // stats = {iterations, |dx|} (fp32) from the device state
  double host_state[4];
  S3_HIP(hipMemcpyAsync(host_state, w.state, sizeof(host_state), hipMemcpyDeviceToHost, st));
  S3_HIP(hipStreamSynchronize(st));
  stats[0] = (float)host_state[1];
  stats[1] = (float)host_state[2];
  return S3_OK;
}
}  // namespace

extern "C" int s3g_gauss_newton_rays(float* Twc, int n_poses, const float* Xs, const float* Cs,
                                     int64_t n_points, const int32_t* ii, const int32_t* jj,
                                     int n_edges, const int64_t* idx_ii2jj,
                                     const uint8_t* valid_match, const float* Q, float sigma_ray,
                                     float sigma_dist, float C_thresh, float Q_thresh,
                                     int max_iter, float delta_thresh, int num_fix,
                                     void* workspace, float* dx, float* stats, void* stream) {
  if (int r = check_args(n_poses, n_edges, n_points, num_fix)) return r;
  S3_REQUIRE(workspace && dx && stats && max_iter >= 0, "s3g_gauss_newton_rays: bad arguments");
  return solve(Twc, n_poses, Xs, Cs, n_points, ii, jj, n_edges, idx_ii2jj, valid_match, Q,
               sigma_ray, sigma_dist, C_thresh, Q_thresh, max_iter, delta_thresh, num_fix,
               workspace, dx, stats, s3::as_stream(stream), CalibArgs());
}

namespace {
int check_calib(const float* K, int height, int width, int pixel_border, int64_t n_points) {
  S3_REQUIRE(K != nullptr, "s3g calib: null K");
  S3_REQUIRE(height > 0 && width > 0, "s3g calib: bad image size %dx%d",
             height, width);
  S3_REQUIRE((int64_t)height * width == n_points,
             "s3g calib: points per pose (%lld) must be height*width (%d x %d)",
             (long long)n_points, height, width);
  return S3_OK;
}
}  // namespace

extern "C" int s3g_calib_system(const float* Twc, int n_poses, const float* Xs, const float* Cs,
                                int64_t n_points, const float* K, const int32_t* ii,
                                const int32_t* jj, int n_edges, const int64_t* idx_ii2jj,
                                const uint8_t* valid_match, const float* Q, int height, int width,
                                int pixel_border, float z_eps, float sigma_pixel,
                                float sigma_depth, float C_thresh, float Q_thresh, int num_fix,
                                void* workspace, double* H, double* b, void* stream) {
  if (int r = check_args(n_poses, n_edges, n_points, num_fix)) return r;
  if (int r = check_calib(K, height, width, pixel_border, n_points)) return r;
  S3_REQUIRE(workspace && H && b, "s3g_calib_system: null workspace/output");
  hipStream_t st = s3::as_stream(stream);
  Ws w = carve(workspace, n_poses, n_edges, n_points, num_fix);
  w.H = H;
  w.b = b;
  const int n = 7 * (n_poses - num_fix);
  CalibArgs cal;
  cal.K = K; cal.height = height; cal.width = width; cal.pixel_border = pixel_border;
  cal.z_eps = z_eps;
  if (int r = queue_csr(ii, jj, n_edges, num_fix, n, w, st)) return r;
  return queue_system(Twc, Xs, Cs, n_points, ii, jj, n_edges, idx_ii2jj, valid_match, Q,
                      sigma_pixel, sigma_depth, C_thresh, Q_thresh, num_fix, n, w, nullptr, st,
                      cal);
}

extern "C" int s3g_gauss_newton_calib(float* Twc, int n_poses, const float* Xs, const float* Cs,
                                      int64_t n_points, const float* K, const int32_t* ii,
                                      const int32_t* jj, int n_edges, const int64_t* idx_ii2jj,
                                      const uint8_t* valid_match, const float* Q, int height,
                                      int width, int pixel_border, float z_eps, float sigma_pixel,
                                      float sigma_depth, float C_thresh, float Q_thresh,
                                      int max_iter, float delta_thresh, int num_fix,
                                      void* workspace, float* dx, float* stats, void* stream) {
  if (int r = check_args(n_poses, n_edges, n_points, num_fix)) return r;
  if (int r = check_calib(K, height, width, pixel_border, n_points)) return r;
  S3_REQUIRE(workspace && dx && stats && max_iter >= 0, "s3g_gauss_newton_calib: bad arguments");
  CalibArgs cal;
  cal.K = K; cal.height = height; cal.width = width; cal.pixel_border = pixel_border;
  cal.z_eps = z_eps;
  return solve(Twc, n_poses, Xs, Cs, n_points, ii, jj, n_edges, idx_ii2jj, valid_match, Q,
               sigma_pixel, sigma_depth, C_thresh, Q_thresh, max_iter, delta_thresh, num_fix,
               workspace, dx, stats, s3::as_stream(stream), cal);
}
