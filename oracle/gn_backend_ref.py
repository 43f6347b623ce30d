"""ORACLE (test infrastructure only) — numpy float64 restatement of the
backend pose-graph Gauss-Newton on rays, mast3r_slam_backends.gauss_newton_rays:

  gauss_newton_rays_cuda   splatt3r_slam/backend/src/gn_kernels.cu:1139-1227
  ray_align_kernel         gn_kernels.cu:812-1137 (residuals, Huber weights,
                           14-dof Jacobians, per-edge H/g blocks)
  relSim3 / actSO3 /       gn_kernels.cu:195-296
  apply_Sim3_adj_inv
  SparseBlock              gn_kernels.cu:56-158 (block assembly; the SimplicialLLT
                           solve is restated as a dense Cholesky, same system)
  pose_retr_kernel         gn_kernels.cu:414-454 (via oracle.pose_retr, the C sim3 restatement)
  calib_proj_kernel        gn_kernels.cu:1230-1542 (calibrated: pixel u, v + log depth
                           residuals; edge_system_calib) and gauss_newton_calib_cuda
                           :1545-1637 (same solve loop)

Parity vs the reference binary is unpinned (the CUDA extension needs Eigen
and nvcc, neither present); the restatement follows the source text and is
checked by the tests against geometric identities (zero residual at the true
poses, recovery of perturbed poses) and used as the checker for the HIP
kernels.
"""
from __future__ import annotations

import numpy as np

HUBER_K = 1.345


def quat_inv(q):
    return np.concatenate([-q[..., :3], q[..., 3:]], -1)


def quat_comp(a, b):
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz], -1)


def act_so3(q, X):
    """gn_kernels.cu:195-205 (uv = 2 q x X; Y = X + w uv + q x uv)."""
    qv, w = q[..., :3], q[..., 3:]
    uv = 2.0 * np.cross(qv, X)
    return X + w * uv + np.cross(qv, uv)


def rel_sim3(Ti, Tj):
    """gn_kernels.cu:251-271: T_ij = T_i^-1 T_j as (t, q, s)."""
    si_inv = 1.0 / Ti[7]
    qi_inv = quat_inv(Ti[3:7])
    qij = quat_comp(qi_inv, Tj[3:7])
    tij = act_so3(qi_inv, Tj[:3] - Ti[:3]) * si_inv
    return tij, qij, si_inv * Tj[7]


def adj_inv(t, q, s, X):
    """gn_kernels.cu:276-296 apply_Sim3_adj_inv on row vectors X [..., 7]."""
    s_inv = 1.0 / s
    Ra = act_so3(q, X[..., 0:3])
    Y = np.empty_like(X)
    Y[..., 0:3] = s_inv * Ra
    Y[..., 3:6] = act_so3(q, X[..., 3:6]) + s_inv * np.cross(t, Ra)
    Y[..., 6] = X[..., 6] + s_inv * (Ra @ t)
    return Y


def huber(r):
    a = np.abs(r)
    return np.where(a < HUBER_K, 1.0, HUBER_K / np.maximum(a, 1e-300))


def edge_system(Ti, Tj, Xi_all, Ci_all, Xj, Cj, idx, valid_match, Q, sigma_ray, sigma_dist,
                C_thresh, Q_thresh):
    """One edge of ray_align_kernel: returns (H [14,14], v [14]) with
    v = sum_rows w err J (J = [Ji, Jj]), H = sum w J^T J."""
    vm = valid_match.astype(bool)
    ind = np.where(vm, idx, 0)
    Xi = Xi_all[ind].astype(np.float64)
    ci = Ci_all[ind].astype(np.float64)
    Xj = Xj.astype(np.float64)
    ri = Xi / np.linalg.norm(Xi, axis=-1, keepdims=True)
    tij, qij, sij = rel_sim3(Ti.astype(np.float64), Tj.astype(np.float64))
    P = sij * act_so3(qij, Xj) + tij
    nj = np.linalg.norm(P, axis=-1)
    rj = P / nj[:, None]
    ni = np.linalg.norm(Xi, axis=-1)
    err = np.concatenate([rj - ri, (nj - ni)[:, None]], -1)        # [n, 4]
    q = Q.astype(np.float64)
    valid = vm & (q > Q_thresh) & (ci > C_thresh) & (Cj > C_thresh)
    sw_r = np.where(valid, np.sqrt(q) / sigma_ray, 0.0)
    sw_d = np.where(valid, np.sqrt(q) / sigma_dist, 0.0)
    sw = np.stack([sw_r, sw_r, sw_r, sw_d], -1)
    w = huber(sw * err) * sw * sw                                     # [n, 4]
    n3 = 1.0 / (nj * nj * nj)
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    ni_j = 1.0 / nj
    dxx, dyy, dzz = ni_j - x * x * n3, ni_j - y * y * n3, ni_j - z * z * n3
    dxy, dxz, dyz = -x * y * n3, -x * z * n3, -y * z * n3
    zero = np.zeros_like(x)
    rx, ry, rz = rj[:, 0], rj[:, 1], rj[:, 2]
    Jloc = np.stack([
        np.stack([dxx, dxy, dxz, zero, rz, -ry, zero], -1),
        np.stack([dxy, dyy, dyz, -rz, zero, rx, zero], -1),
        np.stack([dxz, dyz, dzz, ry, -rx, zero, zero], -1),
        np.stack([rx, ry, rz, zero, zero, zero, nj], -1)], 1)        # [n, 4, 7]
    Jj = adj_inv(Ti[:3].astype(np.float64), Ti[3:7].astype(np.float64), float(Ti[7]), Jloc)
    J = np.concatenate([-Jj, Jj], -1)                                 # [n, 4, 14]
    H = np.einsum("nr,nra,nrb->ab", w, J, J)
    v = np.einsum("nr,nr,nra->a", w, err, J)
    return H, v


def edge_system_calib(Ti, Tj, Xi_all, Ci_all, Xj, Cj, idx, valid_match, Q, sigma_pixel,
                      sigma_depth, C_thresh, Q_thresh, K, height, width, pixel_border, z_eps):
    """One edge of calib_proj_kernel (gn_kernels.cu:1345-1495): rows
    u - u_target, v - v_target (target = matched pixel idx % width,
    idx / width), log z_j - log z_i; valid inside the border with both
    depths > z_eps.  Returns (H [14,14], v [14])."""
    vm = valid_match.astype(bool)
    ind = np.where(vm, idx, 0)
    Xi = Xi_all[ind].astype(np.float64)
    ci = Ci_all[ind].astype(np.float64)
    tij, qij, sij = rel_sim3(Ti.astype(np.float64), Tj.astype(np.float64))
    P = sij * act_so3(qij, Xj.astype(np.float64)) + tij
    fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    valid_z = (P[:, 2] > z_eps) & (Xi[:, 2] > z_eps)
    zs = np.where(valid_z, P[:, 2], 1.0)
    zinv = np.where(valid_z, 1.0 / zs, 0.0)
    zj_log = np.where(valid_z, np.log(zs), 0.0)
    zi_log = np.where(valid_z, np.log(np.where(valid_z, Xi[:, 2], 1.0)), 0.0)
    xz, yz = P[:, 0] * zinv, P[:, 1] * zinv
    u, v = fx * xz + cx, fy * yz + cy
    valid_u = (u > pixel_border) & (u < width - 1 - pixel_border)
    valid_v = (v > pixel_border) & (v < height - 1 - pixel_border)
    err = np.stack([u - ind % width, v - ind // width, zj_log - zi_log], -1)
    q = Q.astype(np.float64)
    valid = vm & (q > Q_thresh) & (ci > C_thresh) & (Cj > C_thresh) & valid_u & valid_v & valid_z
    sw_p = np.where(valid, np.sqrt(q) / sigma_pixel, 0.0)
    sw_d = np.where(valid, np.sqrt(q) / sigma_depth, 0.0)
    sw = np.stack([sw_p, sw_p, sw_d], -1)
    w = huber(sw * err) * sw * sw
    zero, one = np.zeros_like(u), np.ones_like(u)
    Jloc = np.stack([
        np.stack([fx * zinv, zero, -fx * xz * zinv, -fx * xz * yz, fx * (1 + xz * xz), -fx * yz,
                  zero], -1),
        np.stack([zero, fy * zinv, -fy * yz * zinv, -fy * (1 + yz * yz), fy * xz * yz, fy * xz,
                  zero], -1),
        np.stack([zero, zero, zinv, yz, -xz, zero, one], -1)], 1)        # [n, 3, 7]
    Jj = adj_inv(Ti[:3].astype(np.float64), Ti[3:7].astype(np.float64), float(Ti[7]), Jloc)
    J = np.concatenate([-Jj, Jj], -1)
    H = np.einsum("nr,nra,nrb->ab", w, J, J)
    v_ = np.einsum("nr,nr,nra->a", w, err, J)
    return H, v_


def build_system(Twc, Xs, Cs, ii, jj, idx, valid_match, Q, sigma_ray, sigma_dist, C_thresh,
                 Q_thresh, num_fix=1, calib=None):
    """Dense (H, b) over the unfixed poses (SparseBlock.update_lhs/rhs).
    calib = dict(K, height, width, pixel_border, z_eps) selects the
    calibrated residuals (sigma_ray/sigma_dist are then sigma_pixel/sigma_depth)."""
    N = Twc.shape[0]
    n = 7 * (N - num_fix)
    H = np.zeros((n, n))
    b = np.zeros(n)
    for e in range(len(ii)):
        i, j = int(ii[e]), int(jj[e])
        args = (Twc[i], Twc[j], Xs[i], Cs[i, :, 0], Xs[j], Cs[j, :, 0], idx[e],
                valid_match[e, :, 0], Q[e, :, 0], sigma_ray, sigma_dist, C_thresh, Q_thresh)
        He, ve = edge_system_calib(*args, **calib) if calib else edge_system(*args)
        io, jo = i - num_fix, j - num_fix
        for (p, a0) in ((io, 0), (jo, 7)):
            if p < 0:
                continue
            b[7 * p:7 * p + 7] += ve[a0:a0 + 7]
            for (r, b0) in ((io, 0), (jo, 7)):
                if r >= 0:
                    H[7 * p:7 * p + 7, 7 * r:7 * r + 7] += He[a0:a0 + 7, b0:b0 + 7]
    return H, b


def gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid_match, Q, sigma_ray, sigma_dist, C_thresh,
                      Q_thresh, max_iter, delta_thresh, num_fix=1, calib=None):
    """Whole solve on local pose indices ii/jj (already searchsorted into the
    rows of Twc).  Returns (Twc_new float32, dx float32, iterations)."""
    import oracle
    T = np.array(Twc, np.float32)
    dx = np.zeros((T.shape[0] - num_fix, 7), np.float32)
    it = 0
    for it in range(1, max_iter + 1):
        H, b = build_system(T, Xs, Cs, ii, jj, idx, valid_match, Q, sigma_ray, sigma_dist,
                            C_thresh, Q_thresh, num_fix, calib)
        try:
            L = np.linalg.cholesky(H)
            x = np.linalg.solve(L.T, np.linalg.solve(L, b))
            dx = (-x).astype(np.float32).reshape(-1, 7)
        except np.linalg.LinAlgError:
            dx = np.zeros_like(dx)
        T = oracle.pose_retr(T, dx, num_fix)
        if np.linalg.norm(dx) < delta_thresh:
            break
    return T, dx, it


def gauss_newton_calib(Twc, Xs, Cs, K, ii, jj, idx, valid_match, Q, height, width, pixel_border,
                       z_eps, sigma_pixel, sigma_depth, C_thresh, Q_thresh, max_iter,
                       delta_thresh, num_fix=1):
    """gauss_newton_calib_cuda (gn_kernels.cu:1545-1637) on local indices."""
    return gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid_match, Q, sigma_pixel, sigma_depth,
                             C_thresh, Q_thresh, max_iter, delta_thresh, num_fix,
                             calib=dict(K=np.asarray(K, np.float64), height=height, width=width,
                                        pixel_border=pixel_border, z_eps=z_eps))
