"""ORACLE — test infrastructure only.  numpy (float64) restatement of the
tracker's ray/dist Gauss-Newton (splatt3r_slam/tracker.py:156-214) used to
check the fused HIP normal-equation kernel (s3t_ray_dist_normal_eqs).

  act_Sim3 + Jacobian [I, -[p]x, p]   geometry.py:45-52
  point_to_ray_dist (+ Jacobian)      geometry.py:17-34
  huber                               nonlinear_optimizer.py:28-33
  solve / opt_pose_ray_dist_sim3      tracker.py:156-214
  project_calib (+ Jacobian)          geometry.py:63-104
  get_points_poses (calib branch)     tracker.py:142-151
  opt_pose_calib_sim3                 tracker.py:216-270
"""
from __future__ import annotations

import numpy as np


def quat_to_R(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def act_sim3(T, X):
    T = np.asarray(T, np.float64)
    R = quat_to_R(T[3:7])
    return T[7] * (X @ R.T) + T[:3]


def skew(p):
    z = np.zeros(p.shape[0])
    return np.stack([np.stack([z, -p[:, 2], p[:, 1]], -1),
                     np.stack([p[:, 2], z, -p[:, 0]], -1),
                     np.stack([-p[:, 1], p[:, 0], z], -1)], -2)


def point_to_ray_dist(X, jacobian=False):
    d = np.linalg.norm(X, axis=-1, keepdims=True)
    r = X / d
    rd = np.concatenate([r, d], -1)
    if not jacobian:
        return rd
    I = np.eye(3)[None]
    drdX = (I - r[:, :, None] * r[:, None, :]) / d[:, :, None]
    J = np.concatenate([drdX, r[:, None, :]], 1)
    return rd, J


def huber(r, k=1.345):
    a = np.abs(r)
    return np.where(a < k, 1.0, k / np.maximum(a, 1e-300))


def normal_equations(T, Xf, Xk, Q, valid, sigma_ray, sigma_dist, k):
    """H (7x7), g (7), cost for one GN iteration at relative pose T."""
    Xf = Xf.astype(np.float64)
    Xk = Xk.astype(np.float64)
    p = act_sim3(T, Xf)
    dXdT = np.concatenate([np.broadcast_to(np.eye(3), (p.shape[0], 3, 3)), -skew(p),
                           p[:, :, None]], -1)
    rd_f, D = point_to_ray_dist(p, jacobian=True)
    r = point_to_ray_dist(Xk) - rd_f
    J = -D @ dXdT
    sq = np.sqrt(Q.astype(np.float64).reshape(-1, 1)) * valid.reshape(-1, 1)
    si = np.concatenate([np.repeat(sq / sigma_ray, 3, 1), sq / sigma_dist], 1)
    rob = si * np.sqrt(huber(si * r, k))
    A = (rob[..., None] * J).reshape(-1, 7)
    b = (rob * r).reshape(-1, 1)
    return A.T @ A, (-A.T @ b)[:, 0], 0.5 * float((b * b).sum())


def project_calib(P, K, img_size, border=0.0, z_eps=0.0):
    """geometry.py:63-104 -> pz [n,3] (u, v, log z), dpz/dP [n,3,3], valid [n]."""
    K = np.asarray(K, np.float64)
    q = P @ K.T
    uv = q[:, :2] / q[:, 2:3]
    h, w = img_size
    z = P[:, 2]
    valid = ((uv[:, 0] > border) & (uv[:, 0] < w - 1 - border) &
             (uv[:, 1] > border) & (uv[:, 1] < h - 1 - border) & (z > z_eps))
    with np.errstate(divide="ignore", invalid="ignore"):
        logz = np.where(z > z_eps, np.log(np.where(z > z_eps, z, 1.0)), 0.0)
    fx, fy = K[0, 0], K[1, 1]
    zi = 1.0 / z
    D = np.zeros((P.shape[0], 3, 3))
    D[:, 0, 0] = fx * zi
    D[:, 1, 1] = fy * zi
    D[:, 0, 2] = -fx * P[:, 0] * zi * zi
    D[:, 1, 2] = -fy * P[:, 1] * zi * zi
    D[:, 2, 2] = zi
    return np.concatenate([uv, logz[:, None]], 1), D, valid


def calib_measurements(Xk, img_size, depth_eps):
    """tracker.py:145-151: pixel grid (u, v) + log z of the keyframe
    pointmap, zeroed where z <= depth_eps."""
    h, w = img_size
    v, u = np.divmod(np.arange(h * w), w)
    z = Xk[:, 2].astype(np.float64)
    ok = z > depth_eps
    meas = np.stack([u, v, np.log(np.where(ok, z, 1.0))], 1).astype(np.float64)
    meas[~ok] = 0.0
    return meas, ok


def normal_equations_calib(T, Xf, Xk, Q, valid, K, img_size, pixel_border, depth_eps,
                           sigma_pixel, sigma_depth, k):
    """One GN iteration of opt_pose_calib_sim3 (tracker.py:219-246):
    H (7x7), g (7), cost.  Xf: ray-constrained frame points gathered by
    idx_f2k; Xk: keyframe pointmap (its z gives the log-depth measurement)."""
    Xf = Xf.astype(np.float64)
    p = act_sim3(T, Xf)
    dXdT = np.concatenate([np.broadcast_to(np.eye(3), (p.shape[0], 3, 3)), -skew(p),
                           p[:, :, None]], -1)
    pz, D, vproj = project_calib(p, K, img_size, pixel_border, depth_eps)
    meas, vmeas = calib_measurements(Xk, img_size, depth_eps)
    r = meas - pz
    J = -D @ dXdT
    sq = np.sqrt(Q.astype(np.float64).reshape(-1, 1)) * valid.reshape(-1, 1)
    si = np.concatenate([np.repeat(sq / sigma_pixel, 2, 1), sq / sigma_depth], 1)
    si = si * (vproj & vmeas)[:, None]
    rob = si * np.sqrt(huber(si * r, k))
    A = (rob[..., None] * J).reshape(-1, 7)
    b = (rob * r).reshape(-1, 1)
    return A.T @ A, (-A.T @ b)[:, 0], 0.5 * float((b * b).sum())
