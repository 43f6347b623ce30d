"""ORACLE — test infrastructure only.  numpy (float64) restatement of the
tracker's ray/dist Gauss-Newton (splatt3r_slam/tracker.py:156-214) used to
check the fused HIP normal-equation kernel (s3t_ray_dist_normal_eqs).

  act_Sim3 + Jacobian [I, -[p]x, p]   geometry.py:45-52
  point_to_ray_dist (+ Jacobian)      geometry.py:17-34
  huber                               nonlinear_optimizer.py:28-33
  solve / opt_pose_ray_dist_sim3      tracker.py:156-214
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
