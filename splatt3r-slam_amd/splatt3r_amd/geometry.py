"""Calibrated-mode geometry glue (splatt3r_slam/geometry.py:37-42, 107-123).

`constrain_points_to_ray` keeps each point's depth and moves it onto the
ray of its own pixel: P = z * ((u - cx) / fx, (v - cy) / fy, 1).  Plain
elementwise tensor glue on the caller's device (the reference's is too);
the solve it feeds is the HIP kernel behind
mast3r_slam_backends.gauss_newton_calib.
"""
from __future__ import annotations

import torch


def get_pixel_coords(b, img_size, device, dtype):
    """geometry.py:118-123: [b, h, w, 2] grid of (u, v)."""
    h, w = img_size
    u, v = torch.meshgrid(torch.arange(w), torch.arange(h), indexing="xy")
    uv = torch.stack((u, v), dim=-1).unsqueeze(0).repeat(b, 1, 1, 1)
    return uv.to(device=device, dtype=dtype)


def backproject(p, z, K):
    """geometry.py:107-115."""
    tmp1 = (p[..., 0] - K[0, 2]) / K[0, 0]
    tmp2 = (p[..., 1] - K[1, 2]) / K[1, 1]
    dP_dz = torch.empty(p.shape[:-1] + (3, 1), device=z.device, dtype=K.dtype)
    dP_dz[..., 0, 0] = tmp1
    dP_dz[..., 1, 0] = tmp2
    dP_dz[..., 2, 0] = 1.0
    return torch.squeeze(z[..., None, :] * dP_dz, dim=-1)


def constrain_points_to_ray(img_size, Xs, K):
    """geometry.py:37-42: Xs [b, h*w, 3] -> points on their pixel rays."""
    uv = get_pixel_coords(Xs.shape[0], img_size, device=Xs.device, dtype=Xs.dtype).view(
        *Xs.shape[:-1], 2)
    return backproject(uv, Xs[..., 2:3], K)
