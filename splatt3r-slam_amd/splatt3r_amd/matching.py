"""Dense matching, mirroring splatt3r_slam/matching.py (same function names,
arguments and return values), with every stage on HIP kernels:

  prep_for_iter_proj (matching.py:25-49, image.py:5-38) -> s3m_prep_iter_proj
  iter_proj          (matching.py:60-67)               -> s3m_iter_proj
  occlusion check    (matching.py:68-76)               -> s3m_occlusion
  refine_matches     (matching.py:78-85)               -> s3m_refine_matches
  pixel_to_lin       (matching.py:13-15)               -> s3m_pixel_to_lin
"""
from __future__ import annotations

import os

import torch

from splatt3r_amd import _lib
from splatt3r_amd.config import config

# S3_REFINE_LANES=<n>: refine kernel variant for A/B runs (s3m_refine_set_lanes)
if "S3_REFINE_LANES" in os.environ:
    _lib.lib().s3m_refine_set_lanes(int(os.environ["S3_REFINE_LANES"]))


def pixel_to_lin(p1, w):
    return p1[..., 0] + (w * p1[..., 1])


def lin_to_pixel(idx_1_to_2, w):
    u = idx_1_to_2 % w
    v = idx_1_to_2 // w
    return torch.stack((u, v), dim=-1)


def prep_for_iter_proj(X11, X21, idx_1_to_2_init):
    """-> (rays_with_grad_img [b,h,w,9], pts3d_norm [b,hw,3], p_init [b,hw,2])"""
    _lib.require_cuda(X11, X21)
    b, h, w, _ = X11.shape
    X11 = X11.float().contiguous()
    X21 = X21.float().contiguous()
    rays = torch.empty(b, h, w, 9, device=X11.device, dtype=torch.float32)
    pts = torch.empty(b, h * w, 3, device=X11.device, dtype=torch.float32)
    p_init = torch.empty(b, h * w, 2, device=X11.device, dtype=torch.float32)
    idx = None
    if idx_1_to_2_init is not None:
        idx = idx_1_to_2_init.to(torch.int64).contiguous()
    _lib.call("s3m_prep_iter_proj", X11.data_ptr(), X21.data_ptr(), _lib.ptr(idx),
              rays.data_ptr(), pts.data_ptr(), p_init.data_ptr(), b, h, w,
              _lib.stream(X11.device))
    return rays, pts, p_init


def refine_matches(D11, D21, p1, radius, dilation_max):
    """s3m_refine_matches: contiguous fp16 D11 [b,h,w,F] / D21 [b,n,F],
    int64 p1 [b,n,2] -> p1_new."""
    b, h, w, f = D11.shape
    n = D21.shape[1]
    p1_new = torch.empty_like(p1)
    _lib.call("s3m_refine_matches", D11.data_ptr(), D21.data_ptr(), p1.data_ptr(),
              p1_new.data_ptr(), b, h, w, n, f, radius, dilation_max, _lib.stream(D11.device))
    return p1_new


def match(X11, X21, D11, D21, idx_1_to_2_init=None):
    idx_1_to_2, valid_match2 = match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init)
    return idx_1_to_2, valid_match2


def match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=None):
    cfg = cfg or config["matching"]
    b, h, w = X21.shape[:3]
    dev = X11.device
    stream = _lib.stream(dev)
    X11c = X11.float().contiguous()
    X21c = X21.float().contiguous()
    rays, pts, p_init = prep_for_iter_proj(X11c, X21c, idx_1_to_2_init)
    n = h * w
    p = torch.empty(b, n, 2, device=dev, dtype=torch.float32)
    conv = torch.empty(b, n, device=dev, dtype=torch.bool)
    _lib.call("s3m_iter_proj", rays.data_ptr(), pts.data_ptr(), p_init.data_ptr(),
              p.data_ptr(), conv.data_ptr(), b, h, w, n, int(cfg["max_iter"]),
              float(cfg["lambda_init"]), float(cfg["convergence_thresh"]), stream)
    p1 = torch.empty(b, n, 2, device=dev, dtype=torch.int64)
    valid = torch.empty(b, n, device=dev, dtype=torch.bool)
    _lib.call("s3m_occlusion", p.data_ptr(), conv.data_ptr(), X11c.data_ptr(), X21c.data_ptr(),
              p1.data_ptr(), valid.data_ptr(), b, h, w, float(cfg["dist_thresh"]), stream)
    if cfg["radius"] > 0:
        D11h = D11 if D11.dtype == torch.float16 else D11.half()
        D21h = D21 if D21.dtype == torch.float16 else D21.half()
        D11h = D11h.contiguous()
        D21h = D21h.reshape(b, n, -1).contiguous()
        p1 = refine_matches(D11h, D21h, p1, int(cfg["radius"]), int(cfg["dilation_max"]))
    idx = torch.empty(b, n, device=dev, dtype=torch.int64)
    _lib.call("s3m_pixel_to_lin", p1.data_ptr(), idx.data_ptr(), b * n, w, stream)
    return idx, valid.unsqueeze(-1)
