"""Drop-in `mast3r_slam_backends` (reference pybind module,
splatt3r_slam/backend/src/gn.cpp:116-122) over libsplatt3r_hip.so.

Same names, argument order, return lists and errors as the reference:
  iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init,
            cost_thresh) -> [p_new f32 [b,n,2], converged bool [b,n]]
  refine_matches(D11 f16 [b,h,w,F], D21 f16 [b,n,F], p1 i64 [b,n,2], radius,
                 dilation_max) -> [p1_new i64 [b,n,2]]
Non-contiguous inputs raise RuntimeError (reference CHECK_CONTIGUOUS).
gauss_newton_rays / gauss_newton_calib are the backend GN solver
(scheduled after the hot path): they raise
NotImplementedError until that row lands.
"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib


def iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh):
    _lib.require_cuda(rays_img_with_grad, pts_3d_norm, p_init)
    _lib.require_contig("iter_proj", rays_img_with_grad, pts_3d_norm, p_init)
    b, h, w, c = rays_img_with_grad.shape
    if c != 9:
        raise RuntimeError("iter_proj: rays_img_with_grad must have 9 channels")
    n = p_init.shape[1]
    if pts_3d_norm.shape != (b, n, 3) or p_init.shape != (b, n, 2):
        raise RuntimeError("iter_proj: shape mismatch")
    for t in (rays_img_with_grad, pts_3d_norm, p_init):
        if t.dtype != torch.float32:
            raise RuntimeError("iter_proj: expected float32 inputs")
    p_new = torch.zeros(b, n, 2, device=p_init.device, dtype=torch.float32)
    converged = torch.zeros(b, n, device=p_init.device, dtype=torch.bool)
    _lib.call("s3m_iter_proj", rays_img_with_grad.data_ptr(), pts_3d_norm.data_ptr(),
              p_init.data_ptr(), p_new.data_ptr(), converged.data_ptr(), b, h, w, n,
              int(max_iter), float(lambda_init), float(cost_thresh), _lib.stream(p_init.device))
    return [p_new, converged]


def refine_matches(D11, D21, p1, radius, dilation_max):
    _lib.require_cuda(D11, D21, p1)
    _lib.require_contig("refine_matches", D11, D21, p1)
    if D11.dtype != torch.float16 or D21.dtype != torch.float16:
        raise RuntimeError("refine_matches: descriptors must be float16 (matching.py:80-81)")
    if p1.dtype != torch.int64:
        raise RuntimeError("refine_matches: p1 must be int64")
    b, h, w, f = D11.shape
    n = p1.shape[1]
    if D21.shape != (b, n, f) or p1.shape != (b, n, 2):
        raise RuntimeError("refine_matches: shape mismatch")
    p1_new = torch.zeros(b, n, 2, device=p1.device, dtype=torch.int64)
    _lib.call("s3m_refine_matches", D11.data_ptr(), D21.data_ptr(), p1.data_ptr(),
              p1_new.data_ptr(), b, h, w, n, f, int(radius), int(dilation_max),
              _lib.stream(p1.device))
    return [p1_new]


def gauss_newton_rays(*args, **kwargs):
    raise NotImplementedError(
        "gauss_newton_rays: backend GN solver is SURVEY.md §8(f) row f1 (not yet built)")


def gauss_newton_calib(*args, **kwargs):
    raise NotImplementedError(
        "gauss_newton_calib: backend GN solver is SURVEY.md §8(f) row f1 (not yet built)")
