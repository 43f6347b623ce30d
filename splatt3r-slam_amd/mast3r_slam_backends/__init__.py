"""Drop-in `mast3r_slam_backends` (reference pybind module,
splatt3r_slam/backend/src/gn.cpp:116-122) over libsplatt3r_hip.so.

Same names, argument order, return lists and errors as the reference:
  iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init,
            cost_thresh) -> [p_new f32 [b,n,2], converged bool [b,n]]
  refine_matches(D11 f16 [b,h,w,F], D21 f16 [b,n,F], p1 i64 [b,n,2], radius,
                 dilation_max) -> [p1_new i64 [b,n,2]]
Non-contiguous inputs raise RuntimeError (reference CHECK_CONTIGUOUS).
  gauss_newton_rays(Twc f32 [N,8] (updated in place), Xs f32 [N,hw,3],
                    Cs f32 [N,hw,1], ii i64 [E], jj i64 [E], idx_ii2jj i64 [E,hw],
                    valid_match bool [E,hw,1], Q f32 [E,hw,1], sigma_ray, sigma_dist,
                    C_thresh, Q_thresh, max_iter, delta_thresh) -> [dx f32 [N-1,7]]
    (gn.cpp:28-52 -> gn_kernels.cu:1139-1227; include/s3g.h; the whole
    iteration loop runs on the device, pose 0 fixed as in the reference).
  gauss_newton_calib(Twc, Xs, Cs, K f32 [3,3], ii, jj, idx_ii2jj, valid_match, Q,
                     height, width, pixel_border, z_eps, sigma_pixel, sigma_depth,
                     C_thresh, Q_thresh, max_iter, delta_thresh) -> [dx f32 [N-1,7]]
    (gn.cpp:54-80 -> gn_kernels.cu:1545-1637; same device loop as the rays solve)
"""
from __future__ import annotations

import ctypes

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
    from splatt3r_amd.matching import refine_matches as _refine
    return [_refine(D11, D21, p1, int(radius), int(dilation_max))]


_lib.register({
    "s3g_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                              ctypes.c_int]),
    "s3g_ray_system": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "s3g_calib_system": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "s3g_gauss_newton_calib": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                              ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                              ctypes.c_float, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                              ctypes.c_void_p]),
    "s3g_gauss_newton_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                             ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                             ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]),
})

NUM_FIX = 1   # gn_kernels.cu:1156


def _gn_inputs(name, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q):
    _lib.require_cuda(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q)
    _lib.require_contig(name, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q)
    N, hw = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    if Twc.shape != (N, 8) or Cs.shape[:2] != (N, hw) or jj.shape != (E,):
        raise RuntimeError(f"{name}: pose/point shape mismatch")
    if idx_ii2jj.shape[:2] != (E, hw) or valid_match.shape[:2] != (E, hw) or \
            Q.shape[:2] != (E, hw):
        raise RuntimeError(f"{name}: edge shape mismatch")
    for t in (Twc, Xs, Cs, Q):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{name}: expected float32 poses/points/confidences")
    if idx_ii2jj.dtype != torch.int64 or valid_match.dtype != torch.bool:
        raise RuntimeError(f"{name}: idx_ii2jj must be int64 and valid_match bool")
    # create_inds (gn_kernels.cu:160-170): global keyframe ids -> rows of Twc
    unique = torch.unique(torch.cat([ii, jj]), sorted=True)
    if unique.numel() != N:
        raise RuntimeError(f"{name}: Twc/Xs rows ({N}) must be the {unique.numel()} unique "
                           "keyframes of ii/jj, in sorted order")
    ii_l = torch.searchsorted(unique, ii).to(torch.int32).contiguous()
    jj_l = torch.searchsorted(unique, jj).to(torch.int32).contiguous()
    return N, hw, E, ii_l, jj_l


def gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_ray, sigma_dist,
                      C_thresh, Q_thresh, max_iter, delta_thresh):
    N, hw, E, ii_l, jj_l = _gn_inputs("gauss_newton_rays", Twc, Xs, Cs, ii, jj, idx_ii2jj,
                                      valid_match, Q)
    dev = Twc.device
    L = _lib.lib()
    ws = torch.empty(int(L.s3g_workspace_bytes(N, E, hw, NUM_FIX)), dtype=torch.uint8,
                     device=dev)
    dx = torch.zeros(N - NUM_FIX, 7, device=dev, dtype=torch.float32)
    stats = (ctypes.c_float * 2)()
    _lib.call("s3g_gauss_newton_rays", Twc.data_ptr(), N, Xs.data_ptr(), Cs.data_ptr(), hw,
              ii_l.data_ptr(), jj_l.data_ptr(), E, idx_ii2jj.data_ptr(), valid_match.data_ptr(),
              Q.data_ptr(), float(sigma_ray), float(sigma_dist), float(C_thresh),
              float(Q_thresh), int(max_iter), float(delta_thresh), NUM_FIX, ws.data_ptr(),
              dx.data_ptr(), stats, _lib.stream(dev))
    gauss_newton_rays.last_stats = (int(stats[0]), float(stats[1]))
    return [dx]


def ray_system(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_ray, sigma_dist, C_thresh,
               Q_thresh):
    """One iteration's dense normal equations (H, b) in fp64 (diagnostics
    and tests; the reference keeps them inside gauss_newton_rays_cuda)."""
    N, hw, E, ii_l, jj_l = _gn_inputs("ray_system", Twc, Xs, Cs, ii, jj, idx_ii2jj,
                                      valid_match, Q)
    dev = Twc.device
    n = 7 * (N - NUM_FIX)
    L = _lib.lib()
    ws = torch.empty(int(L.s3g_workspace_bytes(N, E, hw, NUM_FIX)), dtype=torch.uint8,
                     device=dev)
    H = torch.empty(n, n, device=dev, dtype=torch.float64)
    b = torch.empty(n, device=dev, dtype=torch.float64)
    _lib.call("s3g_ray_system", Twc.data_ptr(), N, Xs.data_ptr(), Cs.data_ptr(), hw,
              ii_l.data_ptr(), jj_l.data_ptr(), E, idx_ii2jj.data_ptr(), valid_match.data_ptr(),
              Q.data_ptr(), float(sigma_ray), float(sigma_dist), float(C_thresh),
              float(Q_thresh), NUM_FIX, ws.data_ptr(), H.data_ptr(), b.data_ptr(),
              _lib.stream(dev))
    return H, b


def _calib_K(name, K):
    _lib.require_cuda(K)
    if tuple(K.shape) != (3, 3) or K.dtype != torch.float32:
        raise RuntimeError(f"{name}: K must be float32 [3,3]")
    return K.contiguous()


def gauss_newton_calib(Twc, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q, height, width,
                       pixel_border, z_eps, sigma_pixel, sigma_depth, C_thresh, Q_thresh,
                       max_iter, delta_thresh):
    N, hw, E, ii_l, jj_l = _gn_inputs("gauss_newton_calib", Twc, Xs, Cs, ii, jj, idx_ii2jj,
                                      valid_match, Q)
    K = _calib_K("gauss_newton_calib", K)
    dev = Twc.device
    L = _lib.lib()
    ws = torch.empty(int(L.s3g_workspace_bytes(N, E, hw, NUM_FIX)), dtype=torch.uint8,
                     device=dev)
    dx = torch.zeros(N - NUM_FIX, 7, device=dev, dtype=torch.float32)
    stats = (ctypes.c_float * 2)()
    _lib.call("s3g_gauss_newton_calib", Twc.data_ptr(), N, Xs.data_ptr(), Cs.data_ptr(), hw,
              K.data_ptr(), ii_l.data_ptr(), jj_l.data_ptr(), E, idx_ii2jj.data_ptr(),
              valid_match.data_ptr(), Q.data_ptr(), int(height), int(width), int(pixel_border),
              float(z_eps), float(sigma_pixel), float(sigma_depth), float(C_thresh),
              float(Q_thresh), int(max_iter), float(delta_thresh), NUM_FIX, ws.data_ptr(),
              dx.data_ptr(), stats, _lib.stream(dev))
    gauss_newton_calib.last_stats = (int(stats[0]), float(stats[1]))
    return [dx]


def calib_system(Twc, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q, height, width, pixel_border,
                 z_eps, sigma_pixel, sigma_depth, C_thresh, Q_thresh):
    """One iteration's dense (H, b) of the calibrated solve (diagnostics/tests)."""
    N, hw, E, ii_l, jj_l = _gn_inputs("calib_system", Twc, Xs, Cs, ii, jj, idx_ii2jj,
                                      valid_match, Q)
    K = _calib_K("calib_system", K)
    dev = Twc.device
    n = 7 * (N - NUM_FIX)
    L = _lib.lib()
    ws = torch.empty(int(L.s3g_workspace_bytes(N, E, hw, NUM_FIX)), dtype=torch.uint8,
                     device=dev)
    H = torch.empty(n, n, device=dev, dtype=torch.float64)
    b = torch.empty(n, device=dev, dtype=torch.float64)
    _lib.call("s3g_calib_system", Twc.data_ptr(), N, Xs.data_ptr(), Cs.data_ptr(), hw,
              K.data_ptr(), ii_l.data_ptr(), jj_l.data_ptr(), E, idx_ii2jj.data_ptr(),
              valid_match.data_ptr(), Q.data_ptr(), int(height), int(width), int(pixel_border),
              float(z_eps), float(sigma_pixel), float(sigma_depth), float(C_thresh),
              float(Q_thresh), NUM_FIX, ws.data_ptr(), H.data_ptr(), b.data_ptr(),
              _lib.stream(dev))
    return H, b
