"""ORACLE — test infrastructure only.

CPU restatements of the reference algorithms on the hot path, used as the
parity checker.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package; the product path
(splatt3r-slam_amd/) never does.

  sim3_ref.c      <- splatt3r_slam/backend/src/gn_kernels.cu:171-452
  matching_ref.c  <- splatt3r_slam/backend/src/matching_kernels.cu, matching.py, image.py
  raster_ref.c    <- canonical graphdeco 3DGS rasterizer (external submodule, see header)
  tracker_ref.py  <- splatt3r_slam/tracker.py / geometry.py / nonlinear_optimizer.py
  net_ref.py      <- torch fp32 restatement of the MASt3RGaussians forward
  prng.py         <- portable splitmix64 weight generator (no reference counterpart)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    r = subprocess.run(["make", "-s", "-C", HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"oracle build failed:\n{r.stdout}\n{r.stderr}")
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or any(
                os.path.getmtime(os.path.join(HERE, f)) > os.path.getmtime(LIB)
                for f in os.listdir(HERE) if f.endswith(".c")):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ---------------------------------------------------------------- Sim3 ----
def sim3_act(T, X):
    T = _c(T, np.float32).reshape(-1, 8)
    X = _c(X, np.float32).reshape(-1, 3)
    Y = np.empty_like(X)
    lib().oracle_sim3_act_batch(_p(T), ctypes.c_int64(T.shape[0]), _p(X), _p(Y),
                                ctypes.c_int64(X.shape[0]))
    return Y


def _unary(fn, a, din, dout):
    a = _c(a, np.float32).reshape(-1, din)
    out = np.empty((a.shape[0], dout), np.float32)
    getattr(lib(), fn)(_p(a), _p(out), ctypes.c_int64(a.shape[0]))
    return out


def sim3_inv(a):
    return _unary("oracle_sim3_inv_batch", a, 8, 8)


def sim3_exp(xi):
    return _unary("oracle_sim3_exp_batch", xi, 7, 8)


def sim3_mul(a, b):
    a = _c(a, np.float32).reshape(-1, 8)
    b = _c(b, np.float32).reshape(-1, 8)
    out = np.empty_like(a)
    lib().oracle_sim3_mul_batch(_p(a), _p(b), _p(out), ctypes.c_int64(a.shape[0]))
    return out


def sim3_retr(T, xi):
    T = _c(T, np.float32).reshape(-1, 8)
    xi = _c(xi, np.float32).reshape(-1, 7)
    out = np.empty_like(T)
    lib().oracle_sim3_retr_batch(_p(T), _p(xi), _p(out), ctypes.c_int64(T.shape[0]))
    return out


def pose_retr(poses, dx, num_fix):
    poses = _c(poses, np.float32).copy()
    dx = _c(dx, np.float32)
    lib().oracle_pose_retr(_p(poses), _p(dx), ctypes.c_int64(poses.shape[0]),
                           ctypes.c_int64(num_fix))
    return poses


# ------------------------------------------------------------ matching ----
def f32_to_f16_bits(x):
    x = _c(x, np.float32).ravel()
    f = lib().oracle_f32_to_f16
    f.restype = ctypes.c_uint16
    f.argtypes = [ctypes.c_float]
    return np.array([f(float(v)) for v in x], np.uint16)


def iter_proj(rays, pts, p_init, max_iter, lambda_init, cost_thresh):
    rays = _c(rays, np.float32)
    pts = _c(pts, np.float32)
    p_init = _c(p_init, np.float32)
    b, h, w, _ = rays.shape
    n = p_init.shape[1]
    p_new = np.zeros((b, n, 2), np.float32)
    conv = np.zeros((b, n), np.uint8)
    lib().oracle_iter_proj(_p(rays), _p(pts), _p(p_init), _p(p_new), _p(conv), b, h, w, n,
                           int(max_iter), ctypes.c_float(lambda_init),
                           ctypes.c_float(cost_thresh))
    return p_new, conv.astype(bool)


def refine_matches(D11_f16, D21_f16, p1, radius, dilation_max):
    D11 = _c(D11_f16, np.float16).view(np.uint16)
    D21 = _c(D21_f16, np.float16).view(np.uint16)
    p1 = _c(p1, np.int64)
    b, h, w, f = D11.shape
    n = p1.shape[1]
    out = np.zeros((b, n, 2), np.int64)
    lib().oracle_refine_matches(_p(D11), _p(D21), _p(p1), _p(out), b, h, w, n, f,
                                int(radius), int(dilation_max))
    return out


def prep_iter_proj(X11, X21, idx_init=None):
    X11 = _c(X11, np.float32)
    X21 = _c(X21, np.float32)
    b, h, w, _ = X11.shape
    rays = np.zeros((b, h, w, 9), np.float32)
    pts = np.zeros((b, h * w, 3), np.float32)
    p_init = np.zeros((b, h * w, 2), np.float32)
    idx = None if idx_init is None else _c(idx_init, np.int64)
    lib().oracle_prep_iter_proj(_p(X11), _p(X21), None if idx is None else _p(idx),
                                _p(rays), _p(pts), _p(p_init), b, h, w)
    return rays, pts, p_init


def occlusion(p, conv, X11, X21, dist_thresh):
    p = _c(p, np.float32)
    conv = _c(conv, np.uint8)
    X11 = _c(X11, np.float32)
    X21 = _c(X21, np.float32)
    b, h, w, _ = X11.shape
    p1 = np.zeros((b, h * w, 2), np.int64)
    valid = np.zeros((b, h * w), np.uint8)
    lib().oracle_occlusion(_p(p), _p(conv), _p(X11), _p(X21), _p(p1), _p(valid), b, h, w,
                           ctypes.c_float(dist_thresh))
    return p1, valid.astype(bool)


MATCH_CFG = dict(max_iter=10, lambda_init=1e-8, convergence_thresh=1e-6, dist_thresh=1e-1,
                 radius=3, dilation_max=5)  # config/base.yaml:8-14


def match(X11, X21, D11, D21, idx_init=None, cfg=MATCH_CFG):
    """Full matching.match_iterative_proj restated (matching.py:52-90)."""
    b, h, w, _ = np.shape(X11)
    rays, pts, p_init = prep_iter_proj(X11, X21, idx_init)
    p, conv = iter_proj(rays, pts, p_init, cfg["max_iter"], cfg["lambda_init"],
                        cfg["convergence_thresh"])
    p1, valid = occlusion(p, conv, X11, X21, cfg["dist_thresh"])
    if cfg["radius"] > 0:
        D11h = np.asarray(D11, np.float32).astype(np.float16)
        D21h = np.asarray(D21, np.float32).astype(np.float16).reshape(b, h * w, -1)
        p1 = refine_matches(D11h, D21h, p1, cfg["radius"], cfg["dilation_max"])
    idx = p1[..., 0] + w * p1[..., 1]
    return idx, valid[..., None]


# ---------------------------------------------------------- rasterizer ----
class _OracleCam(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int), ("W", ctypes.c_int), ("tanfovx", ctypes.c_float),
                ("tanfovy", ctypes.c_float), ("scale_modifier", ctypes.c_float),
                ("D", ctypes.c_int), ("bg", ctypes.c_float * 3),
                ("viewmatrix", ctypes.c_float * 16), ("projmatrix", ctypes.c_float * 16),
                ("campos", ctypes.c_float * 3)]


def raster(settings: dict, means3D, opacities, shs=None, colors_precomp=None, scales=None,
           rotations=None, cov3D_precomp=None, dL_dout=None, nthreads=8, exp="kernel"):
    """graphdeco forward (+ backward if dL_dout) on the CPU.

    exp = "kernel": the blend's exponential is the HIP kernels' fixed-sequence
    fexp (bit-comparable forward); "libm": glibc expf, the canonical
    graphdeco `exp(power)` (the HIP image then agrees within a tolerance).

    settings: dict with image_height, image_width, tanfovx, tanfovy, bg(3),
    scale_modifier, viewmatrix(16, memory order of the torch arg),
    projmatrix(16), sh_degree, campos(3).
    Returns dict(color [3,H,W], radii [P], num_rendered, and grads if asked).
    """
    H, W = int(settings["image_height"]), int(settings["image_width"])
    cam = _OracleCam()
    cam.H, cam.W = H, W
    cam.tanfovx, cam.tanfovy = float(settings["tanfovx"]), float(settings["tanfovy"])
    cam.scale_modifier = float(settings.get("scale_modifier", 1.0))
    cam.D = int(settings["sh_degree"])
    for k, n in (("bg", 3), ("viewmatrix", 16), ("projmatrix", 16), ("campos", 3)):
        vals = np.asarray(settings[k], np.float32).ravel()
        arr = getattr(cam, k)
        for i in range(n):
            arr[i] = float(vals[i])
    m = _c(means3D, np.float32).reshape(-1, 3)
    P = m.shape[0]
    op = _c(opacities, np.float32).reshape(-1)
    sh = None if shs is None else _c(shs, np.float32).reshape(P, -1, 3)
    M = 0 if sh is None else sh.shape[1]
    col = None if colors_precomp is None else _c(colors_precomp, np.float32).reshape(P, 3)
    sc = None if scales is None else _c(scales, np.float32).reshape(P, 3)
    rot = None if rotations is None else _c(rotations, np.float32).reshape(P, 4)
    cov = None if cov3D_precomp is None else _c(cov3D_precomp, np.float32).reshape(P, 6)
    color = np.zeros((3, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    out = dict(color=color, radii=radii)
    g = None
    if dL_dout is not None:
        g = _c(dL_dout, np.float32).reshape(3, H, W)
        out.update(dL_dmeans2D=np.zeros((P, 3), np.float32), dL_dconic=np.zeros((P, 4), np.float32),
                   dL_dopacity=np.zeros(P, np.float32), dL_dcolors=np.zeros((P, 3), np.float32),
                   dL_dmeans3D=np.zeros((P, 3), np.float32), dL_dcov3D=np.zeros((P, 6), np.float32),
                   dL_dsh=np.zeros((P, max(M, 1), 3), np.float32))
    q = lambda a: None if a is None else _p(a)
    f = lib().oracle_raster
    f.restype = ctypes.c_int64
    gk = ("dL_dmeans2D", "dL_dconic", "dL_dopacity", "dL_dcolors", "dL_dmeans3D", "dL_dcov3D",
          "dL_dsh")
    if exp not in ("kernel", "libm"):
        raise ValueError(f"exp must be 'kernel' or 'libm', not {exp!r}")
    lib().oracle_raster_set_exp(int(exp == "libm"))
    try:
        R = f(ctypes.byref(cam), ctypes.c_int64(P), M, _p(m), q(sc), q(rot), q(cov), q(sh),
              q(col), _p(op), _p(color), _p(radii), q(g),
              *[q(out[k]) if g is not None else None for k in gk], nthreads)
    finally:
        lib().oracle_raster_set_exp(0)
    out["num_rendered"] = int(R)
    return out
