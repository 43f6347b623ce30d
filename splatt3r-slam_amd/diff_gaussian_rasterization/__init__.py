"""Drop-in `diff_gaussian_rasterization` over the HIP tile rasterizer of
libsplatt3r_hip.so (include/gsr.h).

Same public surface as the module the reference imports
(splatt3r_core/src/pixelsplat_src/cuda_splatting.py:4-8,100-125;
splatt3r_slam/visualization.py:35-45,563-594):

  GaussianRasterizationSettings(image_height, image_width, tanfovx, tanfovy,
      bg, scale_modifier, viewmatrix, projmatrix, sh_degree, campos,
      prefiltered, debug)                              (a NamedTuple)
  GaussianRasterizer(settings)(means3D, means2D, opacities, shs=None,
      colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None)
      -> (color [3,H,W] f32, radii [P] i32)
  GaussianRasterizer.markVisible(positions) -> bool [P]

Exactly one of shs / colors_precomp and exactly one of (scales, rotations) /
cov3D_precomp must be given, with the reference's exception messages.
Backward through torch.autograd returns the gradients in the reference
order (means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
cov3Ds_precomp).  There is no CPU path: tensors must live on the GPU.
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple

import torch
import torch.nn as nn

from splatt3r_amd import _lib

P_ = ctypes.c_void_p


class _GsrSettings(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int),
        ("image_width", ctypes.c_int),
        ("tanfovx", ctypes.c_float),
        ("tanfovy", ctypes.c_float),
        ("scale_modifier", ctypes.c_float),
        ("sh_degree", ctypes.c_int),
        ("prefiltered", ctypes.c_int),
        ("debug", ctypes.c_int),
        ("bg", P_),
        ("viewmatrix", P_),
        ("projmatrix", P_),
        ("campos", P_),
    ]


_SP = ctypes.POINTER(_GsrSettings)
_lib.register({
    "gsr_geom_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gsr_image_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "gsr_binning_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gsr_preprocess": (ctypes.c_int, [_SP, ctypes.c_int64, ctypes.c_int] + [P_] * 7 +
                       [P_, P_, ctypes.POINTER(ctypes.c_int64), P_]),
    "gsr_render": (ctypes.c_int, [_SP, ctypes.c_int64, ctypes.c_int64, P_, P_, P_, P_, P_, P_]),
    "gsr_backward": (ctypes.c_int, [_SP, ctypes.c_int64, ctypes.c_int, ctypes.c_int64] +
                     [P_] * 8 + [P_, P_, P_, P_] + [P_] * 9 + [P_]),
    "gsr_mark_visible": (ctypes.c_int, [ctypes.c_int64, P_, P_, P_, P_, P_]),
    "gsr_forward_deferred": (ctypes.c_int, [_SP, ctypes.c_int64, ctypes.c_int] + [P_] * 7 +
                             [P_, P_, P_, ctypes.c_int64, ctypes.c_int, P_, P_, P_, P_]),
    "gsr_set_timing": (None, [ctypes.c_int]),
    "gsr_set_binning": (None, [ctypes.c_int]),
    "gsr_last_timing": (ctypes.c_int, [P_, ctypes.c_int]),
})


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool = False


def _dev_f32(t, device):
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t, dtype=torch.float32)
    return t.detach().to(device=device, dtype=torch.float32).contiguous()


def _settings_struct(rs: GaussianRasterizationSettings, device):
    keep = [_dev_f32(rs.bg, device), _dev_f32(rs.viewmatrix, device),
            _dev_f32(rs.projmatrix, device), _dev_f32(rs.campos, device)]
    s = _GsrSettings(int(rs.image_height), int(rs.image_width), float(rs.tanfovx),
                     float(rs.tanfovy), float(rs.scale_modifier), int(rs.sh_degree),
                     int(bool(rs.prefiltered)), int(bool(rs.debug)),
                     keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr(),
                     keep[3].data_ptr())
    return s, keep


def _opt(t):
    return None if t is None or t.numel() == 0 else t


def _f32c(t):
    return None if t is None else t.detach().to(torch.float32).contiguous()


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales,
                                     rotations, cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings):
        if means3D.ndimension() != 2 or means3D.size(1) != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        _lib.require_cuda(means3D)
        dev = means3D.device
        P = means3D.shape[0]
        H, W = int(raster_settings.image_height), int(raster_settings.image_width)
        sh, colors_precomp = _opt(sh), _opt(colors_precomp)
        scales, rotations, cov3Ds_precomp = _opt(scales), _opt(rotations), _opt(cov3Ds_precomp)
        m3 = _f32c(means3D)
        shc = _f32c(sh)
        M = 0 if shc is None else (shc.shape[1] if shc.dim() == 3 else shc.shape[-1] // 3)
        col = _f32c(colors_precomp)
        op = _f32c(opacities)
        sc, rot, cov = _f32c(scales), _f32c(rotations), _f32c(cov3Ds_precomp)
        s, keep = _settings_struct(raster_settings, dev)
        stream = _lib.stream(dev)
        L = _lib.lib()
        # every pixel / radius is written by gsr_render / gsr_preprocess
        color = torch.empty(3, H, W, device=dev, dtype=torch.float32)
        radii = torch.empty(P, device=dev, dtype=torch.int32)
        geom = torch.empty(int(L.gsr_geom_bytes(P)), device=dev, dtype=torch.uint8)
        img = torch.empty(int(L.gsr_image_bytes(H, W)), device=dev, dtype=torch.uint8)
        nr = ctypes.c_int64(0)
        if P > 0:
            _lib.check(L.gsr_preprocess(ctypes.byref(s), P, M, m3.data_ptr(), _lib.ptr(sc),
                                        _lib.ptr(rot), _lib.ptr(cov), _lib.ptr(shc),
                                        _lib.ptr(col), _lib.ptr(op), radii.data_ptr(),
                                        geom.data_ptr(), ctypes.byref(nr), stream),
                       "gsr_preprocess")
        R = nr.value
        binning = torch.empty(int(L.gsr_binning_bytes(R)), device=dev, dtype=torch.uint8)
        _lib.check(L.gsr_render(ctypes.byref(s), P, R, radii.data_ptr(), geom.data_ptr(),
                                binning.data_ptr(), img.data_ptr(), color.data_ptr(), stream),
                   "gsr_render")
        ctx.raster_settings = raster_settings
        ctx.num_rendered = R
        global last_num_rendered
        last_num_rendered = R
        ctx.M = M
        ctx.has = (shc is not None, col is not None, sc is not None, cov is not None)
        ctx.save_for_backward(m3, shc if shc is not None else m3.new_empty(0),
                              col if col is not None else m3.new_empty(0), op,
                              sc if sc is not None else m3.new_empty(0),
                              rot if rot is not None else m3.new_empty(0),
                              cov if cov is not None else m3.new_empty(0),
                              radii, geom, binning, img)
        ctx.mark_non_differentiable(radii)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii):
        m3, shc, col, op, sc, rot, cov, radii, geom, binning, img = ctx.saved_tensors
        has_sh, has_col, has_sc, has_cov = ctx.has
        shc = shc if has_sh else None
        col = col if has_col else None
        sc = sc if has_sc else None
        rot = rot if has_sc else None
        cov = cov if has_cov else None
        dev = m3.device
        P, M, R = m3.shape[0], ctx.M, ctx.num_rendered
        s, keep = _settings_struct(ctx.raster_settings, dev)
        g = grad_out_color.detach().to(torch.float32).contiguous()
        # gsr_backward zeroes every gradient output itself (one launch)
        z = lambda *shape: torch.empty(*shape, device=dev, dtype=torch.float32)
        dm2, dconic, dop, dcol = z(P, 3), z(P, 4), z(P, 1), z(P, 3)
        dm3, dcov = z(P, 3), z(P, 6)
        dsh = z(P, M, 3) if has_sh else None
        dsc = z(P, 3) if has_sc else None
        drot = z(P, 4) if has_sc else None
        _lib.check(_lib.lib().gsr_backward(
            ctypes.byref(s), P, M, R, m3.data_ptr(), _lib.ptr(sc), _lib.ptr(rot), _lib.ptr(cov),
            _lib.ptr(shc), _lib.ptr(col), op.data_ptr(), radii.data_ptr(), geom.data_ptr(),
            binning.data_ptr(), img.data_ptr(), g.data_ptr(), dm2.data_ptr(), dconic.data_ptr(),
            dop.data_ptr(), dcol.data_ptr(), dm3.data_ptr(), dcov.data_ptr(), _lib.ptr(dsh),
            _lib.ptr(dsc), _lib.ptr(drot), _lib.stream(dev)), "gsr_backward")
        return (dm3, dm2, dsh, dcol if has_col else None, dop, dsc, drot,
                dcov if has_cov else None, None)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            rs = self.raster_settings
            pos = _f32c(positions)
            _lib.require_cuda(pos)
            vm = _dev_f32(rs.viewmatrix, pos.device)
            pm = _dev_f32(rs.projmatrix, pos.device)
            present = torch.zeros(pos.shape[0], device=pos.device, dtype=torch.bool)
            _lib.check(_lib.lib().gsr_mark_visible(pos.shape[0], pos.data_ptr(), vm.data_ptr(),
                                                   pm.data_ptr(), present.data_ptr(),
                                                   _lib.stream(pos.device)), "gsr_mark_visible")
        return present

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or "
                            "precomputed 3D covariance!")
        e = torch.Tensor([])
        shs = e if shs is None else shs
        colors_precomp = e if colors_precomp is None else colors_precomp
        scales = e if scales is None else scales
        rotations = e if rotations is None else rotations
        cov3D_precomp = e if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales,
                                   rotations, cov3D_precomp, rs)


# tile instances (num_rendered) of the most recent forward (bench/diagnostics)
last_num_rendered = 0


def rasterize_deferred(raster_settings, means3D, opacities, shs=None, colors_precomp=None,
                       cov3D_precomp=None, scales=None, rotations=None, capacity=1 << 20,
                       key_bits=32):
    """Forward only, with no host read on the stream (include/gsr.h
    gsr_forward_deferred): binning capacity `capacity` instances, depth sort
    over `key_bits` bits.  Returns (color [3,H,W], radii [P], info) where
    info is a device int64[3] {status, num_rendered, live key bits}; the
    image is the frame only when status == 0 (otherwise re-render with
    GaussianRasterizer and size the next call from info).  An extension of
    this module for callers that consume the image later (the SLAM frame
    loop, splatt3r_amd.slam); the reference API above is unchanged."""
    if (shs is None) == (colors_precomp is None):
        raise Exception("Please provide excatly one of either SHs or precomputed colors!")
    if ((scales is None or rotations is None) and cov3D_precomp is None) or \
            ((scales is not None or rotations is not None) and cov3D_precomp is not None):
        raise Exception("Please provide exactly one of either scale/rotation pair or "
                        "precomputed 3D covariance!")
    _lib.require_cuda(means3D)
    dev = means3D.device
    P = means3D.shape[0]
    H, W = int(raster_settings.image_height), int(raster_settings.image_width)
    m3 = _f32c(means3D)
    shc = _f32c(shs)
    M = 0 if shc is None else (shc.shape[1] if shc.dim() == 3 else shc.shape[-1] // 3)
    col, op = _f32c(colors_precomp), _f32c(opacities)
    sc, rot, cov = _f32c(scales), _f32c(rotations), _f32c(cov3D_precomp)
    s, keep = _settings_struct(raster_settings, dev)
    L = _lib.lib()
    color = torch.empty(3, H, W, device=dev, dtype=torch.float32)
    radii = torch.empty(P, device=dev, dtype=torch.int32)
    geom = torch.empty(int(L.gsr_geom_bytes(P)), device=dev, dtype=torch.uint8)
    img = torch.empty(int(L.gsr_image_bytes(H, W)), device=dev, dtype=torch.uint8)
    binning = torch.empty(int(L.gsr_binning_bytes(int(capacity))), device=dev, dtype=torch.uint8)
    info = torch.empty(3, device=dev, dtype=torch.int64)
    _lib.check(L.gsr_forward_deferred(
        ctypes.byref(s), P, M, m3.data_ptr(), _lib.ptr(sc), _lib.ptr(rot), _lib.ptr(cov),
        _lib.ptr(shc), _lib.ptr(col), _lib.ptr(op), radii.data_ptr(), geom.data_ptr(),
        binning.data_ptr(), int(capacity), int(key_bits), img.data_ptr(), color.data_ptr(),
        info.data_ptr(), _lib.stream(dev)), "gsr_forward_deferred")
    return color, radii, info


def set_timing(enabled: bool) -> None:
    """Enable per-phase HIP-event timing of the next forwards (bench.py)."""
    _lib.lib().gsr_set_timing(1 if enabled else 0)


def last_timing():
    """Device ms of the last forward: preprocess, scan, binning+sort, ranges, blend."""
    arr = (ctypes.c_float * 5)()
    _lib.check(_lib.lib().gsr_last_timing(ctypes.cast(arr, P_), 5), "gsr_last_timing")
    return list(arr)
