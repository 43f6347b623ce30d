"""World-space Gaussian map and its full-map render (SURVEY §8 A11 append /
A14, §8(f) f2).

  SharedGaussians          splatt3r_slam/frame.py:357-463
  should_append_gaussians  main.py:54-73
  render_map               splatt3r_slam/visualization.py:467-600
                           (_render_gs_interactive, minus the GL viewport)

The reference keeps the map in shared-memory torch tensors behind a
multiprocessing lock and appends with boolean-mask indexing; here the map is
a device structure-of-arrays with a device-side count (include/s3w.h
s3w_map): `append` takes the [n, 13] world records of
`splatt3r_utils.world_records` (or the 4-tuple of `gaussians_to_world`) and
runs the opacity filter, the FIFO half-eviction and the truncating copy as
three stream-ordered HIP launches with no host sync.  The map is the
all-gather target of the pair-batch shard (pairs.py): any rank can render
any view.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import numpy as np
import torch

from splatt3r_amd import _lib


class S3wMap(ctypes.Structure):
    _fields_ = [("means", ctypes.c_void_p), ("cov_triu", ctypes.c_void_p),
                ("colors", ctypes.c_void_p), ("opacities", ctypes.c_void_p),
                ("kf_id", ctypes.c_void_p), ("n", ctypes.c_void_p), ("cap", ctypes.c_int64)]


_P = ctypes.c_void_p
_lib.register({
    "s3w_map_append_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "s3w_map_append": (ctypes.c_int, [ctypes.POINTER(S3wMap), _P, _P, ctypes.c_int64,
                                      ctypes.c_float, ctypes.c_int32, _P, _P]),
    "s3w_map_scale": (ctypes.c_int, [_P, _P, _P, ctypes.c_int64, ctypes.c_float, ctypes.c_float,
                                     _P, _P, _P]),
})

# the viz clear colour (visualization.py:523-525)
VIZ_BG = (0.118, 0.137, 0.149)


class SharedGaussians:
    """frame.py:357-463 on the device: same fields, same append semantics."""

    def __init__(self, manager=None, max_gaussians: int = 4 * 1024 * 1024, device="cuda"):
        del manager  # single process per GPU: no multiprocessing manager/lock
        self.max_gaussians = int(max_gaussians)
        self.device = torch.device(device)
        cap = self.max_gaussians
        z = lambda *s, dt=torch.float32: torch.zeros(*s, device=self.device, dtype=dt)
        self.means = z(cap, 3)
        self.cov_triu = z(cap, 6)
        self.colors = z(cap, 3)
        self.opacities = z(cap)
        self.kf_id = z(cap, dt=torch.int32)
        self._n = z(1, dt=torch.int64)
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self._c = S3wMap(self.means.data_ptr(), self.cov_triu.data_ptr(), self.colors.data_ptr(),
                         self.opacities.data_ptr(), self.kf_id.data_ptr(), self._n.data_ptr(),
                         cap)

    @property
    def n_gaussians(self) -> int:
        """Host read of the device count (synchronises the stream)."""
        return int(self._n.item())

    def _workspace(self, n):
        need = int(_lib.lib().s3w_map_append_workspace_bytes(n))
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def append_records(self, records: torch.Tensor, count: torch.Tensor, kf_idx: int,
                       opacity_threshold: float = 0.05):
        """records [n_max, 13] (means 3, cov_triu 6, colour 3, opacity),
        count: device int64 [1] of valid rows (s3w_gaussians_to_world)."""
        _lib.require_cuda(records, count)
        n_max = records.shape[0]
        if n_max == 0:
            return
        records = records.float().contiguous()
        ws = self._workspace(n_max)
        _lib.call("s3w_map_append", ctypes.byref(self._c), records.data_ptr(), count.data_ptr(),
                  n_max, float(opacity_threshold), int(kf_idx), ws.data_ptr(),
                  _lib.stream(self.device))

    def append(self, means, cov_triu, colors, opacities, kf_idx: int,
               opacity_threshold: float = 0.05):
        """frame.py:388-443 with the reference's 4-tuple arguments."""
        n = means.shape[0]
        if n == 0:
            return
        rec = torch.cat([means.reshape(n, 3), cov_triu.reshape(n, 6), colors.reshape(n, 3),
                         opacities.reshape(n, 1)], 1).float().contiguous()
        cnt = torch.full((1,), n, dtype=torch.int64, device=rec.device)
        self.append_records(rec, cnt, kf_idx, opacity_threshold)

    def get_all(self):
        """(means, cov_triu, colors, opacities) sliced to [:n], or None."""
        n = self.n_gaussians
        if n == 0:
            return None
        return self.means[:n], self.cov_triu[:n], self.colors[:n], self.opacities[:n]

    def clear(self):
        self._n.zero_()


def should_append_gaussians(add_new_kf: bool, frame_idx: int, current_T_WC,
                            last_append_T_WC, last_append_frame_idx: int,
                            min_translation: float, min_frame_gap: int) -> bool:
    """main.py:54-73."""
    if add_new_kf:
        return True
    if last_append_T_WC is None:
        return True
    if (frame_idx - last_append_frame_idx) < min_frame_gap:
        return False
    t_cur = current_T_WC.matrix()[0, :3, 3]
    t_last = last_append_T_WC.matrix()[0, :3, 3]
    return torch.linalg.norm(t_cur - t_last).item() >= min_translation


def viz_camera(T_WC_cv: np.ndarray, render_w: int, render_h: int, vfov_deg: float,
               near: float = 0.05, far: float = 100.0):
    """The camera of _render_gs_interactive (visualization.py:490-561) for an
    OpenCV camera-to-world pose: returns (tanfovx, tanfovy, viewmatrix,
    projmatrix, campos, scale) with the scale-invariant factor 1/near, using
    the same torch ops as the reference (get_fov, get_projection_matrix).
    Host tensors; `render_map` moves them to the device."""
    from splatt3r_amd.render import get_fov, get_projection_matrix
    vfov_rad = math.radians(vfov_deg)
    fy = render_h / (2.0 * math.tan(vfov_rad / 2.0))
    fx = fy
    cx, cy = render_w / 2.0, render_h / 2.0
    K_norm = torch.tensor([[fx / render_w, 0, cx / render_w], [0, fy / render_h, cy / render_h],
                           [0, 0, 1]], dtype=torch.float32).unsqueeze(0)
    near_t = torch.tensor([near], dtype=torch.float32)
    far_t = torch.tensor([far], dtype=torch.float32)
    fov_xy = get_fov(K_norm)
    fov_x, fov_y = fov_xy[0, 0], fov_xy[0, 1]
    tan_fov_x = (0.5 * fov_x).tan().item()
    tan_fov_y = (0.5 * fov_y).tan().item()
    inv_near = 1.0 / near_t
    ext = torch.from_numpy(np.asarray(T_WC_cv, np.float32)).unsqueeze(0).clone()
    ext[..., :3, 3] *= inv_near[:, None]
    proj = get_projection_matrix(near_t * inv_near, far_t * inv_near, fov_x.unsqueeze(0),
                                 fov_y.unsqueeze(0))
    proj_t = proj[0].T
    view_t = ext[0].inverse().T
    full_proj = view_t @ proj_t
    return (tan_fov_x, tan_fov_y, view_t.contiguous(), full_proj.contiguous(),
            ext[0, :3, 3].contiguous(), inv_near.item(), (inv_near ** 2).item())


def gl_to_cv_T_WC(T_CW_gl: np.ndarray) -> np.ndarray:
    """visualization.py:490-499: OpenGL world-to-camera -> OpenCV
    camera-to-world."""
    cv2gl = np.diag([1.0, -1.0, -1.0, 1.0]).astype(np.float32)
    return np.linalg.inv(cv2gl @ np.asarray(T_CW_gl, np.float32))


@torch.inference_mode()
def render_map(gmap: SharedGaussians, T_WC_cv: np.ndarray, render_w: int, render_h: int,
               vfov_deg: float, bg=VIZ_BG, n: Optional[int] = None, clamp: bool = True,
               camera=None):
    """Full-map render (visualization.py:467-600): every Gaussian of the map
    rasterized with colors_precomp from an OpenCV camera-to-world pose.
    Returns the [3, H, W] image (clamped to [0, 1] like the viz when clamp).
    `camera`: a precomputed viz_camera tuple (the host camera math is torch
    CPU code whose last bit depends on the host's vector ISA)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    dev = gmap.device
    if n is None:
        n = gmap.n_gaussians
    if n == 0:
        return None
    tx, ty, view_t, full_proj, campos, s, s2 = (
        camera if camera is not None else viz_camera(T_WC_cv, render_w, render_h, vfov_deg))
    sc_means = torch.empty(n, 3, device=dev)
    sc_cov = torch.empty(n, 6, device=dev)
    _lib.call("s3w_map_scale", gmap.means.data_ptr(), gmap.cov_triu.data_ptr(),
              gmap._n.data_ptr(), n, float(s), float(s2), sc_means.data_ptr(), sc_cov.data_ptr(),
              _lib.stream(dev))
    st = GaussianRasterizationSettings(
        image_height=render_h, image_width=render_w, tanfovx=tx, tanfovy=ty,
        bg=torch.tensor(bg, dtype=torch.float32, device=dev), scale_modifier=1.0,
        viewmatrix=view_t.to(dev), projmatrix=full_proj.to(dev), sh_degree=0,
        campos=campos.to(dev), prefiltered=False, debug=False)
    image, _ = GaussianRasterizer(st)(means3D=sc_means, means2D=torch.zeros_like(sc_means),
                                      shs=None, colors_precomp=gmap.colors[:n],
                                      opacities=gmap.opacities[:n, None],
                                      cov3D_precomp=sc_cov)
    return image.clamp(0, 1) if clamp else image
