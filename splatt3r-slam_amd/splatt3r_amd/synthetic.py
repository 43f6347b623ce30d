"""Synthetic workloads (there is no network for datasets or checkpoints).

raster_microbench_scene: BASELINE config 3 exactly as SURVEY.md §8(d) C3
  defines it — P Gaussians in front of a camera at the origin looking +z,
  960x540, K = [[776,0,480],[0,776,270],[0,0,1]], near 0.1 / far 1000 with
  the scale-invariant x10 of cuda_splatting.py:67-76; z ~ U(2,8), x,y
  uniform in the frustum at that z; scales exp(U(ln .005, ln .03)) per axis;
  rotations normalised N(0,1)^4 (xyzw); cov6 = triu(R S^2 R^T); opacity
  U(.05,.99); SH DC N(0,1)*.5; bg 0; dL/dimage N(0,1).  numpy PCG64 seeds 0
  (scene) and 1 (grad).
"""
from __future__ import annotations

import numpy as np
import torch

C3_K = np.array([[776.0, 0.0, 480.0], [0.0, 776.0, 270.0], [0.0, 0.0, 1.0]], np.float32)
C3_HW = (540, 960)
C3_P = 4_194_304


def quat_xyzw_to_rot(q: np.ndarray) -> np.ndarray:
    i, j, k, r = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    two_s = 2.0 / (np.sum(q * q, -1) + 1e-8)
    R = np.stack([1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                  two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                  two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)],
                 -1)
    return R.reshape(-1, 3, 3)


def raster_microbench_scene(P: int, H: int = C3_HW[0], W: int = C3_HW[1], K=C3_K,
                            seed: int = 0, chunk: int = 1 << 20):
    """Returns a dict of float32 numpy arrays in *unscaled* world units:
    means [P,3], cov6 [P,6], opacities [P,1], shs [P,1,3], K, H, W."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    means = np.empty((P, 3), np.float32)
    cov6 = np.empty((P, 6), np.float32)
    for s in range(0, P, chunk):
        n = min(chunk, P - s)
        z = rng.uniform(2.0, 8.0, n)
        u = rng.uniform(0.0, W, n)
        v = rng.uniform(0.0, H, n)
        means[s:s + n, 0] = (u - cx) / fx * z
        means[s:s + n, 1] = (v - cy) / fy * z
        means[s:s + n, 2] = z
        sc = np.exp(rng.uniform(np.log(0.005), np.log(0.03), (n, 3)))
        q = rng.normal(size=(n, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        R = quat_xyzw_to_rot(q)
        cov = np.einsum("nik,nk,njk->nij", R, sc * sc, R)
        iu = np.triu_indices(3)
        cov6[s:s + n] = cov[:, iu[0], iu[1]]
    opac = rng.uniform(0.05, 0.99, (P, 1)).astype(np.float32)
    shs = (rng.normal(size=(P, 1, 3)) * 0.5).astype(np.float32)
    return dict(means=means, cov6=cov6, opacities=opac, shs=shs, K=K, H=H, W=W)


def raster_grad(H: int, W: int, seed: int = 1) -> np.ndarray:
    return np.random.Generator(np.random.PCG64(seed)).normal(size=(3, H, W)).astype(np.float32)


def identity_camera_settings(K, H, W, device, near=0.1, far=1000.0, bg=(0.0, 0.0, 0.0)):
    """Settings of render_cuda for a camera at the origin (world == camera),
    scale-invariant.  Returns (settings, scale)."""
    from splatt3r_amd.render import camera_settings, normalize_intrinsics
    Kt = torch.as_tensor(K, dtype=torch.float32, device=device)[None]
    intr = normalize_intrinsics(Kt, (H, W))
    ext = torch.eye(4, device=device)[None]
    nr = torch.full((1,), near, device=device)
    fr = torch.full((1,), far, device=device)
    bgt = torch.tensor([bg], dtype=torch.float32, device=device)
    st, scale = camera_settings(ext, intr, nr, fr, (H, W), bgt, 0)
    return st[0], float(scale[0])


def settings_to_dict(rs) -> dict:
    """GaussianRasterizationSettings -> plain dict of host values (for the oracle)."""
    t = lambda x: x.detach().float().cpu().numpy().ravel() if torch.is_tensor(x) else np.asarray(x)
    return dict(image_height=rs.image_height, image_width=rs.image_width, tanfovx=rs.tanfovx,
                tanfovy=rs.tanfovy, bg=t(rs.bg), scale_modifier=rs.scale_modifier,
                viewmatrix=t(rs.viewmatrix), projmatrix=t(rs.projmatrix),
                sh_degree=rs.sh_degree, campos=t(rs.campos))


def smooth_texture(TH: int, TW: int, seed: int) -> np.ndarray:
    """[3, TH, TW] float32 in [0, 1]: three octaves of bicubically upsampled
    uniform noise (cells 64 / 16 / 4 px), numpy PCG64 `seed`."""
    rng = np.random.default_rng(seed)
    tex = np.zeros((3, TH, TW), np.float32)
    for cell, amp in ((64, 0.5), (16, 0.3), (4, 0.2)):
        g = rng.random((3, TH // cell + 2, TW // cell + 2)).astype(np.float32)
        t = torch.from_numpy(g)[None]
        up = torch.nn.functional.interpolate(t, scale_factor=cell, mode="bicubic",
                                             align_corners=False)[0, :, :TH, :TW]
        tex += amp * up.numpy()
    return np.clip(tex, 0.0, 1.0)


def tum_like_sequence(n: int, H: int = 384, W: int = 512, seed: int = 0, step_px: float = 3.0,
                      device="cuda") -> torch.Tensor:
    """C2 stand-in when the TUM fr1_desk frames are absent: n frames of a
    slowly panning camera over a smooth multi-scale noise texture (numpy
    PCG64 `seed`), already resized/cropped to the 512x384 the reference's
    resize_img produces from 640x480, normalised like ImgNorm.
    Returns [n, 1, 3, H, W] float32 on `device`."""
    pad = int(np.ceil(step_px * n)) + 8
    tex = smooth_texture(H + pad, W + pad, seed)
    texd = torch.from_numpy(tex).to(device)
    out = torch.empty(n, 1, 3, H, W, device=device)
    for i in range(n):
        oy = int(round(0.5 * step_px * i)) + 4
        ox = int(round(step_px * i)) + 4
        out[i, 0] = (texd[:, oy:oy + H, ox:ox + W] - 0.5) / 0.5
    return out


def c5_map_batches(n: int, seed: int = 0, device="cuda", chunk: int = 1 << 20):
    """C5 stand-in map content (bench.py bench_map, tests): n synthetic
    world Gaussians in a 4 m x 2.5 m x 4 m room in front of an identity
    camera, in keyframe-sized batches of `chunk` of the reference's
    SharedGaussians.append arguments (means [m,3], cov_triu [m,6],
    colours [m,3], opacities [m] >= 0.35, so the 0.3 filter keeps all)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    iu = torch.triu_indices(3, 3, device=dev)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        u = lambda *sh: torch.rand(*sh, generator=g, device=dev)
        means = (u(m, 3) - 0.5) * torch.tensor([4.0, 2.5, 4.0], device=dev) + \
            torch.tensor([0.0, 0.0, 4.0], device=dev)
        sc = torch.exp(torch.log(torch.tensor(0.004, device=dev)) + u(m, 3) * 2.0)
        q = torch.nn.functional.normalize(torch.randn(m, 4, generator=g, device=dev), dim=1)
        x, y, z, w = q.unbind(1)
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                         2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                         2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
                        1).reshape(m, 3, 3)
        cov = torch.einsum("nik,nk,njk->nij", R, sc * sc, R)
        yield means, cov[:, iu[0], iu[1]].contiguous(), u(m, 3), 0.35 + 0.65 * u(m)
