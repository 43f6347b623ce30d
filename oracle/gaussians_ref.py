"""ORACLE — test infrastructure only.  torch-CPU restatement of
gaussians_to_world (splatt3r_slam/splatt3r_utils.py:180-328) for checking the
HIP pass (include/s3w.h).  build_covariance / quaternion_to_matrix follow
splatt3r_core/utils/geometry.py:24-62 (same matmul chain), RGB2SH
utils/sh_utils.py:114-115.  The function itself is not importable from the
reference here (its module needs lietorch/cv2); this restatement is pinned
by tests/test_gaussians.py's hand-checked cases."""
from __future__ import annotations

import numpy as np
import torch

C0 = 0.28209479177387814


def quaternion_to_matrix(q, eps: float = 1e-8):
    i, j, k, r = torch.unbind(q, dim=-1)
    two_s = 2 / ((q * q).sum(dim=-1) + eps)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)),
                    -1)
    return o.reshape(*q.shape[:-1], 3, 3)


def build_covariance(scale, rotation_xyzw):
    S = scale.diag_embed()
    R = quaternion_to_matrix(rotation_xyzw)
    return R @ S @ S.transpose(-1, -2) @ R.transpose(-1, -2)


def gaussians_to_world(preds, img, M, spatial_stride=1, depth_min=0.05,
                       depth_max_percentile=0.98, max_scale=0.5, min_confidence=1.5):
    """preds: list of dicts (means/scales/rotations/sh/opacities[/conf], [B,H,W,..]);
    img: [B,3,H,W] normalised; M: [4,4] (sR | t).  Returns the 4-tuple or None."""
    R, t = M[:3, :3], M[:3, 3]
    s = max(1, int(spatial_stride))
    row, col = torch.triu_indices(3, 3)
    outs = []
    for pred in preds:
        means = pred["means"][:, ::s, ::s, :].reshape(-1, 3)
        scales = pred["scales"][:, ::s, ::s, :].reshape(-1, 3)
        rots = pred["rotations"][:, ::s, ::s, :].reshape(-1, 4)
        sh = pred["sh"][:, ::s, ::s].clone()
        opas = pred["opacities"][:, ::s, ::s, :].reshape(-1)
        conf = pred["conf"][:, ::s, ::s].reshape(-1) if "conf" in pred else None
        hwc = (img * 0.5 + 0.5).clamp(0, 1).permute(0, 2, 3, 1)[:, ::s, ::s, :]
        sh[..., 0] = sh[..., 0] + (hwc - 0.5) / C0
        sh = sh.reshape(-1, 3, sh.shape[-1])
        z = means[:, 2]
        valid = z > depth_min
        if bool(valid.any()) and depth_max_percentile < 1.0:
            valid = valid & (z <= torch.quantile(z[valid], depth_max_percentile))
        valid = valid & (scales.max(dim=-1).values < max_scale)
        if conf is not None and min_confidence > 0:
            valid = valid & (conf >= min_confidence)
        means, scales, rots, sh, opas = (x[valid] for x in (means, scales, rots, sh, opas))
        if means.shape[0] == 0:
            continue
        cov_w = R @ build_covariance(scales, rots) @ R.T
        outs.append(((R @ means.T).T + t, cov_w[:, row, col],
                     (sh[:, :, 0] * C0 + 0.5).clamp(0, 1), opas))
    if not outs:
        return None
    return tuple(torch.cat(x, 0) for x in zip(*outs))


class MapRef:
    """numpy restatement of SharedGaussians (splatt3r_slam/frame.py:357-463):
    opacity filter, FIFO half-eviction when full, truncating append."""

    def __init__(self, cap):
        self.cap = cap
        self.n = 0
        self.means = np.zeros((cap, 3), np.float32)
        self.cov = np.zeros((cap, 6), np.float32)
        self.colors = np.zeros((cap, 3), np.float32)
        self.opac = np.zeros(cap, np.float32)
        self.kf = np.zeros(cap, np.int32)

    def append(self, means, cov, colors, opac, kf_idx, thr):
        m = opac > thr
        means, cov, colors, opac = means[m], cov[m], colors[m], opac[m]
        n_new = means.shape[0]
        if n_new == 0:
            return
        n = self.n
        space = self.cap - n
        if space <= 0:
            half = self.cap // 2
            for a in (self.means, self.cov, self.colors, self.opac, self.kf):
                a[:half] = a[self.cap - half:].copy()
            n = half
            space = self.cap - n
        k = min(n_new, space)
        self.means[n:n + k] = means[:k]
        self.cov[n:n + k] = cov[:k]
        self.colors[n:n + k] = colors[:k]
        self.opac[n:n + k] = opac[:k]
        self.kf[n:n + k] = kf_idx
        self.n = n + k
