"""Drop-in `lietorch` subset (Sim3 / SE3) backed by the HIP kernels of
libsplatt3r_hip.so (include/s3lie.h).

Covers the surface Splatt3R-SLAM uses:
  Sim3.Identity (main.py:398, frame.py:24,160), Sim3 * Sim3 and .inv()
  (tracker.py:180,212,225,264), .act (geometry.py:46, tracker.py:98),
  .retr (tracker.py:195,247), .data / .embedded_dim (frame.py:266),
  SE3(...).matrix() (splatt3r_utils.py:161-164, main.py:70-71), plus
  exp / log for completeness.

Layout: Sim3 data [..., 8] = t(3) q(xyzw,4) s(1); SE3 data [..., 7].
Batch dimensions broadcast like lietorch's apply_op.  Device tensors run the
HIP kernels on torch's current stream; CPU tensors are accepted only for the
group-level ops (mul / inv / retr / matrix / exp), which run the library's
native host implementation (no point action on CPU).
"""
from __future__ import annotations

import ctypes

import torch

from splatt3r_amd import _lib

__all__ = ["Sim3", "SE3", "LieGroup"]


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.float32).contiguous()


def _host_map(fn_name: str, out_dim: int, *arrays: torch.Tensor) -> torch.Tensor:
    """Apply a per-element host entry point (CPU tensors, small batches)."""
    n = arrays[0].shape[0]
    out = torch.empty(n, out_dim, dtype=torch.float32)
    fn = getattr(_lib.lib(), fn_name)
    for i in range(n):
        fn(*[a[i].data_ptr() for a in arrays], out[i].data_ptr())
    return out


class LieGroup:
    embedded_dim = 0
    manifold_dim = 0

    def __init__(self, data: torch.Tensor):
        if data.shape[-1] != self.embedded_dim:
            raise ValueError(
                f"{type(self).__name__} expects data[..., {self.embedded_dim}], "
                f"got {tuple(data.shape)}")
        self.data = data

    # --- tensor-like plumbing -------------------------------------------
    @property
    def shape(self):
        return self.data.shape[:-1]

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    def __len__(self):
        return self.shape[0]

    def __getitem__(self, idx):
        return type(self)(self.data[idx])

    def __setitem__(self, idx, other):
        self.data[idx] = other.data

    def to(self, *args, **kw):
        return type(self)(self.data.to(*args, **kw))

    def cpu(self):
        return type(self)(self.data.cpu())

    def cuda(self):
        return type(self)(self.data.cuda())

    def float(self):
        return type(self)(self.data.float())

    def detach(self):
        return type(self)(self.data.detach())

    def clone(self):
        return type(self)(self.data.clone())

    def view(self, *dims):
        return type(self)(self.data.view(*dims, self.embedded_dim))

    def __repr__(self):
        return f"{type(self).__name__}({self.data})"


class Sim3(LieGroup):
    embedded_dim = 8
    manifold_dim = 7

    @classmethod
    def Identity(cls, *batch, device=None, dtype=torch.float32, requires_grad=False):
        data = torch.zeros(*batch, 8, device=device, dtype=dtype)
        data[..., 6] = 1.0
        data[..., 7] = 1.0
        return cls(data)

    # --- binary / unary ops ---------------------------------------------
    def __mul__(self, other):
        if isinstance(other, Sim3):
            return Sim3(_mul(self.data, other.data))
        if isinstance(other, torch.Tensor):
            return self.act(other)
        return NotImplemented

    def inv(self):
        bshape = self.shape
        a = _f32(self.data).reshape(-1, 8)
        if a.is_cuda:
            out = torch.empty_like(a)
            _lib.call("s3lie_sim3_inv", a.data_ptr(), out.data_ptr(), a.shape[0],
                      _lib.stream(a.device))
        else:
            out = _host_map("s3lie_sim3_inv_host", 8, a)
        return Sim3(out.view(*bshape, 8))

    def act(self, p: torch.Tensor) -> torch.Tensor:
        if p.shape[-1] != 3:
            raise ValueError("Sim3.act expects points [..., 3]")
        _lib.require_cuda(self.data, p)
        bshape = torch.broadcast_shapes(self.shape, p.shape[:-1])
        n = 1
        for d in bshape:
            n *= d
        T = _f32(self.data)
        if T[..., 0].numel() == 1:
            T = T.reshape(1, 8)
            n_T = 1
        else:
            T = T.expand(*bshape, 8).contiguous().reshape(-1, 8)
            n_T = n
        X = _f32(p).expand(*bshape, 3).contiguous().reshape(-1, 3)
        Y = torch.empty_like(X)
        _lib.call("s3lie_sim3_act", T.data_ptr(), n_T, X.data_ptr(), Y.data_ptr(), n,
                  _lib.stream(X.device))
        return Y.view(*bshape, 3)

    @classmethod
    def exp(cls, xi: torch.Tensor):
        bshape = xi.shape[:-1]
        x = _f32(xi).reshape(-1, 7)
        out = torch.empty(x.shape[0], 8, device=x.device, dtype=torch.float32)
        if x.is_cuda:
            _lib.call("s3lie_sim3_exp", x.data_ptr(), out.data_ptr(), x.shape[0],
                      _lib.stream(x.device))
        else:  # Exp(xi) = Exp(xi) * Identity
            ident = cls.Identity(x.shape[0]).data
            out = _host_map("s3lie_sim3_retr_host", 8, ident, x)
        return cls(out.view(*bshape, 8))

    def log(self) -> torch.Tensor:
        _lib.require_cuda(self.data)
        bshape = self.shape
        a = _f32(self.data).reshape(-1, 8)
        out = torch.empty(a.shape[0], 7, device=a.device, dtype=torch.float32)
        _lib.call("s3lie_sim3_log", a.data_ptr(), out.data_ptr(), a.shape[0],
                  _lib.stream(a.device))
        return out.view(*bshape, 7)

    def retr(self, a: torch.Tensor):
        """Left retraction Exp(a) * X (lietorch semantics)."""
        bshape = torch.broadcast_shapes(self.shape, a.shape[:-1])
        n = 1
        for d in bshape:
            n *= d
        T = _f32(self.data)
        xi = _f32(a)
        if T.is_cuda:
            nT = 1 if T[..., 0].numel() == 1 else n
            nX = 1 if xi[..., 0].numel() == 1 else n
            T = T.reshape(1, 8) if nT == 1 else T.expand(*bshape, 8).contiguous().reshape(-1, 8)
            xi = xi.reshape(1, 7) if nX == 1 else xi.expand(*bshape, 7).contiguous().reshape(-1, 7)
            out = torch.empty(n, 8, device=T.device, dtype=torch.float32)
            _lib.call("s3lie_sim3_retr", T.data_ptr(), nT, xi.data_ptr(), nX, out.data_ptr(), n,
                      _lib.stream(T.device))
        else:
            T = T.expand(*bshape, 8).contiguous().reshape(-1, 8)
            xi = xi.expand(*bshape, 7).contiguous().reshape(-1, 7)
            out = _host_map("s3lie_sim3_retr_host", 8, T, xi)
        return Sim3(out.view(*bshape, 8))

    def matrix(self) -> torch.Tensor:
        return _matrix(self.data, "s3lie_sim3_matrix", 8)


class SE3(LieGroup):
    embedded_dim = 7
    manifold_dim = 6

    @classmethod
    def Identity(cls, *batch, device=None, dtype=torch.float32, requires_grad=False):
        data = torch.zeros(*batch, 7, device=device, dtype=dtype)
        data[..., 6] = 1.0
        return cls(data)

    def matrix(self) -> torch.Tensor:
        return _matrix(self.data, "s3lie_se3_matrix", 7)


def _mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    bshape = torch.broadcast_shapes(a.shape[:-1], b.shape[:-1])
    n = 1
    for d in bshape:
        n *= d
    A, B = _f32(a), _f32(b)
    if A.is_cuda:
        na = 1 if A[..., 0].numel() == 1 else n
        nb = 1 if B[..., 0].numel() == 1 else n
        A = A.reshape(1, 8) if na == 1 else A.expand(*bshape, 8).contiguous().reshape(-1, 8)
        B = B.reshape(1, 8) if nb == 1 else B.expand(*bshape, 8).contiguous().reshape(-1, 8)
        out = torch.empty(n, 8, device=A.device, dtype=torch.float32)
        _lib.call("s3lie_sim3_mul", A.data_ptr(), na, B.data_ptr(), nb, out.data_ptr(), n,
                  _lib.stream(A.device))
    else:
        A = A.expand(*bshape, 8).contiguous().reshape(-1, 8)
        B = B.expand(*bshape, 8).contiguous().reshape(-1, 8)
        out = _host_map("s3lie_sim3_mul_host", 8, A, B)
    return out.view(*bshape, 8)


def _matrix(data: torch.Tensor, fn: str, dim: int) -> torch.Tensor:
    bshape = data.shape[:-1]
    a = _f32(data).reshape(-1, dim)
    if not a.is_cuda:
        # 4x4 assembly of a handful of poses on the host (no kernel needed)
        return _matrix_host(a, dim).view(*bshape, 4, 4)
    out = torch.empty(a.shape[0], 4, 4, device=a.device, dtype=torch.float32)
    _lib.call(fn, a.data_ptr(), out.data_ptr(), a.shape[0], _lib.stream(a.device))
    return out.view(*bshape, 4, 4)


def _matrix_host(a: torch.Tensor, dim: int) -> torch.Tensor:
    # Same formula as sim3_math.hpp quat_to_rot; CPU harness use only.
    t, q = a[:, :3], a[:, 3:7]
    x, y, z, w = q.unbind(-1)
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    R = torch.stack([
        1 - (ty * y + tz * z), ty * x - tz * w, tz * x + ty * w,
        ty * x + tz * w, 1 - (tx * x + tz * z), tz * y - tx * w,
        tz * x - ty * w, tz * y + tx * w, 1 - (tx * x + ty * y)], -1).view(-1, 3, 3)
    if dim == 8:
        R = R * a[:, 7, None, None]
    M = torch.zeros(a.shape[0], 4, 4)
    M[:, :3, :3] = R
    M[:, :3, 3] = t
    M[:, 3, 3] = 1
    return M
