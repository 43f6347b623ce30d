"""FrameTracker mirroring splatt3r_slam/tracker.py:14-300.

The control flow (match → filter → GN → pointmap fusion → keyframe test)
stays on the host as in the reference.  Each Gauss-Newton iteration is one
fused HIP launch (s3t_ray_dist_normal_eqs: act_Sim3 + ray/dist residuals +
Huber weights + J^T J / J^T r / cost reduction) followed by a 36-float
download, a 7x7 Cholesky on the host and the Sim3 retraction on the host —
the reference does ~30 torch launches, a cuBLAS A^T A, a GPU Cholesky and an
`.item()` sync per iteration (tracker.py:156-214).
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

import lietorch
from splatt3r_amd import _lib
from splatt3r_amd.config import config

P_ = ctypes.c_void_p
_lib.register({
    "s3t_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "s3t_ray_dist_normal_eqs": (ctypes.c_int, [P_, P_, P_, P_, P_, ctypes.c_int64, ctypes.c_float,
                                               ctypes.c_float, ctypes.c_float, P_, P_, P_]),
})

_TRIU = [(a, b) for a in range(7) for b in range(a, 7)]
_DEBUG = os.environ.get("S3_TRACK_DEBUG", "0") == "1"


class CholeskyError(RuntimeError):
    pass


def check_convergence(it, rel_error_threshold, delta_norm_threshold, old_cost, new_cost, delta):
    """nonlinear_optimizer.py:5-25."""
    rel_dec = math.fabs((old_cost - new_cost) / old_cost)
    delta_norm = float(np.linalg.norm(delta))
    return rel_dec < rel_error_threshold or delta_norm < delta_norm_threshold


class NormalEquations:
    """Device workspace + pinned host buffer for the fused GN reduction."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = None
        self.out = torch.empty(36, device=self.device)
        self.host = torch.empty(36, pin_memory=True)
        self.pose = (ctypes.c_float * 8)()

    def __call__(self, T: np.ndarray, Xf, Xk, Q, valid, sigma_ray, sigma_dist, huber_k):
        n = Xf.shape[0]
        _lib.require_cuda(Xf, Xk, Q, valid)
        _lib.require_contig("s3t_ray_dist_normal_eqs", Xf, Xk, Q, valid)
        need = _lib.lib().s3t_workspace_bytes(n)
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        for k in range(8):
            self.pose[k] = float(T[k])
        st = _lib.stream(self.device)
        _lib.call("s3t_ray_dist_normal_eqs", ctypes.addressof(self.pose), Xf.data_ptr(),
                  Xk.data_ptr(), Q.data_ptr(), valid.data_ptr(), n, sigma_ray, sigma_dist,
                  huber_k, self.ws.data_ptr(), self.out.data_ptr(), st)
        self.host.copy_(self.out, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        v = self.host.numpy().astype(np.float64)
        H = np.empty((7, 7))
        for q, (a, b) in enumerate(_TRIU):
            H[a, b] = H[b, a] = v[q]
        return H, v[28:35].copy(), float(v[35])


def solve_normal_eqs(H, g):
    """Cholesky solve of H tau = g (tracker.py:168-171); raises
    CholeskyError where torch.linalg.cholesky would raise."""
    if not (np.all(np.isfinite(H)) and np.all(np.isfinite(g))):
        raise CholeskyError("non-finite normal equations")
    try:
        L = np.linalg.cholesky(H)
    except np.linalg.LinAlgError as e:
        raise CholeskyError(str(e)) from e
    y = np.linalg.solve(L, g)
    return np.linalg.solve(L.T, y)


def _retr_host(T: np.ndarray, tau: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(T, dtype=np.float32).reshape(1, 8)
    x = np.ascontiguousarray(tau, dtype=np.float32).reshape(1, 7)
    out = np.empty((1, 8), np.float32)
    _lib.lib().s3lie_sim3_retr_host(a.ctypes.data, x.ctypes.data, out.ctypes.data)
    return out[0]


class FrameTracker:
    def __init__(self, model, frames, device):
        self.cfg = config["tracking"]
        self.model = model
        self.keyframes = frames
        self.device = device
        self.normal_eqs = NormalEquations(device)
        self.last_iters = 0
        self.reset_idx_f2k()

    def reset_idx_f2k(self):
        self.idx_f2k = None

    def track(self, frame):
        """tracker.py:28-127; returns (new_kf, match_info, try_reloc)."""
        from splatt3r_amd.splatt3r_utils import splatt3r_match_asymmetric
        keyframe = self.keyframes.last_keyframe()
        idx_f2k, valid_match_k, Xff, Cff, Qff, Xkf, Ckf, Qkf = splatt3r_match_asymmetric(
            self.model, frame, keyframe, idx_i2j_init=self.idx_f2k)
        self.idx_f2k = idx_f2k.clone()
        idx_f2k = idx_f2k[0]
        valid_match_k = valid_match_k[0]
        Qk = torch.sqrt(Qff[idx_f2k] * Qkf)
        frame.update_pointmap(Xff, Cff)

        if config["use_calib"]:
            raise NotImplementedError("calibrated tracking (opt_pose_calib_sim3) is §8(f) work")
        Xf, Xk, T_WCf, T_WCk, Cf, Ck = self.get_points_poses(frame, keyframe, idx_f2k)

        valid_Cf = Cf > self.cfg["C_conf"]
        valid_Ck = Ck > self.cfg["C_conf"]
        valid_Q = Qk > self.cfg["Q_conf"]
        valid_opt = valid_match_k & valid_Cf & valid_Ck & valid_Q
        valid_kf = valid_match_k & valid_Q

        match_frac = float(valid_opt.sum()) / valid_opt.numel()
        if match_frac < self.cfg["min_match_frac"]:
            print(f"Skipped frame {frame.frame_id}")
            return False, [], True
        try:
            T_WCf, T_CkCf = self.opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid_opt)
        except CholeskyError:
            print(f"Cholesky failed {frame.frame_id}")
            return False, [], True
        frame.T_WC = T_WCf

        Xkk = T_CkCf.act(Xkf)
        keyframe.update_pointmap(Xkk, Ckf)
        self.keyframes[len(self.keyframes) - 1] = keyframe

        match_frac_k = float(valid_kf.sum()) / valid_kf.numel()
        unique_frac_f = torch.unique(idx_f2k[valid_match_k[:, 0]]).shape[0] / valid_kf.numel()
        new_kf = min(match_frac_k, unique_frac_f) < self.cfg["match_frac_thresh"]
        if new_kf:
            self.reset_idx_f2k()
        return (new_kf, [keyframe.X_canon, keyframe.get_average_conf(), frame.X_canon,
                         frame.get_average_conf(), Qkf, Qff], False)

    def get_points_poses(self, frame, keyframe, idx_f2k):
        """tracker.py:129-154 (uncalibrated branch)."""
        Cf = frame.get_average_conf()
        Ck = keyframe.get_average_conf()
        return (frame.X_canon[idx_f2k], keyframe.X_canon, frame.T_WC, keyframe.T_WC,
                Cf[idx_f2k], Ck)

    def opt_pose_ray_dist_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid):
        """tracker.py:173-214 with the per-iteration work fused on the GPU."""
        cfg = self.cfg
        T_CkCf = T_WCk.inv() * T_WCf
        T = T_CkCf.data.reshape(8).detach().cpu().numpy().astype(np.float32)
        Xf = Xf.float().contiguous()
        Xk = Xk.float().contiguous()
        Q = Qk.float().contiguous()
        valid = valid.contiguous()
        old_cost = float("inf")
        for step in range(cfg["max_iters"]):
            H, g, new_cost = self.normal_eqs(T, Xf, Xk, Q, valid, cfg["sigma_ray"],
                                             cfg["sigma_dist"], cfg["huber"])
            if _DEBUG:
                print(f"[gn] step {step} n={Xf.shape[0]} valid={int(valid.sum())} cost={new_cost:.4g} "
                      f"Hdiag={np.diag(H)} g={g} T={T} "
                      f"finite Xf={bool(torch.isfinite(Xf).all())} Xk={bool(torch.isfinite(Xk).all())} "
                      f"Q={bool(torch.isfinite(Q).all())} |Xf|min={float(Xf.norm(dim=-1).min()):.3g} "
                      f"|Xk|min={float(Xk.norm(dim=-1).min()):.3g}", flush=True)
            tau = solve_normal_eqs(H, g)
            T = _retr_host(T, tau)
            self.last_iters = step + 1
            if check_convergence(step, cfg["rel_error"], cfg["delta_norm"], old_cost, new_cost,
                                 tau):
                break
            old_cost = new_cost
            if step == cfg["max_iters"] - 1:
                print("max iters reached 0")
        T_CkCf = lietorch.Sim3(torch.from_numpy(T.copy()).to(Xf.device).view(1, 8))
        return T_WCk * T_CkCf, T_CkCf
