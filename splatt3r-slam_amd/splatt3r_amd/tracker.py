"""FrameTracker mirroring splatt3r_slam/tracker.py:14-300.

The control flow (match → filter → GN → pointmap fusion → keyframe test)
stays on the host as in the reference.  Each Gauss-Newton iteration is one
fused HIP launch (s3t_ray_dist_normal_eqs: act_Sim3 + ray/dist residuals +
Huber weights + J^T J / J^T r / cost reduction; s3t_gn_iterations_calib
for the calibrated pixel + log-depth residuals of opt_pose_calib_sim3,
tracker.py:216-270) followed by a 36-float
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
    "s3t_gn_iterations": (ctypes.c_int, [P_, P_, P_, P_, ctypes.c_int64, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_float, ctypes.c_float, P_, P_, P_, P_, P_]),
    "s3t_calib_normal_eqs": (ctypes.c_int, [P_, P_, P_, P_, P_, ctypes.c_int64, P_, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_float, ctypes.c_float, P_, P_,
                                            P_]),
    "s3t_gn_iterations_calib": (ctypes.c_int, [P_, P_, P_, P_, ctypes.c_int64, P_, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                               ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                               ctypes.c_float, P_, P_, P_, P_, P_]),
    "s3t_track_prep": (ctypes.c_int, [P_, P_, P_, P_, P_, P_, P_, ctypes.c_int64, ctypes.c_float,
                                      ctypes.c_float, P_, P_, P_, P_, P_, P_]),
})


def track_prep(idx, vm, Xf, Cf, Ck, Qff, Qkf, C_conf, Q_conf):
    """tracker.py:28-91's correspondence filter in one HIP pass
    (include/s3t.h s3t_track_prep): returns (Xf[idx] [n,3], Qk =
    sqrt(Qff[idx] * Qkf) [n,1], valid_opt [n,1] bool, counts int64 [3] =
    (valid_opt.sum(), (vm & Qk > Q_conf).sum(), unique(idx[vm]).numel())),
    all on the device, no host sync."""
    n = idx.shape[0]
    dev = idx.device
    t = [x.contiguous() for x in (idx, vm, Xf.float(), Cf.float(), Ck.float(), Qff.float(),
                                  Qkf.float())]
    _lib.require_cuda(*t)
    Xo = torch.empty(n, 3, device=dev)
    Qo = torch.empty(n, 1, device=dev)
    vo = torch.empty(n, 1, device=dev, dtype=torch.bool)
    hit = torch.empty(n + 192, device=dev, dtype=torch.int32)   # flags + count slots (s3t.h)
    cnt = torch.empty(3, device=dev, dtype=torch.int64)
    _lib.call("s3t_track_prep", *(x.data_ptr() for x in t), n, float(C_conf), float(Q_conf),
              Xo.data_ptr(), Qo.data_ptr(), vo.data_ptr(), hit.data_ptr(), cnt.data_ptr(),
              _lib.stream(dev))
    return Xo, Qo, vo, cnt
GN_CHUNK = 8   # iterations queued per host check of the device-side GN state

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
    """Device workspace, pose slot and pinned host buffers for the fused GN
    reduction.  `launch` queues one iteration (pose read from the device
    slot); `fetch` waits for it and returns (H, g, cost) on the host."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = None
        self.out = torch.empty(36, device=self.device)
        self.host = torch.empty(36, pin_memory=True)
        self.pose = torch.empty(8, device=self.device)
        self.pose_host = torch.empty(8, pin_memory=True)
        self.state = torch.empty(4, dtype=torch.float64, device=self.device)
        self.state_init = torch.tensor([float("inf"), 0.0, 0.0, 0.0], dtype=torch.float64).pin_memory()
        self.state_host = torch.empty(4, dtype=torch.float64, pin_memory=True)

    def gn_begin(self, cfg):
        """Reset the device GN state (the pose slot must already hold T)."""
        self.state.copy_(self.state_init, non_blocking=True)

    def _workspace(self, name, n, *ts):
        _lib.require_cuda(*ts)
        _lib.require_contig(name, *ts)
        need = _lib.lib().s3t_workspace_bytes(n)
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)

    def gn_queue(self, Xf, Xk, Q, valid, cfg, iters, calib=None):
        """Queue `iters` device-side GN iterations; the state is copied to
        the pinned host mirror behind them (read after a sync).  `calib`
        = (K host float32[9], (h, w)) selects the calibrated residuals
        (opt_pose_calib_sim3) instead of the ray/dist ones."""
        n = Xf.shape[0]
        if calib is None:
            self._workspace("s3t_gn_iterations", n, Xf, Xk, Q, valid)
            _lib.call("s3t_gn_iterations", Xf.data_ptr(), Xk.data_ptr(), Q.data_ptr(),
                      valid.data_ptr(), n, cfg["sigma_ray"], cfg["sigma_dist"], cfg["huber"],
                      int(iters), int(cfg["max_iters"]), float(cfg["rel_error"]),
                      float(cfg["delta_norm"]), self.pose.data_ptr(), self.state.data_ptr(),
                      self.ws.data_ptr(), self.out.data_ptr(), _lib.stream(self.device))
        else:
            K9, (h, w) = calib
            self._workspace("s3t_gn_iterations_calib", n, Xf, Xk, Q, valid)
            _lib.call("s3t_gn_iterations_calib", Xf.data_ptr(), Xk.data_ptr(), Q.data_ptr(),
                      valid.data_ptr(), n, K9.ctypes.data, int(h), int(w),
                      float(cfg["pixel_border"]), float(cfg["depth_eps"]),
                      float(cfg["sigma_pixel"]), float(cfg["sigma_depth"]), float(cfg["huber"]),
                      int(iters), int(cfg["max_iters"]), float(cfg["rel_error"]),
                      float(cfg["delta_norm"]), self.pose.data_ptr(), self.state.data_ptr(),
                      self.ws.data_ptr(), self.out.data_ptr(), _lib.stream(self.device))
        self.state_host.copy_(self.state, non_blocking=True)

    def set_pose_host(self, T: np.ndarray):
        """Stream-ordered upload of a host pose into the device slot."""
        self.pose_host.numpy()[:] = T
        self.pose.copy_(self.pose_host, non_blocking=True)

    def launch(self, Xf, Xk, Q, valid, sigma_ray, sigma_dist, huber_k):
        n = Xf.shape[0]
        _lib.require_cuda(Xf, Xk, Q, valid)
        _lib.require_contig("s3t_ray_dist_normal_eqs", Xf, Xk, Q, valid)
        need = _lib.lib().s3t_workspace_bytes(n)
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        _lib.call("s3t_ray_dist_normal_eqs", self.pose.data_ptr(), Xf.data_ptr(), Xk.data_ptr(),
                  Q.data_ptr(), valid.data_ptr(), n, sigma_ray, sigma_dist, huber_k,
                  self.ws.data_ptr(), self.out.data_ptr(), _lib.stream(self.device))
        self.host.copy_(self.out, non_blocking=True)

    def launch_calib(self, Xf, Xk, Q, valid, K9, img_size, cfg):
        n = Xf.shape[0]
        self._workspace("s3t_calib_normal_eqs", n, Xf, Xk, Q, valid)
        h, w = img_size
        _lib.call("s3t_calib_normal_eqs", self.pose.data_ptr(), Xf.data_ptr(), Xk.data_ptr(),
                  Q.data_ptr(), valid.data_ptr(), n, K9.ctypes.data, int(h), int(w),
                  float(cfg["pixel_border"]), float(cfg["depth_eps"]), float(cfg["sigma_pixel"]),
                  float(cfg["sigma_depth"]), float(cfg["huber"]), self.ws.data_ptr(),
                  self.out.data_ptr(), _lib.stream(self.device))
        self.host.copy_(self.out, non_blocking=True)

    def fetch(self):
        _lib.wait_stream(self.device)
        return self.unpack(self.host.numpy())

    @staticmethod
    def unpack(v):
        v = v.astype(np.float64)
        H = np.empty((7, 7))
        for q, (a, b) in enumerate(_TRIU):
            H[a, b] = H[b, a] = v[q]
        return H, v[28:35].copy(), float(v[35])

    def __call__(self, T: np.ndarray, Xf, Xk, Q, valid, sigma_ray, sigma_dist, huber_k):
        self.set_pose_host(T)
        self.launch(Xf, Xk, Q, valid, sigma_ray, sigma_dist, huber_k)
        return self.fetch()


# S3_GN_EVENT_WAIT=0: the tracker's decision wait also covers the render
# queued behind the GN chunk (A/B)
_GN_EVENT_WAIT = os.environ.get("S3_GN_EVENT_WAIT", "1") != "0"


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

    def track(self, frame, before_sync=None, ahead=None, keep_info=True):
        """tracker.py:28-127; returns (new_kf, match_info, try_reloc).

        before_sync(T_WC): called with the device-side pose after the first
        queued GN chunk, before the host waits for it, so the caller can
        queue work that depends only on that pose (the frontend's render).
        Its result is kept in self.spec; self.spec_valid says whether that
        pose is the final one (GN stopped inside the first chunk).
        ahead(): the next frame for a shared decode (splatt3r_utils
        _decode_ahead), or None.  keep_info=False: the match info list is not
        built (None; the frontend drops it: no Q copies, no average-conf
        passes per frame)."""
        self.spec, self.spec_valid = None, False
        from splatt3r_amd.splatt3r_utils import splatt3r_match_asymmetric
        mark = getattr(self, "mark", None)       # host-phase recorder (diagnostic)
        keyframe = self.keyframes.last_keyframe()
        if mark:
            mark("track_start")
        idx_f2k, valid_match_k, Xff, Cff, Qff, Xkf, Ckf, Qkf = splatt3r_match_asymmetric(
            self.model, frame, keyframe, idx_i2j_init=self.idx_f2k, ahead=ahead)
        # matching.match returns a fresh tensor that nothing writes later, so
        # the reference's clone (tracker.py:40) is not needed to keep it
        self.idx_f2k = idx_f2k
        idx_f2k = idx_f2k[0]
        if mark:
            mark("matched")
        valid_match_k = valid_match_k[0]
        frame.update_pointmap(Xff, Cff)

        use_calib = config["use_calib"]
        img_size = tuple(frame.img.shape[-2:])
        calib = None
        if use_calib:
            calib = (self._host_K(keyframe.K), img_size)
        Xf_all, Xk, T_WCf, T_WCk, Cf_all, Ck = self._points_poses_full(
            frame, keyframe, img_size, use_calib, keyframe.K)
        # gathers by idx_f2k, Qk = sqrt(Qff[idx] * Qkf), the valid_opt /
        # valid_kf masks and the decision counts (incl. unique(idx[valid]))
        # in one HIP pass, without a host sync
        Xf, Qk, valid_opt, stats = track_prep(idx_f2k, valid_match_k, Xf_all, Cf_all, Ck, Qff,
                                              Qkf, self.cfg["C_conf"], self.cfg["Q_conf"])
        n = valid_opt.numel()
        # pinned mirror reused frame to frame: the host reads it before the
        # next frame's copy is queued
        if getattr(self, "_stats_host", None) is None:
            self._stats_host = torch.empty(3, dtype=torch.int64, pin_memory=True)
        stats_host = self._stats_host
        stats_host.copy_(stats, non_blocking=True)
        # queue the first GN chunk at the device-side relative pose, then one
        # sync covers the decision statistics and (usually) the whole GN
        T_CkCf = T_WCk.inv() * T_WCf
        Xf = Xf.float().contiguous()
        Xk = Xk.float().contiguous()
        Q = Qk.float().contiguous()
        valid_c = valid_opt.contiguous()
        ne = self.normal_eqs
        ne.pose.copy_(T_CkCf.data.reshape(8))
        ne.gn_begin(self.cfg)
        ne.gn_queue(Xf, Xk, Q, valid_c, self.cfg, GN_CHUNK, calib)
        # the host waits for the GN chunk and the statistics copies only: the
        # render queued by before_sync keeps the device busy while the host
        # runs the post-GN glue and issues the next launches
        gn_done = torch.cuda.Event()
        gn_done.record(torch.cuda.current_stream(ne.device))
        gpu_mark = getattr(self, "gpu_mark", None)   # device-time marker (diagnostic)
        if gpu_mark:
            gpu_mark("gn_end")
        if mark:
            mark("gn_queued")
        if before_sync is not None:
            self.spec = before_sync(T_WCk * lietorch.Sim3(ne.pose.clone().view(1, 8)))
        if mark:
            mark("spec_queued")
        if _GN_EVENT_WAIT:
            _lib.wait_event(gn_done)
        else:
            _lib.wait_stream(ne.device)
        n_opt, n_kf, n_unique = stats_host.tolist()
        if mark:
            mark("gn_done")

        if n_opt / n < self.cfg["min_match_frac"]:
            print(f"Skipped frame {frame.frame_id}")
            return False, [], True
        try:
            T_WCf, T_CkCf = self._gn_finish(Xf, Xk, Q, valid_c, T_WCk, calib)
        except CholeskyError:
            print(f"Cholesky failed {frame.frame_id}")
            return False, [], True
        frame.T_WC = T_WCf

        Xkk = T_CkCf.act(Xkf)
        # under the keyframe lock: a backend reader snapshots either the old
        # or the new (X_canon, C, N), with a ready event covering the fusion
        with self.keyframes.lock:
            keyframe.update_pointmap(Xkk, Ckf)
            self.keyframes[len(self.keyframes) - 1] = keyframe

        match_frac_k = n_kf / n
        unique_frac_f = n_unique / n
        self.last_fracs = (n_opt / n, match_frac_k, unique_frac_f)
        new_kf = min(match_frac_k, unique_frac_f) < self.cfg["match_frac_thresh"]
        if new_kf:
            self.reset_idx_f2k()
        if not keep_info:
            return new_kf, None, False
        # Qkf / Qff are views of the pair plan's outputs (splatt3r_match_asymmetric):
        # copies for a caller that keeps the match info past this frame
        return (new_kf, [keyframe.X_canon, keyframe.get_average_conf(), frame.X_canon,
                         frame.get_average_conf(), Qkf.clone(), Qff.clone()], False)

    def _host_K(self, K):
        """K as a host float32[9], cached per tensor (K is constant for a
        sequence; one device read instead of one per frame)."""
        key = (K.data_ptr(), K.device)
        if getattr(self, "_K_key", None) != key:
            self._K_key = key
            self._K9 = np.ascontiguousarray(K.detach().float().cpu().numpy().reshape(9))
        return self._K9

    def _points_poses_full(self, frame, keyframe, img_size=None, use_calib=False, K=None):
        """get_points_poses before the gather by idx_f2k (track_prep gathers)."""
        Xf = frame.X_canon
        Xk = keyframe.X_canon
        if use_calib:
            from splatt3r_amd.geometry import constrain_points_to_ray
            Xf = constrain_points_to_ray(img_size, Xf[None], K).squeeze(0)
            Xk = constrain_points_to_ray(img_size, Xk[None], K).squeeze(0)
        return Xf, Xk, frame.T_WC, keyframe.T_WC, frame.get_average_conf(), keyframe.get_average_conf()

    def get_points_poses(self, frame, keyframe, idx_f2k, img_size=None, use_calib=False, K=None):
        """tracker.py:129-154.  With use_calib both pointmaps are first
        constrained to their pixel rays; the calibrated measurements (pixel
        grid + log keyframe depth, tracker.py:145-151) are formed inside the
        GN kernel from Xk (include/s3t.h s3t_gn_iterations_calib)."""
        Xf = frame.X_canon
        Xk = keyframe.X_canon
        if use_calib:
            from splatt3r_amd.geometry import constrain_points_to_ray
            Xf = constrain_points_to_ray(img_size, Xf[None], K).squeeze(0)
            Xk = constrain_points_to_ray(img_size, Xk[None], K).squeeze(0)
        Cf = frame.get_average_conf()
        Ck = keyframe.get_average_conf()
        return Xf[idx_f2k], Xk, frame.T_WC, keyframe.T_WC, Cf[idx_f2k], Ck

    def _gn_finish(self, Xf, Xk, Q, valid, T_WCk, calib=None):
        """Drive the device-side GN loop (first chunk already queued and
        synced) to its flag; returns (T_WCf, T_CkCf)."""
        cfg, ne = self.cfg, self.normal_eqs
        extra = 0
        while True:
            iters, flag = int(ne.state_host[1]), int(ne.state_host[2])
            if flag != 0 or iters >= cfg["max_iters"]:
                break
            ne.gn_queue(Xf, Xk, Q, valid, cfg, min(GN_CHUNK, cfg["max_iters"] - iters), calib)
            _lib.wait_stream(ne.device)
            extra += 1
        self.spec_valid = extra == 0
        self.last_iters = iters
        if _DEBUG:
            print(f"[gn] iters={iters} flag={flag} cost={float(ne.state_host[3]):.6g}", flush=True)
        if flag == 2:
            raise CholeskyError("normal equations not positive definite")
        if flag == 3:
            print("max iters reached 0")
        T_CkCf = lietorch.Sim3(ne.pose.clone().view(1, 8))
        return T_WCk * T_CkCf, T_CkCf

    def opt_pose_ray_dist_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid):
        """tracker.py:173-214: the whole GN loop runs on the device
        (s3t_gn_iterations), checked by the host once per chunk."""
        ne = self.normal_eqs
        Xf = Xf.float().contiguous()
        Xk = Xk.float().contiguous()
        Q = Qk.float().contiguous()
        valid = valid.contiguous()
        T_CkCf = T_WCk.inv() * T_WCf
        ne.pose.copy_(T_CkCf.data.reshape(8))
        ne.gn_begin(self.cfg)
        ne.gn_queue(Xf, Xk, Q, valid, self.cfg, GN_CHUNK)
        _lib.wait_stream(ne.device)
        return self._gn_finish(Xf, Xk, Q, valid, T_WCk)

    def opt_pose_calib_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid, K, img_size):
        """tracker.py:216-270 on the device (s3t_gn_iterations_calib).  Xf:
        ray-constrained frame points gathered by idx_f2k; Xk: ray-constrained
        keyframe pointmap (its pixel grid and log depth are the measurement,
        built inside the kernel instead of the reference's meas_k /
        valid_meas_k tensors)."""
        ne = self.normal_eqs
        Xf = Xf.float().contiguous()
        Xk = Xk.float().contiguous()
        Q = Qk.float().contiguous()
        valid = valid.contiguous()
        calib = (self._host_K(K), tuple(img_size))
        T_CkCf = T_WCk.inv() * T_WCf
        ne.pose.copy_(T_CkCf.data.reshape(8))
        ne.gn_begin(self.cfg)
        ne.gn_queue(Xf, Xk, Q, valid, self.cfg, GN_CHUNK, calib)
        _lib.wait_stream(ne.device)
        return self._gn_finish(Xf, Xk, Q, valid, T_WCk, calib)

    def opt_pose_ray_dist_sim3_host(self, Xf, Xk, T_WCf, T_WCk, Qk, valid):
        """Host-driven variant (one fused normal-equation launch + host
        Cholesky per iteration), kept for A/B checks of the device loop."""
        cfg = self.cfg
        ne = self.normal_eqs
        T = (T_WCk.inv() * T_WCf).data.reshape(8).detach().cpu().numpy().astype(np.float32)
        Xf = Xf.float().contiguous()
        Xk = Xk.float().contiguous()
        Q = Qk.float().contiguous()
        valid = valid.contiguous()
        old_cost = float("inf")
        for step in range(cfg["max_iters"]):
            H, g, new_cost = ne(T, Xf, Xk, Q, valid, cfg["sigma_ray"], cfg["sigma_dist"],
                                cfg["huber"])
            tau = solve_normal_eqs(H, g)
            T = _retr_host(T, tau)
            self.last_iters = step + 1
            if check_convergence(step, cfg["rel_error"], cfg["delta_norm"], old_cost, new_cost,
                                 tau):
                break
            old_cost = new_cost
            if step == cfg["max_iters"] - 1:
                print("max iters reached 0")
        ne.set_pose_host(T)
        T_CkCf = lietorch.Sim3(ne.pose.clone().view(1, 8))
        return T_WCk * T_CkCf, T_CkCf
