"""FactorGraph of the SLAM backend (splatt3r_slam/global_opt.py:12-158),
ray mode: keyframe pairs -> batched symmetric decode + matching (one fused
pair plan per batch, splatt3r_utils.splatt3r_match_symmetric) -> two-way
edges -> the device-resident Gauss-Newton of include/s3g.h
(mast3r_slam_backends.gauss_newton_rays).

Same attribute names, edge bookkeeping and acceptance rule as the
reference; solve_GN_calib (config use_calib) runs the calibrated device
solve (mast3r_slam_backends.gauss_newton_calib) on points constrained to
their pixel rays.

Multi-GPU: with a `shard` (pairs.PairShard over W > 1
ranks) add_factors sends the pair list to every rank, pair p is decoded and
matched on rank p mod W, and rank 0 receives idx / valid / Q for all pairs
in order; edges and the GN solve are then exactly the single-rank ones.
"""
from __future__ import annotations

import torch

import lietorch
import mast3r_slam_backends
from splatt3r_amd.config import config
from splatt3r_amd.pairs import q_weighted
from splatt3r_amd.splatt3r_utils import splatt3r_match_symmetric


class FactorGraph:
    def __init__(self, model, frames, K=None, device="cuda", shard=None, match_fn=None):
        self.model = model
        self.shard = shard
        # splatt3r_match_symmetric(model, ...) unless injected (protocol tests)
        self.match_fn = match_fn or (lambda *a: splatt3r_match_symmetric(model, *a))
        self.frames = frames
        self.device = device
        self.cfg = config["local_opt"]
        L = lambda dt: torch.as_tensor([], dtype=dt, device=device)
        self.ii, self.jj = L(torch.long), L(torch.long)
        self.idx_ii2jj, self.idx_jj2ii = L(torch.long), L(torch.long)
        self.valid_match_j, self.valid_match_i = L(torch.bool), L(torch.bool)
        self.Q_ii2jj, self.Q_jj2ii = L(torch.float32), L(torch.float32)
        self.window_size = self.cfg["window_size"]
        self.K = K

    def add_factors(self, ii, jj, min_match_frac, is_reloc=False):
        """global_opt.py:30-99."""
        if self.shard is not None and self.shard.ws > 1:
            idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qj, Qi = \
                self.shard.match_pairs(ii, jj)
        else:
            kf_ii = [self.frames[i] for i in ii]
            kf_jj = [self.frames[j] for j in jj]
            feat_i = torch.cat([k.feat for k in kf_ii])
            feat_j = torch.cat([k.feat for k in kf_jj])
            pos_i = torch.cat([k.pos for k in kf_ii])
            pos_j = torch.cat([k.pos for k in kf_jj])
            shape_i = [k.img_true_shape for k in kf_ii]
            shape_j = [k.img_true_shape for k in kf_jj]
            m = self.match_fn(feat_i, pos_i, feat_j, pos_j, shape_i, shape_j)
            idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qj, Qi = q_weighted(
                m, self.cfg["Q_conf"])
        valid_j = valid_match_j & (Qj > self.cfg["Q_conf"])
        valid_i = valid_match_i & (Qi > self.cfg["Q_conf"])
        match_frac_j = valid_j.sum(dim=(1, 2)) / (valid_j.shape[1] * valid_j.shape[2])
        match_frac_i = valid_i.sum(dim=(1, 2)) / (valid_i.shape[1] * valid_i.shape[2])
        ii_t = torch.as_tensor(ii, device=self.device)
        jj_t = torch.as_tensor(jj, device=self.device)
        # both directions must clear the threshold; consecutive edges always stay
        invalid = (torch.minimum(match_frac_j, match_frac_i) < min_match_frac) & \
            ~(ii_t == jj_t - 1)
        if is_reloc and bool(invalid.any()):
            return False
        keep = ~invalid
        self.ii = torch.cat([self.ii, ii_t[keep]])
        self.jj = torch.cat([self.jj, jj_t[keep]])
        self.idx_ii2jj = torch.cat([self.idx_ii2jj, idx_i2j[keep]])
        self.idx_jj2ii = torch.cat([self.idx_jj2ii, idx_j2i[keep]])
        self.valid_match_j = torch.cat([self.valid_match_j, valid_match_j[keep]])
        self.valid_match_i = torch.cat([self.valid_match_i, valid_match_i[keep]])
        self.Q_ii2jj = torch.cat([self.Q_ii2jj, Qj[keep]])
        self.Q_jj2ii = torch.cat([self.Q_jj2ii, Qi[keep]])
        return bool(keep.sum() > 0)

    def get_unique_kf_idx(self):
        return torch.unique(torch.cat([self.ii, self.jj]), sorted=True)

    def prep_two_way_edges(self):
        """global_opt.py:105-111."""
        ii = torch.cat((self.ii, self.jj), dim=0)
        jj = torch.cat((self.jj, self.ii), dim=0)
        idx = torch.cat((self.idx_ii2jj, self.idx_jj2ii), dim=0)
        valid = torch.cat((self.valid_match_j, self.valid_match_i), dim=0)
        Q = torch.cat((self.Q_ii2jj, self.Q_jj2ii), dim=0)
        return ii, jj, idx, valid, Q

    def get_poses_points(self, unique_kf_idx):
        kfs = [self.frames[int(i)] for i in unique_kf_idx]
        Xs = torch.stack([k.X_canon for k in kfs])
        T_WCs = lietorch.Sim3(torch.stack([k.T_WC.data.reshape(1, 8) for k in kfs]))
        Cs = torch.stack([k.get_average_conf() for k in kfs])
        return Xs, T_WCs, Cs

    def _publish(self, unique, pose_data, pin):
        """global_opt.py:155-158 / :211-215: write the optimised poses back
        (through Keyframes.set_poses: deferred to the frontend's stream when
        this runs on the backend worker thread)."""
        idx = unique[pin:].tolist()
        rows = pose_data[pin:]
        if hasattr(self.frames, "set_poses"):
            self.frames.set_poses(idx, rows)
            return
        for r, i in enumerate(idx):
            self.frames[i].T_WC = lietorch.Sim3(rows[r:r + 1].clone())

    def solve_GN_rays(self):
        """global_opt.py:121-158."""
        pin = self.cfg["pin"]
        unique = self.get_unique_kf_idx()
        if unique.numel() <= pin:
            return None
        Xs, T_WCs, Cs = self.get_poses_points(unique)
        ii, jj, idx, valid, Q = self.prep_two_way_edges()
        pose_data = T_WCs.data[:, 0, :].contiguous()
        (dx,) = mast3r_slam_backends.gauss_newton_rays(
            pose_data, Xs.contiguous().float(), Cs.contiguous().float(), ii.contiguous(),
            jj.contiguous(), idx.contiguous(), valid.contiguous(), Q.contiguous().float(),
            self.cfg["sigma_ray"], self.cfg["sigma_dist"], self.cfg["C_conf"],
            self.cfg["Q_conf"], self.cfg["max_iters"], self.cfg["delta_norm"])
        self._publish(unique, pose_data, pin)
        return dx

    def solve_GN_calib(self):
        """global_opt.py:160-215."""
        from splatt3r_amd.geometry import constrain_points_to_ray
        K = self.K
        pin = self.cfg["pin"]
        unique = self.get_unique_kf_idx()
        if unique.numel() <= pin:
            return None
        Xs, T_WCs, Cs = self.get_poses_points(unique)
        img_size = self.frames[0].img.shape[-2:]
        Xs = constrain_points_to_ray(img_size, Xs, K)
        ii, jj, idx, valid, Q = self.prep_two_way_edges()
        height, width = img_size
        pose_data = T_WCs.data[:, 0, :].contiguous()
        (dx,) = mast3r_slam_backends.gauss_newton_calib(
            pose_data, Xs.contiguous().float(), Cs.contiguous().float(), K.float(),
            ii.contiguous(), jj.contiguous(), idx.contiguous(), valid.contiguous(),
            Q.contiguous().float(), height, width, self.cfg["pixel_border"],
            self.cfg["depth_eps"], self.cfg["sigma_pixel"], self.cfg["sigma_depth"],
            self.cfg["C_conf"], self.cfg["Q_conf"], self.cfg["max_iters"],
            self.cfg["delta_norm"])
        self._publish(unique, pose_data, pin)
        return dx
