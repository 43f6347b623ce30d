"""Keyframe-pair batches across GPUs: the one unit of the
reference that shards.

FactorGraph.add_factors (global_opt.py:30-99) decodes each new (i, j)
keyframe pair in both orders and matches both directions
(splatt3r_utils.py:466-576) with no state shared between pairs.  Here:

  * keyframe features are broadcast from rank 0 when a keyframe is created
    (`PairShard.broadcast_keyframe`, one RCCL broadcast of the [1, N, 1024]
    fp32 encoder output, 3.1 MB at 512x384), so no rank re-encodes;
  * `PairShard.match_pairs(ii, jj)` sends the pair list to every rank, pair
    p runs on rank p mod W as ONE batched symmetric decode (grouped decoder
    branches + heads over the rank's pairs) + matching, each rank folds the
    reference's Q-weighting into its results (Qj, Qi), and rank 0 gathers
    idx / valid / Q (26 B per pixel per pair) with three all-gathers and
    restores the pair order; the GN solve stays on rank 0 (global_opt.py);
  * the world Gaussians of a rank's pairs reach every rank's map buffer with
    one all-gather (`gather_map`, 52 B per Gaussian).

Ranks other than 0 sit in `PairShard.serve()` and execute the tasks rank 0
broadcasts (keyframe, pair batch, stop).  With gloo (CPU tests) the
collectives stage through host memory; with RCCL they run on the device.
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

from splatt3r_amd.splatt3r_utils import splatt3r_match_symmetric, world_records

GAUSS_FLOATS = 13   # means 3 + cov_triu 6 + colour 3 + opacity 1 (52 B)

OP_STOP, OP_KEYFRAME, OP_PAIRS = 0, 1, 2


def shard(pairs, ws: int, rank: int):
    """Pair p -> rank p mod ws (no cross-pair state, splatt3r_utils.py:473-490)."""
    return pairs[rank::ws]


def _backend():
    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def _staged(t: torch.Tensor, fn):
    """Run a collective on `t` (in place); gloo moves device tensors through
    the host."""
    if _backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        fn(h)
        t.copy_(h)
    else:
        fn(t)
    return t


def _all_gather_equal(t: torch.Tensor, ws: int) -> list[torch.Tensor]:
    """All-gather of equal-shape tensors (rank order)."""
    if _backend() == "nccl":
        out = torch.empty((ws * t.shape[0],) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
        dist.all_gather_into_tensor(out, t.contiguous())
        return list(out.split(t.shape[0]))
    src = t.cpu() if t.is_cuda else t
    parts = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(parts, src.contiguous())
    return [p.to(t.device) for p in parts]


def gather_map(recs: torch.Tensor, ws: int) -> torch.Tensor:
    """The map exchange: every rank contributes its [n_r, 13] world records,
    every rank receives all of them in rank order (one all-gather; shards
    of unequal size are padded to the largest and trimmed after)."""
    if ws == 1:
        return recs
    dev = recs.device
    n = torch.tensor([recs.shape[0]], device=dev, dtype=torch.int64)
    ns = [int(x) for x in _all_gather_equal(n, ws)]
    nmax = max(ns)
    buf = torch.zeros(nmax, recs.shape[1], device=dev, dtype=recs.dtype)
    buf[:recs.shape[0]] = recs
    parts = _all_gather_equal(buf, ws)
    return torch.cat([p[:k] for p, k in zip(parts, ns)])


def q_weighted(m, Q_conf):
    """The per-direction confidences add_factors forms (global_opt.py:56-66):
    Qj = sqrt(Qii[idx_i2j] * Qji), Qi = sqrt(Qjj[idx_j2i] * Qij)."""
    idx_i2j, idx_j2i, valid_j, valid_i, Qii, Qjj, Qji, Qij = m
    b = torch.arange(idx_i2j.shape[0], device=idx_i2j.device)[:, None].repeat(
        1, idx_i2j.shape[1])
    Qj = torch.sqrt(Qii[b, idx_i2j] * Qji)
    Qi = torch.sqrt(Qjj[b, idx_j2i] * Qij)
    return idx_i2j, idx_j2i, valid_j, valid_i, Qj, Qi


class PairShard:
    """Rank-side state of the pair shard: the keyframe features every rank
    holds, and the execution of this rank's share of a pair batch.

    match_fn(feat_i, pos_i, feat_j, pos_j, shape_i, shape_j) -> the 8-tuple
    of splatt3r_match_symmetric; injectable so the collective protocol is
    testable without the network (tests/test_pairs.py)."""

    def __init__(self, model, device, match_fn: Optional[Callable] = None, Q_conf=None):
        from splatt3r_amd.config import config
        self.model = model
        self.device = torch.device(device)
        self.ws = dist.get_world_size() if _backend() else 1
        self.rank = dist.get_rank() if _backend() else 0
        self.match_fn = match_fn or (lambda *a: splatt3r_match_symmetric(model, *a))
        self.Q_conf = config["local_opt"]["Q_conf"] if Q_conf is None else Q_conf
        self.kf: dict[int, tuple] = {}   # keyframe index -> (feat, pos, true_shape)
        self.stats = dict(pairs=0, keyframes=0)

    # ------------------------------------------------------------ tasks ---
    def _header(self, op=0, a=0, b=0):
        h = torch.tensor([op, a, b], dtype=torch.int64, device=self.device)
        if self.ws > 1:
            _staged(h, lambda t: dist.broadcast(t, 0))
        return [int(x) for x in h.tolist()]

    def _bcast(self, t):
        if self.ws > 1:
            _staged(t, lambda x: dist.broadcast(x, 0))
        return t

    def broadcast_keyframe(self, idx: int, frame=None):
        """Rank 0: frame = the new keyframe (its encoder output is cached on
        every rank).  Other ranks call it from serve()."""
        if self.rank == 0:
            N, C = frame.feat.shape[-2:]
            H, W = (int(v) for v in frame.img_true_shape.reshape(-1)[:2].tolist())
            self._header(OP_KEYFRAME, idx, (N << 32) | C)
            dims = torch.tensor([H, W], dtype=torch.int64, device=self.device)
            self._bcast(dims)
            feat = frame.feat.reshape(1, N, C).float().contiguous()
            self._bcast(feat)
            pos = frame.pos.reshape(1, N, 2).contiguous()
        else:
            raise RuntimeError("broadcast_keyframe is called on rank 0; workers use serve()")
        self.kf[idx] = (feat, pos, torch.tensor([[H, W]], dtype=torch.int32))
        self.stats["keyframes"] += 1

    def _recv_keyframe(self, idx, nc):
        N, C = nc >> 32, nc & 0xFFFFFFFF
        dims = self._bcast(torch.zeros(2, dtype=torch.int64, device=self.device))
        H, W = (int(v) for v in dims.tolist())
        feat = self._bcast(torch.empty(1, N, C, device=self.device))
        # token positions are a function of the image size (PositionGetter,
        # croco/models/blocks.py:193-205): rebuilt, not sent
        from splatt3r_amd.net import positions
        pos = positions(1, H // 16, W // 16, self.device)
        self.kf[idx] = (feat, pos, torch.tensor([[H, W]], dtype=torch.int32))
        self.stats["keyframes"] += 1

    def register_local(self, idx: int, frame):
        """Single-rank use: cache a keyframe without a broadcast."""
        self.kf[idx] = (frame.feat, frame.pos, frame.img_true_shape)

    # ----------------------------------------------------------- pairs ----
    def _run_local(self, pairs):
        if not pairs:
            return None
        fi = torch.cat([self.kf[i][0] for i, _ in pairs])
        pi = torch.cat([self.kf[i][1] for i, _ in pairs])
        fj = torch.cat([self.kf[j][0] for _, j in pairs])
        pj = torch.cat([self.kf[j][1] for _, j in pairs])
        si = [self.kf[i][2] for i, _ in pairs]
        sj = [self.kf[j][2] for _, j in pairs]
        self.stats["pairs"] += len(pairs)
        return q_weighted(self.match_fn(fi, pi, fj, pj, si, sj), self.Q_conf)

    def match_pairs(self, ii, jj):
        """Rank 0: idx_i2j, idx_j2i [n, hw] i64, valid_j, valid_i [n, hw, 1]
        bool, Qj, Qi [n, hw, 1] f32 for the pairs (ii[p], jj[p]) in order."""
        pairs = list(zip((int(i) for i in ii), (int(j) for j in jj)))
        n = len(pairs)
        if self.ws == 1:
            return self._run_local(pairs)
        self._header(OP_PAIRS, n)
        pl = torch.tensor(pairs, dtype=torch.int64, device=self.device).reshape(n, 2)
        self._bcast(pl)
        return self._pairs_collective(pairs)

    def _pairs_collective(self, pairs):
        ws, rank = self.ws, self.rank
        n = len(pairs)
        mine = shard(pairs, ws, rank)
        res = self._run_local(mine)
        per = -(-n // ws)
        (feat, _, shp) = self.kf[pairs[0][0]]
        hw = int(shp.reshape(-1)[0]) * int(shp.reshape(-1)[1])
        dev = self.device
        idx = torch.zeros(per, 2, hw, dtype=torch.int64, device=dev)
        val = torch.zeros(per, 2, hw, dtype=torch.uint8, device=dev)
        q = torch.zeros(per, 2, hw, dtype=torch.float32, device=dev)
        if res is not None:
            k = len(mine)
            idx[:k, 0], idx[:k, 1] = res[0], res[1]
            val[:k, 0], val[:k, 1] = res[2][..., 0], res[3][..., 0]
            q[:k, 0], q[:k, 1] = res[4][..., 0], res[5][..., 0]
        idx_all = _all_gather_equal(idx, ws)
        val_all = _all_gather_equal(val, ws)
        q_all = _all_gather_equal(q, ws)
        if rank != 0:
            return None
        # pair p sits on rank p % ws at local slot p // ws
        order = [(p % ws, p // ws) for p in range(n)]
        I = torch.stack([idx_all[r][s] for r, s in order])
        V = torch.stack([val_all[r][s] for r, s in order]).bool()
        Qt = torch.stack([q_all[r][s] for r, s in order])
        return I[:, 0], I[:, 1], V[:, 0, :, None], V[:, 1, :, None], Qt[:, 0, :, None], \
            Qt[:, 1, :, None]

    # ---------------------------------------------------------- workers ---
    def serve(self):
        """Ranks > 0: execute rank 0's tasks until OP_STOP."""
        assert self.rank != 0
        while True:
            op, a, b = self._header()
            if op == OP_STOP:
                return
            if op == OP_KEYFRAME:
                self._recv_keyframe(a, b)
            elif op == OP_PAIRS:
                pl = self._bcast(torch.empty(a, 2, dtype=torch.int64, device=self.device))
                self._pairs_collective([tuple(int(v) for v in p) for p in pl.tolist()])

    def stop(self):
        if self.rank == 0 and self.ws > 1:
            self._header(OP_STOP)


def world_gaussians(res, T_WC: torch.Tensor, img: torch.Tensor) -> torch.Tensor:
    """Per-pixel Gaussians of one predicted view ([H,W,...] dict) -> [h*w, 13]
    world records (means, cov triu, RGB colour, opacity): the transform of
    gaussians_to_world (splatt3r_utils.py:290-318) at stride 1 with its
    filters off, as one HIP pass (include/s3w.h).  Labelled unfiltered in
    the bench: the map records of the pair shard, not the reference's
    per-frame gaussians_to_world output."""
    from lietorch import Sim3
    M = Sim3(T_WC.reshape(1, 8)).matrix()[0]
    out, _ = world_records(res, img[0] if img.dim() == 4 else img, M)
    return out


@torch.inference_mode()
def bench_pairs(model, frames, ws, rank, dev, pairs_per_rank=4, n_kf=8, reps=3):
    """keyframe-pairs/s of the sharded FactorGraph.add_factors path: rank 0
    creates n_kf keyframes (encoder + broadcast to every rank), then issues
    add_factors over consecutive keyframes plus 3 retrieval-like earlier
    partners per keyframe (main.py:153-173, k = 3), ws * pairs_per_rank pairs
    per batch; ranks > 0 serve.  After each batch the jj self-predictions
    of every rank's pairs become world records and are all-gathered into
    every rank's map buffer (unfiltered, stride 1)."""
    from splatt3r_amd.frame import Keyframes, create_frame
    from splatt3r_amd.gaussian_map import SharedGaussians
    from splatt3r_amd.global_opt import FactorGraph
    H, W = frames.shape[-2:]
    torch.cuda.synchronize()
    n_kf = max(2, min(n_kf, frames.shape[0]))
    sh = PairShard(model, dev)
    kfs = Keyframes()
    allp = []
    for k in range(1, n_kf):
        allp.append((k - 1, k))
        for d in (2, 3, 4):
            if k - d >= 0:
                allp.append((k - d, k))
    total = ws * pairs_per_rank
    allp = (allp * (total // len(allp) + 1))[:total]
    t_bc = 0.0
    if rank == 0:
        for k in range(n_kf):
            f = create_frame(k, frames[k], device=dev)
            f.feat, f.pos, _ = model.encoder._encode_image(f.img, f.img_true_shape)
            kfs.append(f)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if ws > 1:
                sh.broadcast_keyframe(k, f)
            else:
                sh.register_local(k, f)
            torch.cuda.synchronize()
            t_bc += time.perf_counter() - t0
        if ws > 1:
            sh.stop()
        fg = FactorGraph(model, kfs, device=dev, shard=sh)
        ii = [p[0] for p in allp]
        jj = [p[1] for p in allp]
    else:
        sh.serve()              # receive the keyframes
    gmap = SharedGaussians(max_gaussians=max(1, 2 * total * H * W), device=dev)
    pp = model.encoder.pair_plan(len(shard(allp, ws, rank)), H, W, tag="backend")

    def one_batch():
        if rank == 0:
            fg.add_factors(ii, jj, 0.0)
            if ws > 1:
                sh.stop()
        else:
            sh.serve()
        # the jj self-predictions of this rank's pairs -> world records ->
        # every rank's map (the last decoded order is (jj, ii): res[0] = jj)
        mine = shard(allp, ws, rank)
        recs = [world_gaussians({k: v[b] for k, v in pp.res[0].items()},
                                torch.tensor([0, 0, 0, 0, 0, 0, 1, 1.0], device=dev),
                                frames[j]) for b, (_, j) in enumerate(mine)]
        gathered = gather_map(torch.cat(recs, 0), ws)
        gmap.clear()
        gmap.append_records(gathered, torch.tensor([gathered.shape[0]], device=dev), 0, -1.0)
        return gathered

    one_batch()                 # build + capture plans
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gathered = one_batch()
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    if ws > 1:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
    out = dict(kf_pairs_per_s=total / t, pairs=total, pairs_per_rank=len(shard(allp, ws, rank)),
               ms_per_batch=t * 1e3, map_gaussians=int(gathered.shape[0]),
               map_records="unfiltered stride-1 jj self-predictions (52 B each)",
               path="FactorGraph.add_factors -> PairShard (pair p on rank p mod W) -> "
                    "gather to rank 0; map all-gather")
    if ws > 1:
        out["keyframe_broadcast_ms"] = t_bc / n_kf * 1e3
        out["allgather_MB_per_rank"] = len(shard(allp, ws, rank)) * H * W * GAUSS_FLOATS * 4 / 1e6
    return out
