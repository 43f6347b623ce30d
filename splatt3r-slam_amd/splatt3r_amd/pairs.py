"""Keyframe-pair batches across GPUs: the one unit of the
reference that shards.  FactorGraph.add_factors (global_opt.py:30-99)
decodes each new (i, j) keyframe pair in both orders and matches both
directions (splatt3r_utils.py:466-576); here pair p goes to rank p mod W,
each rank runs its shard as ONE batched symmetric decode (grouped decoder
branches + heads over Bp pairs) + matching, converts its pairs' Gaussians to
world space, and the per-rank world Gaussians are exchanged with a single
RCCL all-gather (the only collective on the path; 52 B per Gaussian).
Match results (idx/valid/Q) stay on the rank that computed them and are
gathered to rank 0 only by the GN backend (§8(f) f1, not built yet).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from splatt3r_amd.splatt3r_utils import splatt3r_match_symmetric, world_records

GAUSS_FLOATS = 13   # means 3 + cov_triu 6 + colour 3 + opacity 1 (52 B)


def shard(pairs, ws: int, rank: int):
    """Pair p -> rank p mod ws (no cross-pair state, splatt3r_utils.py:473-490)."""
    return pairs[rank::ws]


def gather_map(recs: torch.Tensor, ws: int) -> torch.Tensor:
    """The map exchange: every rank contributes its [n_r, 13] world records,
    every rank receives all of them in rank order (one all-gather; shards
    of unequal size are padded to the largest and trimmed after)."""
    if ws == 1:
        return recs
    dev = recs.device
    n = torch.tensor([recs.shape[0]], device=dev, dtype=torch.int64)
    ns = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(ns, n)
    ns = [int(x) for x in ns]
    nmax = max(ns)
    buf = torch.zeros(nmax, recs.shape[1], device=dev, dtype=recs.dtype)
    buf[:recs.shape[0]] = recs
    if dist.get_backend() == "nccl":
        out = torch.empty(ws * nmax, recs.shape[1], device=dev, dtype=recs.dtype)
        dist.all_gather_into_tensor(out, buf)
        parts = out.split(nmax)
    else:
        parts = [torch.empty_like(buf) for _ in range(ws)]
        dist.all_gather(parts, buf)
    return torch.cat([p[:k] for p, k in zip(parts, ns)])


def world_gaussians(res, T_WC: torch.Tensor, img: torch.Tensor) -> torch.Tensor:
    """Per-pixel Gaussians of one predicted view ([H,W,...] dict) -> [h*w, 13]
    world records (means, cov triu, RGB colour, opacity): the transform of
    gaussians_to_world (splatt3r_utils.py:290-318) at stride 1 with its
    filters off, as one HIP pass (include/s3w.h)."""
    from lietorch import Sim3
    M = Sim3(T_WC.reshape(1, 8)).matrix()[0]
    out, _ = world_records(res, img[0] if img.dim() == 4 else img, M)
    return out


@torch.inference_mode()
def process_shard(model, feats, poss, poses, imgs, my_pairs, shape):
    """Batched symmetric decode + matching for this rank's pairs, and the
    world Gaussians of the ii / jj self-predictions.  Returns
    (match tuple, [2*len(my_pairs)*h*w, 13] world records)."""
    ii = torch.tensor([p[0] for p in my_pairs], device=feats.device)
    jj = torch.tensor([p[1] for p in my_pairs], device=feats.device)
    m = splatt3r_match_symmetric(model, feats[ii], poss[ii], feats[jj], poss[jj], shape, shape)
    enc = model.encoder
    pp = enc.pair_plan(len(my_pairs), *shape)
    recs = []
    # pp holds the last decoded order (jj, ii): res[0] = jj self-prediction
    for b, (i, j) in enumerate(my_pairs):
        r = {k: v[b] for k, v in pp.res[0].items()}
        recs.append(world_gaussians(r, poses[j], imgs[j]))
    return m, torch.cat(recs, 0)


def bench_pairs(model, frames, ws, rank, dev, pairs_per_rank=4, n_kf=8, reps=3):
    """keyframe-pairs/s over all ranks: pairs = consecutive keyframes plus
    3 retrieval-like earlier partners per keyframe (main.py:153-173, k=3),
    seed-free and identical on every rank."""
    H, W = frames.shape[-2:]
    torch.cuda.synchronize()
    n_kf = max(2, min(n_kf, frames.shape[0]))
    feats, poss = [], []
    for k in range(n_kf):
        f, p, _ = model.encoder._encode_image(frames[k], None)
        feats.append(f)
        poss.append(p)
    feats, poss = torch.cat(feats), torch.cat(poss)
    poses = torch.zeros(n_kf, 8, device=dev)
    poses[:, 6] = 1.0
    poses[:, 7] = 1.0
    poses[:, 0] = torch.arange(n_kf, device=dev, dtype=torch.float32) * 0.01
    imgs = [frames[k] for k in range(n_kf)]
    allp = []
    for k in range(1, n_kf):
        allp.append((k - 1, k))
        for d in (2, 3, 4):
            if k - d >= 0:
                allp.append((k - d, k))
    total = ws * pairs_per_rank
    allp = (allp * (total // len(allp) + 1))[:total]
    mine = shard(allp, ws, rank)
    shape = (H, W)
    process_shard(model, feats, poss, poses, imgs, mine, shape)   # build + capture plans
    torch.cuda.synchronize()
    n_local = len(mine) * H * W   # the jj self-prediction of every local pair
    times, t_gather = [], []
    for _ in range(reps):
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, recs = process_shard(model, feats, poss, poses, imgs, mine, shape)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        gathered = gather_map(recs, ws)
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        t2 = time.perf_counter()
        times.append(t2 - t0)
        t_gather.append(t2 - t1)
    t = sorted(times)[len(times) // 2]
    if ws > 1:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
    return dict(kf_pairs_per_s=total / t, pairs=total, pairs_per_rank=len(mine),
                ms_per_batch=t * 1e3, allgather_ms=sorted(t_gather)[len(t_gather) // 2] * 1e3,
                allgather_MB_per_rank=n_local * GAUSS_FLOATS * 4 / 1e6,
                map_gaussians=int(gathered.shape[0]))
