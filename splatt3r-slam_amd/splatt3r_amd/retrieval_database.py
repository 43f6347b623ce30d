"""Keyframe retrieval, device half —
splatt3r_slam/retrieval_database.py over include/s3q.h.

`RetrievalDatabase.prep_features` (retrieval_database.py:24-41) and
`quantize_custom` (:95-104) keep their names, inputs and outputs; both run
as HIP kernels (fp64 whiteners, fp32 projector, 'l2norm' attention + top-nfeat
token selection, fused L2-distance + top-k over the codebook).  The weights
come from the MASt3R retrieval checkpoint (`Retriever`, mast3r/retrieval/
processor.py:62-96: prewhiten / projector / postwhiten, nfeat, and the ASMK
codebook centroids); `RetrievalWeights` holds them as device tensors.

The ASMK inverted file (the third-party `asmk` package the reference drives
through `update` / `query` / `add_to_ivf_custom`, :43-134; absent here and
unpinned) is restated from its published algorithm (binary ASMK*, Tolias et
al. ICCV'13) with Retriever's asmk_params (processor.py:84-89) as two HIP
passes (include/s3q.h): `s3q_asmk_aggregate` (per visual word, sign bits of
the summed residuals) and `s3q_asmk_search` (a flat device-resident inverted
file scanned with XOR + popcount, exact int64 scores).  The database lives
on the device and grows geometrically; one host read of the per-image
scores per query (the reference's torch.topk on the CPU).
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Tuple

import torch

from splatt3r_amd import _lib

_lib.register({
    "s3q_whiten": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]),
    "s3q_linear": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4 + [ctypes.c_void_p]),
    "s3q_select_local": (ctypes.c_int, [ctypes.c_void_p] * 2 + [ctypes.c_int] * 4 +
                         [ctypes.c_void_p] * 4),
    "s3q_row_sqnorm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "s3q_l2_topk_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int] * 3),
    "s3q_l2_topk": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 +
                    [ctypes.c_void_p] * 4),
    "s3q_asmk_aggregate_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "s3q_asmk_aggregate": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 +
                           [ctypes.c_void_p] * 5),
    "s3q_asmk_search": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int] +
                        [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_float, ctypes.c_void_p, ctypes.c_int,
                                                 ctypes.c_void_p, ctypes.c_void_p]),
})

# asmk_params of Retriever (processor.py:84-89)
ASMK_PARAMS = {"build_ivf": {"kernel": {"binary": True}, "ivf": {"use_idf": False},
                             "quantize": {"multiple_assignment": 1}, "aggregate": {}},
               "query_ivf": {"quantize": {"multiple_assignment": 5}, "aggregate": {},
                             "search": {"topk": None},
                             "similarity": {"similarity_threshold": 0.0, "alpha": 3.0}}}


@dataclasses.dataclass
class RetrievalWeights:
    proj_W: Optional[torch.Tensor]          # [dim, 1024] f32 (last nn.Linear); None = Identity
    proj_b: Optional[torch.Tensor]          # [dim] f32
    centroids: torch.Tensor                 # [n_clusters, dim] f32 (ASMK codebook)
    prewhiten: Optional[Tuple[torch.Tensor, torch.Tensor]] = None    # (m [1,1024] f64, P f64)
    postwhiten: Optional[Tuple[torch.Tensor, torch.Tensor]] = None   # (m [1,dim] f64, P f64)
    residual: bool = False
    nfeat: int = 300
    # hidden projector layers before the last Linear (build_projector,
    # model.py:144-157: Linear -> LayerNorm -> GELU per entry of hdims[:-1]):
    # [(W [h, d] f32, b [h], ln_w [h], ln_b [h])]
    hidden: tuple = ()
    imsize: int = 512


def _load_retrieval_ckpt(path: str):
    """torch.load(weights_only=True) of the retrieval .pth (processor.py:66-70):
    the training Namespace under 'args' is the one non-tensor global it holds
    and is allowed explicitly; nothing else in the file is executed."""
    import argparse
    with torch.serialization.safe_globals([argparse.Namespace]):
        return torch.load(path, map_location="cpu", weights_only=True)


def _codebook_path(modelname: str) -> str:
    """The ASMK codebook beside the checkpoint (processor.py:80-83 names it
    <prefix>_codebook.pkl).  A pickle is never loaded here: the centroids
    array [n_clusters, dim] is read from <prefix>_codebook.npy (numpy,
    allow_pickle=False) or <prefix>_codebook.safetensors (key 'centroids')."""
    import os
    d, b = os.path.split(modelname)
    stem = os.path.join(d, "_".join(b.split("_")[:-1]) + "_codebook")
    for ext in (".npy", ".safetensors"):
        if os.path.isfile(stem + ext):
            return stem + ext
    if os.path.isfile(stem + ".pkl"):
        raise RuntimeError(
            f"{stem}.pkl is a pickle (the asmk codebook cache); it is not loaded by this build. "
            f"Export its centroids once, where the asmk package is installed, e.g. "
            f"numpy.save('{stem}.npy', asmk_method.codebook.centroids), and place the .npy "
            f"beside the checkpoint")
    raise FileNotFoundError(f"codebook not found: {stem}.npy / .safetensors")


def _load_centroids(path: str) -> torch.Tensor:
    if path.endswith(".npy"):
        import numpy as np
        return torch.from_numpy(np.load(path, allow_pickle=False)).float()
    from safetensors.torch import load_file
    return load_file(path)["centroids"].float()


def load_retrieval_weights(modelname: str, device="cuda") -> RetrievalWeights:
    """Retriever.__init__ (processor.py:66-91): the retrieval head's weights
    from the checkpoint's 'model' state dict (prewhiten.m / .p, projector.*,
    postwhiten.m / .p; backbone.* ignored, the SLAM model's encoder is the
    backbone) and its 'args' (hdims, residual, nfeat, featweights), plus the
    ASMK codebook centroids."""
    import os
    if not os.path.isfile(modelname):
        raise FileNotFoundError(modelname)
    print(f"Loading retrieval model from {modelname}")
    ck = _load_retrieval_ckpt(modelname)
    args, sd = ck["args"], ck["model"]
    fw = getattr(args, "featweights", "l2norm")
    if fw != "l2norm":
        raise NotImplementedError(fw)            # model.py:131-134 raises the same
    hd = getattr(args, "hdims", "1024")
    hdims = [int(x) for x in hd.split("_")] if isinstance(hd, str) and len(hd) > 0 else list(hd or [])
    f32 = lambda k: sd[k].to(device=device, dtype=torch.float32).contiguous()
    f64 = lambda k: sd[k].to(device=device, dtype=torch.float64).contiguous()
    white = lambda n: (f64(f"{n}.m"), f64(f"{n}.p")) if f"{n}.p" in sd else None
    hidden, W, b = [], None, None
    if hdims:
        # nn.Sequential: Linear (3 i), LayerNorm (3 i + 1), GELU per hidden dim
        for i in range(len(hdims) - 1):
            j = 3 * i
            hidden.append((f32(f"projector.{j}.weight"), f32(f"projector.{j}.bias"),
                           f32(f"projector.{j + 1}.weight"), f32(f"projector.{j + 1}.bias")))
        j = 3 * (len(hdims) - 1)
        W, b = f32(f"projector.{j}.weight"), f32(f"projector.{j}.bias")
    cen = _load_centroids(_codebook_path(modelname)).to(device)
    return RetrievalWeights(W, b, cen, white("prewhiten"), white("postwhiten"),
                            residual=bool(getattr(args, "residual", False)),
                            nfeat=getattr(args, "nfeat", 300), hidden=tuple(hidden),
                            imsize=int(getattr(args, "imsize", 512)))


def _chk(t, dtype, name):
    _lib.require_cuda(t)
    if t.dtype != dtype:
        raise RuntimeError(f"{name}: expected {dtype}, got {t.dtype}")
    return t.contiguous()


def whiten(x, m, P):
    """Whitener.forward (model.py:62-75): ((x - m) @ P) in fp64, cast back."""
    x = _chk(x, torch.float32, "whiten")
    P = _chk(P, torch.float64, "whiten")
    K, N = P.shape
    M = x.numel() // K
    out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
    mp = _chk(m, torch.float64, "whiten").data_ptr() if m is not None else None
    _lib.call("s3q_whiten", x.data_ptr(), mp, P.data_ptr(), out.data_ptr(), M, K, N,
              _lib.stream(x.device))
    return out


def linear(x, W, b, residual=False):
    x = _chk(x, torch.float32, "linear")
    W = _chk(W, torch.float32, "linear")
    N, K = W.shape
    M = x.numel() // K
    out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
    bp = _chk(b, torch.float32, "linear").data_ptr() if b is not None else None
    _lib.call("s3q_linear", x.data_ptr(), W.data_ptr(), bp, out.data_ptr(), M, K, N,
              int(bool(residual)), _lib.stream(x.device))
    return out


def how_select_local(feat, attn_src, nfeat):
    """how_select_local (model.py:89-103) with attention = ||attn_src||_2:
    -> (topk_features [B,k,D], topk_attn [B,k], topk_indices [B,k])."""
    feat = _chk(feat, torch.float32, "how_select_local")
    attn_src = _chk(attn_src, torch.float32, "how_select_local")
    B, T, D = feat.shape
    if nfeat < 0:
        nfeat = int(-nfeat * T)
    k = min(int(nfeat), T)
    fo = torch.empty(B, k, D, device=feat.device, dtype=torch.float32)
    ao = torch.empty(B, k, device=feat.device, dtype=torch.float32)
    io = torch.empty(B, k, device=feat.device, dtype=torch.int64)
    _lib.call("s3q_select_local", attn_src.data_ptr(), feat.data_ptr(), B, T, D, k,
              fo.data_ptr(), ao.data_ptr(), io.data_ptr(), _lib.stream(feat.device))
    return fo, ao, io


def row_sqnorm(x):
    x = _chk(x, torch.float32, "row_sqnorm")
    R, D = x.shape
    out = torch.empty(R, device=x.device, dtype=torch.float32)
    _lib.call("s3q_row_sqnorm", x.data_ptr(), R, D, out.data_ptr(), _lib.stream(x.device))
    return out


def l2_topk(q, centroids, c_sqnorm, k):
    """Indices [M,k] i64 and distances [M,k] of the k nearest centroids."""
    q = _chk(q, torch.float32, "l2_topk")
    c = _chk(centroids, torch.float32, "l2_topk")
    M, D = q.shape
    C = c.shape[0]
    if c.shape[1] != D:
        raise RuntimeError("l2_topk: dim mismatch")
    idx = torch.empty(M, k, device=q.device, dtype=torch.int64)
    dist = torch.empty(M, k, device=q.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty(int(L.s3q_l2_topk_workspace_bytes(M, C, k)), device=q.device,
                     dtype=torch.uint8)
    _lib.call("s3q_l2_topk", q.data_ptr(), c.data_ptr(), c_sqnorm.data_ptr(), M, C, D, int(k),
              idx.data_ptr(), dist.data_ptr(), ws.data_ptr(), _lib.stream(q.device))
    return idx, dist


def asmk_aggregate(feats, words, centroids):
    """aggregate_image (binary): feats [n, D] f32, words [n, k] i64 ->
    (unique words [u] i32, codes [u, D/32] u32, device count [1] i32); the
    arrays are sized n*k, the first `count` rows valid."""
    feats = _chk(feats, torch.float32, "asmk_aggregate")
    words = words.to(torch.int64).contiguous()
    n, D = feats.shape
    k = words.shape[1]
    dev = feats.device
    out_w = torch.empty(n * k, dtype=torch.int32, device=dev)
    out_c = torch.empty(n * k, D // 32, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    ws = torch.empty(int(_lib.lib().s3q_asmk_aggregate_workspace_bytes(n, k)), dtype=torch.uint8,
                     device=dev)
    _lib.call("s3q_asmk_aggregate", feats.data_ptr(), words.data_ptr(), centroids.data_ptr(), n, k,
              D, out_w.data_ptr(), out_c.data_ptr(), cnt.data_ptr(), ws.data_ptr(),
              _lib.stream(dev))
    return out_w, out_c, cnt


class InvertedFile:
    """Flat device inverted file: one (word, image, code) entry per
    aggregated word of every database image (asmk ivf.add)."""

    def __init__(self, n_words: int, D: int, device):
        self.n_words, self.D, self.device = n_words, D, device
        self.n = 0
        self.n_images = 0
        self.words = torch.empty(0, dtype=torch.int32, device=device)
        self.images = torch.empty(0, dtype=torch.int32, device=device)
        self.codes = torch.empty(0, D // 32, dtype=torch.int32, device=device)
        self.slot = torch.full((n_words,), -1, dtype=torch.int32, device=device)

    def add(self, words, codes, count: int, image: int):
        need = self.n + count
        if need > self.words.shape[0]:
            cap = max(need, 2 * self.words.shape[0], 4096)
            grow = lambda t, *s: torch.cat([t[:self.n], torch.empty(cap - self.n, *s, dtype=t.dtype,
                                                                     device=self.device)])
            self.words = grow(self.words)
            self.images = grow(self.images)
            self.codes = grow(self.codes, self.D // 32)
        self.words[self.n:need] = words[:count]
        self.images[self.n:need] = image
        self.codes[self.n:need] = codes[:count]
        self.n = need
        self.n_images = max(self.n_images, image + 1)

    def search(self, q_words, q_codes, q_count, alpha=3, threshold=0.0):
        """-> float64 host scores [n_images] (exact: sum of s^alpha / D^alpha)."""
        sc = torch.zeros(max(1, self.n_images), dtype=torch.int64, device=self.device)
        _lib.call("s3q_asmk_search", q_words.data_ptr(), q_codes.data_ptr(), q_count.data_ptr(),
                  q_words.shape[0], self.words.data_ptr(), self.images.data_ptr(),
                  self.codes.data_ptr(), self.n, self.D, int(alpha), float(threshold),
                  self.slot.data_ptr(), self.n_words, sc.data_ptr(), _lib.stream(self.device))
        return sc[:self.n_images].cpu().double() / float(self.D) ** alpha


class RetrievalDatabase:
    """retrieval_database.py:9-134: prep_features / quantize_custom on the
    device kernels above, the ASMK inverted file restated on the device."""

    def __init__(self, modelname, backbone=None, device="cuda"):
        """retrieval_database.py:9-22: `modelname` is the retrieval checkpoint
        path (weights + ASMK codebook beside it, load_retrieval_weights) or
        already-loaded RetrievalWeights; `backbone` is the SLAM model's
        encoder (load_retriever passes model.encoder), whose features the
        caller hands to update() (frame.feat)."""
        weights = (modelname if isinstance(modelname, RetrievalWeights)
                   else load_retrieval_weights(str(modelname), device))
        self.backbone = backbone
        self.w = weights
        self.kf_counter = 0
        self.kf_ids = []
        self.query_dtype = torch.float32
        self.query_device = device
        self.centroids = weights.centroids.to(device=device, dtype=torch.float32).contiguous()
        self._c_sq = row_sqnorm(self.centroids)
        self.ivf = InvertedFile(self.centroids.shape[0], self.centroids.shape[1], device)
        prm = ASMK_PARAMS["query_ivf"]["similarity"]
        self.alpha = int(prm["alpha"])
        self.sim_threshold = float(prm["similarity_threshold"])

    def prep_features(self, backbone_feat):
        """retrieval_database.py:24-41 -> topk_features [B, nfeat, dim]."""
        w = self.w
        x = backbone_feat.float().contiguous()
        if w.prewhiten is not None:
            x = whiten(x, *w.prewhiten)
        h = x
        for Wh, bh, lw, lb in w.hidden:      # build_projector's hidden layers
            h = linear(h, Wh, bh)
            h = torch.nn.functional.gelu(torch.nn.functional.layer_norm(h, h.shape[-1:], lw, lb))
        if w.proj_W is None:                 # hdims empty: nn.Identity
            proj = h + x if w.residual else h
        elif w.residual and w.hidden:
            proj = linear(h, w.proj_W, w.proj_b) + x
        else:
            proj = linear(h, w.proj_W, w.proj_b, w.residual)
        post = whiten(proj, *w.postwhiten) if w.postwhiten is not None else proj
        feats, _, _ = how_select_local(post, proj, w.nfeat)
        return feats

    def quantize_custom(self, qvecs, params):
        """retrieval_database.py:95-104 -> indices [M, multiple_assignment]."""
        k = params["quantize"]["multiple_assignment"]
        idx, _ = l2_topk(qvecs.to(self.query_dtype), self.centroids, self._c_sq, k)
        return idx

    def update(self, frame, add_after_query, k, min_thresh=0.0):
        """retrieval_database.py:43-72: query (if the database is not empty)
        -> keyframe indices of the top-k scores above min_thresh; then add
        the frame when add_after_query."""
        feat = self.prep_features(frame.feat)[0]   # one frame at a time
        topk_inds = []
        topk_codes = None
        if self.kf_counter > 0:
            scores, topk_codes = self.query(feat)
            top = torch.topk(scores.float(), min(k, self.ivf.n_images))
            topk_inds = top.indices[top.values > min_thresh].tolist()
        if add_after_query:
            self.add_to_database(feat, topk_codes)
        return topk_inds

    def query(self, feat):
        """retrieval_database.py:74-87 + accumulate_scores (:106-134):
        quantise (5 words), aggregate, search -> (scores [n_images] f64 host,
        topk_codes [n, 5] device)."""
        codes = self.quantize_custom(feat, ASMK_PARAMS["query_ivf"])
        qw, qc, qn = asmk_aggregate(feat, codes, self.centroids)
        return self.ivf.search(qw, qc, qn, self.alpha, self.sim_threshold), codes

    def add_to_database(self, feat, topk_codes=None):
        """add_to_ivf_custom (:136-166) + bookkeeping (:89-93): reuse the
        query's first assignment when present (build multiple_assignment 1)."""
        k1 = ASMK_PARAMS["build_ivf"]["quantize"]["multiple_assignment"]
        codes = (self.quantize_custom(feat, ASMK_PARAMS["build_ivf"]) if topk_codes is None
                 else topk_codes[:, :k1].contiguous())
        w, c, n = asmk_aggregate(feat, codes, self.centroids)
        self.ivf.add(w, c, int(n.item()), self.kf_counter)
        self.kf_ids.append(self.kf_counter)
        self.kf_counter += 1


def synthetic_retrieval_weights(device, dim=1024, n_clusters=65536, nfeat=300, seed=0):
    """Weights of the retrieval checkpoint's shapes (the checkpoint and its
    ASMK codebook are not available offline): portable generator, unit
    centroids."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    W = (torch.randn(dim, 1024, generator=g) / 32.0).to(device)
    b = torch.zeros(dim, device=device)
    cen = torch.nn.functional.normalize(torch.randn(n_clusters, dim, generator=g), dim=1).to(device)
    P = (torch.randn(1024, 1024, generator=g, dtype=torch.float64) / 32.0).to(device)
    m = torch.zeros(1, 1024, dtype=torch.float64, device=device)
    return RetrievalWeights(W, b, cen, (m, P), (m, P), nfeat=nfeat)


def bench(device, iters=20, C=65536, dim=1024, nfeat=300, k=5):
    """Per-keyframe retrieval device work at the checkpoint's shapes
    (synthetic weights): prep_features on [1,768,1024] and the query
    quantisation of nfeat vectors against C centroids (k = 5)."""
    g = torch.Generator(device="cpu").manual_seed(0)
    W = (torch.randn(dim, 1024, generator=g) / 32.0).to(device)
    b = torch.zeros(dim, device=device)
    cen = torch.nn.functional.normalize(torch.randn(C, dim, generator=g), dim=1).to(device)
    P = (torch.randn(1024, 1024, generator=g, dtype=torch.float64) / 32.0).to(device)
    m = torch.zeros(1, 1024, dtype=torch.float64, device=device)
    db = RetrievalDatabase(RetrievalWeights(W, b, cen, (m, P), (m, P), nfeat=nfeat), device)
    feat = torch.randn(1, 768, 1024, device=device)
    q = db.prep_features(feat)[0]
    prm = {"quantize": {"multiple_assignment": k}}
    for _ in range(3):
        db.prep_features(feat)
        db.quantize_custom(q, prm)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_prep = t_q = 0.0
    for _ in range(iters):
        ev[0].record()
        db.prep_features(feat)
        ev[1].record()
        db.quantize_custom(q, prm)
        ev[2].record()
        torch.cuda.synchronize()
        t_prep += ev[0].elapsed_time(ev[1])
        t_q += ev[1].elapsed_time(ev[2])
    t_prep /= iters
    t_q /= iters
    flops_q = 2.0 * nfeat * C * dim
    return {"prep_features_ms": t_prep, "quantize_ms": t_q,
            "quantize_tflops_fp32": flops_q / (t_q * 1e-3) / 1e12,
            "shape": f"prep [1,768,1024]; quantize {nfeat}x{C}x{dim}, k={k}"}
