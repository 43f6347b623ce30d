"""ORACLE (test infrastructure only) — torch-CPU restatement of the keyframe
retrieval features and codebook quantisation:

  Whitener.forward        mast3r/retrieval/model.py:55-75 (fp64 centring + PCA)
  RetrievalModel.projector model.py:143-156 (Linear 1024->1024, optional residual)
  attention 'l2norm'      model.py:133-134 (x.norm(dim=-1))
  how_select_local        model.py:89-103 (topk over tokens + gather)
  prep_features           splatt3r_slam/retrieval_database.py:24-41
  quantize_custom         retrieval_database.py:95-104 (|q|^2 + |c|^2 - 2 q c^T, topk smallest)

The reference's retrieval checkpoint and ASMK codebook are not available
offline, so parity is pinned on synthetic weights/centroids of the
checkpoint's shapes; the text above is the restated algorithm.
"""
from __future__ import annotations

import torch


def whiten(x, m, P):
    """Whitener.forward with l2norm=None: ((x.double() - m) @ P).to(x.dtype)."""
    shape = x.shape
    xr = x.reshape(-1, shape[-1]).double()
    if m is not None:
        xr = xr - m.reshape(1, -1)
    return (xr @ P).reshape(*shape[:-1], P.shape[1]).to(x.dtype)


def prep_features(feat, prewhiten, W, b, residual, postwhiten, nfeat):
    """prewhiten -> projector (+ residual) -> attention = L2 norm ->
    postwhiten -> top-nfeat tokens by attention.  prewhiten/postwhiten are
    (m, P) or None (nn.Identity)."""
    x = whiten(feat, *prewhiten) if prewhiten is not None else feat
    proj = torch.nn.functional.linear(x, W, b) + (x if residual else 0.0)
    attn = proj.norm(dim=-1)
    post = whiten(proj, *postwhiten) if postwhiten is not None else proj
    k = min(int(nfeat), attn.shape[1])
    topk_attn, topk_idx = torch.topk(attn, k, dim=1)
    feats = torch.gather(post, 1, topk_idx.unsqueeze(-1).expand(-1, -1, post.shape[2]))
    return feats, topk_attn, topk_idx


def quantize(qvecs, centroids, k):
    """quantize_custom: indices of the k smallest l2 distances per row, and
    the distances."""
    l2 = (torch.sum(qvecs ** 2, dim=1)[:, None] + torch.sum(centroids ** 2, dim=1)[None, :]
          - 2 * (qvecs @ centroids.mT))
    t = torch.topk(l2, k, dim=1, largest=False)
    return t.indices, t.values, l2


# ------------------------------------------------------------------ ASMK ---
# Restatement of the third-party `asmk` package's binary ASMK* as
# RetrievalDatabase drives it (retrieval_database.py:43-134) with
# Retriever's asmk_params (mast3r/retrieval/processor.py:84-89): build with
# multiple_assignment 1, query with 5, similarity threshold 0, alpha 3, no
# idf.  The package is absent (not vendored, unpinned): parity is pinned to
# this text.  Residual sums are taken in float64 (asmk: float32); scores are
# exact (s = D - 2 hamming, s^3 / D^3).
import numpy as np


def asmk_aggregate(feats, words, centroids):
    """aggregate_image: unique words ascending; per word the sign bits of
    sum over assigned descriptors of (x - c_w), packed LSB-first in uint32."""
    feats = np.asarray(feats, np.float32)
    words = np.asarray(words).reshape(feats.shape[0], -1)
    D = feats.shape[1]
    uw = np.unique(words)
    codes = np.zeros((uw.shape[0], D // 32), np.uint32)
    for u, w in enumerate(uw):
        sel = (words == w).any(axis=1)
        r = (feats[sel] - centroids[w][None].astype(np.float32)).astype(np.float64).sum(0)
        bits = (r > 0).reshape(D // 32, 32).astype(np.uint64)
        codes[u] = (bits << np.arange(32, dtype=np.uint64)).sum(1).astype(np.uint32)
    return uw.astype(np.int32), codes


def _popcount32(x):
    x = x.astype(np.uint64)
    c = np.zeros(x.shape, np.int64)
    for b in range(32):
        c += ((x >> np.uint64(b)) & np.uint64(1)).astype(np.int64)
    return c


def asmk_search(q_words, q_codes, db_words, db_images, db_codes, D, n_images, alpha=3,
                threshold=0.0):
    """ivf.search with the ASMK kernel: per query word, the database entries
    of that word; sim = 1 - 2 hamming / D, kept when >= threshold, raised to
    alpha and summed per image.  Returns float64 scores [n_images]."""
    scores = np.zeros(n_images, np.float64)
    slot = {int(w): i for i, w in enumerate(q_words)}
    for e in range(len(db_words)):
        q = slot.get(int(db_words[e]))
        if q is None:
            continue
        ham = int(_popcount32(np.bitwise_xor(db_codes[e], q_codes[q])).sum())
        s = D - 2 * ham
        if s / D >= threshold:
            scores[int(db_images[e])] += float(s) ** alpha / float(D) ** alpha
    return scores


class RetrievalDBRef:
    """RetrievalDatabase.update (retrieval_database.py:43-72) over the
    restated IVF; quantisation by `quantize` above."""

    def __init__(self, centroids):
        self.centroids = np.asarray(centroids, np.float32)
        self.kf_counter = 0
        self.db = []      # (word, image, code)

    def update(self, feat, add_after_query, k, min_thresh=0.0):
        import torch
        f = np.asarray(feat, np.float32)
        topk_codes = None
        inds = []
        if self.kf_counter > 0:
            idx5, _, _ = quantize(torch.from_numpy(f), torch.from_numpy(self.centroids), 5)
            topk_codes = idx5.numpy()
            qw, qc = asmk_aggregate(f, topk_codes, self.centroids)
            D = f.shape[1]
            dbw = np.array([d[0] for d in self.db], np.int32)
            dbi = np.array([d[1] for d in self.db], np.int32)
            dbc = np.stack([d[2] for d in self.db]) if self.db else np.zeros((0, D // 32), np.uint32)
            scores = asmk_search(qw, qc, dbw, dbi, dbc, D, self.kf_counter)
            kk = min(k, self.kf_counter)
            t = torch.topk(torch.from_numpy(scores.astype(np.float32)), kk)
            inds = t.indices[t.values > min_thresh].tolist()
        if add_after_query:
            if topk_codes is None:
                idx1, _, _ = quantize(torch.from_numpy(f), torch.from_numpy(self.centroids), 1)
                codes1 = idx1.numpy()
            else:
                codes1 = topk_codes[:, :1]
            w, c = asmk_aggregate(f, codes1, self.centroids)
            self.db += [(int(a), self.kf_counter, b) for a, b in zip(w, c)]
            self.kf_counter += 1
        return inds
