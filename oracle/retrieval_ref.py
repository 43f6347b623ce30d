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
