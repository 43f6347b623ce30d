"""Keyframe retrieval features + codebook quantisation:
HIP (include/s3q.h) vs the torch-CPU oracle/retrieval_ref.py.  The reference
retrieval checkpoint and ASMK codebook are not available offline: weights
and centroids are synthetic tensors of the checkpoint's shapes (projector
1024->1024, codebook 65536 x 1024, nfeat 300)."""
import numpy as np
import pytest
import torch

from oracle import retrieval_ref as R


def _weights(dim=1024, din=1024, C=65536, seed=0, whiten=True):
    g = torch.Generator().manual_seed(seed)
    W = torch.randn(dim, din, generator=g) / din ** 0.5
    b = torch.randn(dim, generator=g) * 0.01
    cen = torch.nn.functional.normalize(torch.randn(C, dim, generator=g), dim=1)
    pre = post = None
    if whiten:
        pre = (torch.randn(1, din, generator=g, dtype=torch.float64) * 0.1,
               torch.randn(din, din, generator=g, dtype=torch.float64) / din ** 0.5)
        post = (torch.randn(1, dim, generator=g, dtype=torch.float64) * 0.1,
                torch.randn(dim, dim, generator=g, dtype=torch.float64) / dim ** 0.5)
    return W, b, cen, pre, post


def test_oracle_quantize_is_exhaustive_nearest():
    g = torch.Generator().manual_seed(1)
    q, c = torch.randn(7, 16, generator=g), torch.randn(50, 16, generator=g)
    idx, d, _ = R.quantize(q, c, 3)
    bf = torch.cdist(q.double(), c.double()) ** 2
    assert torch.equal(idx[:, 0], bf.argmin(1))
    assert torch.allclose(d.double(), bf.gather(1, idx), atol=1e-4)


def test_api_refuses_cpu_tensors():
    from splatt3r_amd import retrieval_database as RD
    with pytest.raises(RuntimeError, match="GPU only"):
        RD.row_sqnorm(torch.zeros(4, 4))


def _dev(t):
    return None if t is None else t.cuda()


@pytest.mark.gpu
def test_hip_whiten_and_linear_vs_oracle():
    from splatt3r_amd import retrieval_database as RD
    W, b, _, pre, _ = _weights(C=256)
    x = torch.randn(1, 768, 1024)
    ref = R.whiten(x, *pre)
    got = RD.whiten(x.cuda(), *map(_dev, pre)).cpu()
    assert torch.allclose(got, ref, rtol=1e-6, atol=1e-6)
    ref = torch.nn.functional.linear(x, W, b) + x
    got = RD.linear(x.cuda(), W.cuda(), b.cuda(), residual=True).cpu()
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-4)
    # ragged sizes
    x2 = torch.randn(37, 100)
    W2 = torch.randn(70, 100)
    assert torch.allclose(RD.linear(x2.cuda(), W2.cuda(), None).cpu(),
                          x2 @ W2.T, rtol=1e-4, atol=1e-4)


def _check_topk(idx, val, ref_idx, ref_val, all_vals, tol):
    """Same selection up to near-ties: every chosen value matches the
    reference's value at that rank within tol, and indices agree wherever
    the reference's neighbouring ranks are separated by more than tol."""
    assert torch.allclose(val, ref_val, rtol=0, atol=tol)
    same = idx == ref_idx
    if not bool(same.all()):
        bad = (~same).nonzero()
        for r, c in bad.tolist():
            # a swap is allowed only between (near-)equal values
            assert abs(float(all_vals[r, idx[r, c]]) - float(ref_val[r, c])) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("whiten", [True, False])
def test_hip_prep_features_vs_oracle(whiten):
    from splatt3r_amd import retrieval_database as RD
    W, b, cen, pre, post = _weights(C=512, whiten=whiten)
    feat = torch.randn(1, 768, 1024)
    ref_f, ref_a, ref_i = R.prep_features(feat, pre, W, b, False, post, 300)
    db = RD.RetrievalDatabase(RD.RetrievalWeights(W.cuda(), b.cuda(), cen.cuda(),
                                                  tuple(map(_dev, pre)) if pre else None,
                                                  tuple(map(_dev, post)) if post else None),
                              device="cuda")
    got = db.prep_features(feat.cuda()).cpu()
    assert got.shape == (1, 300, 1024)
    # attention values + token order
    x = R.whiten(feat, *pre) if pre else feat
    proj = torch.nn.functional.linear(x, W, b)
    post_t = R.whiten(proj, *post) if post else proj
    fo, ao, io = RD.how_select_local(post_t.cuda(), proj.cuda(), 300)
    _check_topk(io.cpu(), ao.cpu(), ref_i, ref_a, proj.norm(dim=-1), 1e-4)
    # the selected rows: the oracle's postwhitened tokens at the chosen indices
    sel = post_t[0, io.cpu()[0]]
    assert torch.allclose(got[0], sel, rtol=1e-4, atol=1e-4)
    assert torch.allclose(got[0][:50], ref_f[0][:50], rtol=1e-4, atol=1e-4) or \
        bool((io.cpu()[0, :50] != ref_i[0, :50]).any())


@pytest.mark.gpu
def test_hip_select_local_ties_keep_lower_index():
    from splatt3r_amd import retrieval_database as RD
    x = torch.ones(2, 64, 8)
    x[1, 10] = 2.0
    fo, ao, io = RD.how_select_local(x.cuda(), x.cuda(), 5)
    assert io[0].tolist() == [0, 1, 2, 3, 4]
    assert io[1].tolist() == [10, 0, 1, 2, 3]
    assert torch.equal(fo.cpu()[1, 0], x[1, 10])


@pytest.mark.gpu
@pytest.mark.parametrize("M,C,D,k", [(300, 65536, 1024, 5), (300, 65536, 1024, 1),
                                     (37, 1000, 96, 8), (1, 300, 1024, 5)])
def test_hip_quantize_vs_oracle(M, C, D, k):
    from splatt3r_amd import retrieval_database as RD
    g = torch.Generator().manual_seed(M + C + k)
    c = torch.nn.functional.normalize(torch.randn(C, D, generator=g), dim=1)
    q = torch.nn.functional.normalize(torch.randn(M, D, generator=g), dim=1) + 0.3 * c[:M % C + 1].mean(0)
    ref_i, ref_d, l2 = R.quantize(q, c, k)
    cd = c.cuda()
    idx, dist = RD.l2_topk(q.cuda(), cd, RD.row_sqnorm(cd), k)
    _check_topk(idx.cpu(), dist.cpu(), ref_i, ref_d, l2, 1e-4)


@pytest.mark.gpu
def test_hip_quantize_duplicate_centroids_lower_index_first():
    from splatt3r_amd import retrieval_database as RD
    c = torch.randn(700, 32)
    c[650] = c[3]
    q = c[3:4].clone()
    cd = c.cuda()
    idx, dist = RD.l2_topk(q.cuda(), cd, RD.row_sqnorm(cd), 2)
    assert idx.cpu().tolist() == [[3, 650]]


@pytest.mark.gpu
def test_hip_quantize_custom_params():
    from splatt3r_amd import retrieval_database as RD
    W, b, cen, _, _ = _weights(C=4096, whiten=False)
    db = RD.RetrievalDatabase(RD.RetrievalWeights(W.cuda(), b.cuda(), cen.cuda()), device="cuda")
    q = torch.randn(300, 1024).cuda()
    for step, k in (("build_ivf", 1), ("query_ivf", 5)):
        idx = db.quantize_custom(q, RD.ASMK_PARAMS[step])
        assert idx.shape == (300, k) and idx.dtype == torch.int64
