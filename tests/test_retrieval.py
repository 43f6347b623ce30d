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
    # rows may differ only where the device path's own projection broke a
    # near-tie of attention values the other way: such a row must be the
    # postwhitened token whose attention is within tol of that rank's value
    row_ok = torch.isclose(got[0], sel, rtol=1e-4, atol=1e-4).all(-1)
    norms = proj.norm(dim=-1)[0]
    for c in (~row_ok).nonzero().flatten().tolist():
        j = int((post_t[0] - got[0, c]).abs().amax(-1).argmin())
        assert torch.allclose(post_t[0, j], got[0, c], rtol=1e-4, atol=1e-4)
        assert abs(float(norms[j]) - float(ao.cpu()[0, c])) <= 1e-4, (c, j)
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


# ------------------------------------------------------------------ ASMK ---
def _asmk_case(seed, n=300, D=1024, C=4096, k=5):
    g = torch.Generator().manual_seed(seed)
    cen = torch.nn.functional.normalize(torch.randn(C, D, generator=g), dim=1)
    feats = torch.nn.functional.normalize(torch.randn(n, D, generator=g), dim=1)
    return cen, feats


def test_oracle_asmk_self_match_scores_one_per_word():
    """An image queried against itself (same assignments) scores 1 per
    shared word (hamming 0): sum = number of words."""
    from oracle.retrieval_ref import asmk_aggregate, asmk_search, quantize
    cen, f = _asmk_case(0, n=40, D=64, C=256)
    idx, _, _ = quantize(f, cen, 1)
    w, c = asmk_aggregate(f.numpy(), idx.numpy(), cen.numpy())
    s = asmk_search(w, c, w, np.zeros(len(w), np.int32), c, 64, 1)
    assert s[0] == len(w)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 5])
def test_hip_asmk_aggregate_matches_oracle(k):
    from oracle.retrieval_ref import asmk_aggregate as ref_agg, quantize
    from splatt3r_amd.retrieval_database import asmk_aggregate
    cen, f = _asmk_case(1)
    idx, _, _ = quantize(f, cen, k)
    w, c, n = asmk_aggregate(f.cuda(), idx.cuda(), cen.cuda())
    rw, rc = ref_agg(f.numpy(), idx.numpy(), cen.numpy())
    n = int(n.item())
    assert n == len(rw)
    np.testing.assert_array_equal(w[:n].cpu().numpy(), rw)
    np.testing.assert_array_equal(c[:n].cpu().numpy().view(np.uint32), rc)


@pytest.mark.gpu
def test_hip_retrieval_database_update_matches_oracle():
    """RetrievalDatabase.update over a keyframe sequence (query k=3 then add,
    retrieval_database.py:43-72): same retrieved keyframes as the restated
    ASMK database on the same features, and the revisited place is found."""
    from oracle.retrieval_ref import RetrievalDBRef, asmk_search
    from splatt3r_amd.retrieval_database import RetrievalDatabase, RetrievalWeights
    D, C = 256, 2048
    g = torch.Generator().manual_seed(3)
    cen = torch.nn.functional.normalize(torch.randn(C, D, generator=g), dim=1)
    W = RetrievalWeights(torch.eye(D, 1024)[:D].cuda(), torch.zeros(D).cuda(), cen.cuda(), nfeat=100)
    db = RetrievalDatabase(W, device="cuda")
    ref = RetrievalDBRef(cen.numpy())
    places = [torch.nn.functional.normalize(torch.randn(100, D, generator=g), dim=1)
              for _ in range(5)]
    seq = [0, 1, 2, 3, 4, 2, 0]          # keyframes 5 and 6 revisit places 2 and 0
    got_all = []
    for t, p in enumerate(seq):
        feat = torch.nn.functional.normalize(places[p] + 0.05 * torch.randn(100, D, generator=g),
                                             dim=1)
        # bypass prep_features: the ASMK half is under test here
        fd = feat.cuda()
        scores_codes = None
        inds = []
        if db.kf_counter > 0:
            scores, codes = db.query(fd)
            top = torch.topk(scores.float(), min(3, db.ivf.n_images))
            inds = top.indices[top.values > 5e-3].tolist()
            scores_codes = codes
        db.add_to_database(fd, scores_codes)
        want = ref.update(feat.numpy(), True, 3, 5e-3)
        assert inds == want, (t, inds, want)
        got_all.append(inds)
    assert got_all[5][0] == 2 and got_all[6][0] == 0


# ------------------------------------------- checkpoint-backed constructor ---
def _write_retrieval_ckpt(tmp_path, hdims="1024", residual=False, C=64, seed=5):
    """A file with the layout of the MASt3R retrieval checkpoint
    (processor.py:66-78: {'args': Namespace, 'model': state dict without the
    frozen backbone}) and the codebook beside it as .npy (the reference's
    <prefix>_codebook.pkl is a pickle, not read by this build)."""
    import argparse
    g = torch.Generator().manual_seed(seed)
    dims = [int(x) for x in hdims.split("_")] if hdims else []
    sd = {"prewhiten.m": torch.randn(1, 1024, generator=g, dtype=torch.float64) * 0.1,
          "prewhiten.p": torch.randn(1024, 1024, generator=g, dtype=torch.float64) / 32}
    d = 1024
    for i, h in enumerate(dims):
        sd[f"projector.{3 * i}.weight"] = torch.randn(h, d, generator=g) / d ** 0.5
        sd[f"projector.{3 * i}.bias"] = torch.randn(h, generator=g) * 0.01
        if i < len(dims) - 1:
            sd[f"projector.{3 * i + 1}.weight"] = 1 + 0.1 * torch.randn(h, generator=g)
            sd[f"projector.{3 * i + 1}.bias"] = 0.1 * torch.randn(h, generator=g)
        d = h
    sd["postwhiten.m"] = torch.randn(1, d, generator=g, dtype=torch.float64) * 0.1
    sd["postwhiten.p"] = torch.randn(d, d, generator=g, dtype=torch.float64) / d ** 0.5
    args = argparse.Namespace(pretrained="x", freeze_backbone=1, prewhiten=-1, hdims=hdims,
                              residual=residual, postwhiten=-1, featweights="l2norm", nfeat=300,
                              nclusters=C, imsize=512)
    path = tmp_path / "MASt3R_ViTLarge_BaseDecoder_512_catmlpdpt_metric_retrieval_trainingfree.pth"
    torch.save({"args": args, "model": sd}, str(path))
    cen = torch.nn.functional.normalize(torch.randn(C, d, generator=g), dim=1).numpy()
    np.save(str(tmp_path / "MASt3R_ViTLarge_BaseDecoder_512_catmlpdpt_metric_retrieval_codebook.npy"),
            cen)
    return str(path), sd, cen


def test_retrieval_checkpoint_maps_onto_weights(tmp_path):
    from splatt3r_amd.retrieval_database import load_retrieval_weights
    path, sd, cen = _write_retrieval_ckpt(tmp_path, hdims="512_1024")
    w = load_retrieval_weights(path, device="cpu")
    assert torch.equal(w.prewhiten[1], sd["prewhiten.p"]) and w.prewhiten[1].dtype == torch.float64
    assert torch.equal(w.postwhiten[0], sd["postwhiten.m"])
    assert len(w.hidden) == 1 and torch.equal(w.hidden[0][0], sd["projector.0.weight"])
    assert torch.equal(w.hidden[0][2], sd["projector.1.weight"])
    assert torch.equal(w.proj_W, sd["projector.3.weight"])
    assert torch.equal(w.centroids, torch.from_numpy(cen))
    assert w.nfeat == 300 and not w.residual


def test_retrieval_codebook_pickle_is_refused(tmp_path):
    from splatt3r_amd.retrieval_database import load_retrieval_weights
    path, _, _ = _write_retrieval_ckpt(tmp_path)
    npy = tmp_path / "MASt3R_ViTLarge_BaseDecoder_512_catmlpdpt_metric_retrieval_codebook.npy"
    npy.rename(npy.with_suffix(".pkl"))
    with pytest.raises(RuntimeError, match="pickle"):
        load_retrieval_weights(path, device="cpu")


def test_retrieval_missing_checkpoint_raises(tmp_path):
    from splatt3r_amd.retrieval_database import load_retrieval_weights
    with pytest.raises(FileNotFoundError):
        load_retrieval_weights(str(tmp_path / "nope.pth"), device="cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("hdims,residual", [("1024", False), ("1024", True), ("512_1024", False)])
def test_hip_load_retriever_from_checkpoint_vs_torch(tmp_path, hdims, residual):
    """load_retriever(model, path) (splatt3r_utils.py:69-89) -> prep_features
    on the device == RetrievalModel.extract_features_and_attention +
    how_select_local (model.py:62-157, 89-103) in torch fp64/fp32 on the CPU."""
    from types import SimpleNamespace
    from splatt3r_amd.splatt3r_utils import load_retriever
    path, sd, cen = _write_retrieval_ckpt(tmp_path, hdims=hdims, residual=residual)
    db = load_retriever(SimpleNamespace(encoder="enc"), path, device="cuda")
    assert db.backbone == "enc" and db.centroids.shape == (64, 1024)
    feat = torch.randn(1, 768, 1024, generator=torch.Generator().manual_seed(2))
    x = R.whiten(feat, sd["prewhiten.m"], sd["prewhiten.p"])
    h = x
    dims = hdims.split("_")
    for i in range(len(dims) - 1):
        h = torch.nn.functional.linear(h, sd[f"projector.{3 * i}.weight"], sd[f"projector.{3 * i}.bias"])
        h = torch.nn.functional.gelu(torch.nn.functional.layer_norm(
            h, h.shape[-1:], sd[f"projector.{3 * i + 1}.weight"], sd[f"projector.{3 * i + 1}.bias"]))
    j = 3 * (len(dims) - 1)
    proj = torch.nn.functional.linear(h, sd[f"projector.{j}.weight"], sd[f"projector.{j}.bias"])
    if residual:
        proj = proj + x
    post = R.whiten(proj, sd["postwhiten.m"], sd["postwhiten.p"])
    attn = proj.norm(dim=-1)
    got = db.prep_features(feat.cuda()).cpu()
    ta, ti = torch.topk(attn, 300, dim=1)
    # rows at the reference's top-300 attention order, up to near-ties
    sel = post[0, ti[0]]
    ok = torch.isclose(got[0], sel, rtol=2e-4, atol=2e-4).all(-1)
    gap = (ta[0, :-1] - ta[0, 1:]).abs()
    for c in (~ok).nonzero().flatten().tolist():
        near = min(float(gap[c - 1]) if c > 0 else 1.0, float(gap[c]) if c < 299 else 1.0)
        assert near < 1e-3, c


def test_every_name_the_reference_imports_from_splatt3r_utils():
    """main.py:41-47, tracker.py:12, global_opt.py:8, frame.py:6,
    dataloader.py:10 import these from splatt3r_slam.splatt3r_utils."""
    import importlib
    names = {"load_splatt3r", "load_retriever", "splatt3r_inference_mono", "splatt3r_render",
             "gaussians_to_world", "splatt3r_match_asymmetric", "splatt3r_match_symmetric",
             "resize_img"}
    import os
    ref = "/root/reference"
    if os.path.isdir(ref):                     # cross-check the list where the reference is
        import re
        for f in ("main.py", "splatt3r_slam/tracker.py", "splatt3r_slam/global_opt.py",
                  "splatt3r_slam/frame.py", "splatt3r_slam/dataloader.py"):
            src = open(os.path.join(ref, f)).read()
            for m in re.finditer(r"from splatt3r_slam\.splatt3r_utils import \(?([^)]*?)\)?\n"
                                 r"(?=\S|$)", src, re.S):
                got = {n.strip() for n in m.group(1).replace("\n", ",").split(",") if n.strip()}
                assert got <= names, got - names
    mod = importlib.import_module("splatt3r_amd.splatt3r_utils")
    for n in sorted(names):
        assert callable(getattr(mod, n)), n
