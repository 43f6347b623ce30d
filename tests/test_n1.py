"""North-star acceptance N1: rendered RGB within 1e-3 mean-L1 of the
reference path.

Reference side (tests/golden/n1_render.npz, oracle/gen_golden.py `n1`): the
reference network (imported reference modules, portable-PRNG weights with
the conditioned init `weights.n1_init`) on smooth uint8 frames -> the
reference render glue (splatt3r_utils.py:332-432 -> decoder_splatting_cuda.py
-> cuda_splatting.py, imported, with a stub that captures the rasterizer
inputs) -> oracle.raster (canonical graphdeco forward, oracle/raster_ref.c).
Each image is stored in fp32 and as the reference CUDA path computes it
(TF32 matrix products, main.py:195, emulated by gen_golden.tf32_mode).

Why a conditioned init: the reference init of the Gaussian head
(catmlp_dpt_head.py:222-238) makes every scale e^-7 (sub-pixel splats) and
every opacity ~sigmoid(-2); rendered with it the image is a step function of
the means (round 2: d_ref = |ref_tf32 - ref_fp32| up to 2.5e-3, and an
all-black image passed the 1e-3 bar on two views).  `n1_init` keeps the
PRNG streams and only re-scales the final convs: scales of ~10-30 px that
vary per splat, colours from the image, opacity ~0.5, points in front of the
camera.  The fixture is then well conditioned: every view has mean >= 0.1
and d_ref <= 2e-4 (`test_n1_fixture_is_conditioned`).

Bar, per image (small 48x64, full 384x512 = C2, full 320x512 = C4; self,
moved and look-at views), no escape clause:
  * mean |ours - ref_tf32| <= 1e-3 and mean |ours - ref_fp32| <= 1e-3;
  * relative mean-L1 (vs the reference image's mean) < 2 %;
  * the Gaussian head outputs (scales non-constant, opacities, means) within
    the network tolerance of tests/test_net.py;
  * glue + rasterizer alone (the reference head outputs fed to our render,
    small configs): mean |ours - ref_fp32| <= 1e-5.
All distances are recorded by the `parity` fixture.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

N1_TOL = 1e-3
REL_TOL = 0.02
GLUE_TOL = 1e-5
DREF_MAX = 2e-4
HEAD_TOL = 8e-3          # tests/test_net.py TOL["heads"], relative to scale
POSES = ("self", "moved", "lookat")
KEYS = ("means", "scales", "rotations", "sh", "opacities")
CASES = {"small_off": ("small", True, 48, 64), "small_nooff": ("small", False, 48, 64),
         "full_384x512": ("full", True, 384, 512), "full_320x512": ("full", True, 320, 512)}


def _load():
    return np.load(os.path.join(GOLDEN, "n1_render.npz"))


def _ref_images(n1, tag, pose):
    """(fp32 image, TF32 image) as float64 [3, H, W]."""
    img = n1[f"{tag}_{pose}_image_u16"].astype(np.float64) / float(n1["q16"])
    return img, img + n1[f"{tag}_{pose}_tf32_delta"].astype(np.float64) / float(n1["dq"])


def _normalise(u8):
    """uint8 HxWx3 -> ImgNorm [1,3,H,W] (bit-identical to gen_golden.n1_normalise)."""
    a = torch.from_numpy(u8.astype(np.float32) / np.float32(255.0)).permute(2, 0, 1)[None]
    return ((a - 0.5) / 0.5).contiguous()


def _cfg(n1, tag):
    from splatt3r_amd import weights as W
    kind, use_off, _, _ = CASES[tag]
    base = W.FULL if kind == "full" else dataclasses.replace(W.SMALL, use_offsets=use_off)
    return W.n1_init(base, float(n1[f"{tag}_scale_bias"]))


def test_n1_fixture_is_conditioned():
    """Every reference view carries signal and the reference's own TF32 path
    is far inside the 1e-3 bar (so the bar can fail)."""
    n1 = _load()
    for tag in CASES:
        for pose in POSES:
            ref, ref_t = _ref_images(n1, tag, pose)
            assert ref.mean() >= 0.1, (tag, pose, ref.mean())
            assert (ref.sum(0) > 0).mean() > 0.5, (tag, pose)
            assert np.abs(ref_t - ref).mean() <= DREF_MAX, (tag, pose)
        sc = n1[f"{tag}_res1_scales"]
        assert np.log(sc).std() > 0.02, tag          # scales vary (not the constant e^-7)
        assert 0.2 < float(np.median(n1[f"{tag}_res1_opacities"])) < 0.8, tag


def test_n1_init_differs_from_reference_init_only_in_final_convs():
    """n1_init re-scales the two final 1x1 convs and nothing else."""
    from splatt3r_amd import weights as W
    cfg = W.n1_init(W.SMALL, -1.2)
    for name, shape in W.manifest(W.SMALL):
        a = W.prng_tensor_numpy(1234, name, shape, W.SMALL)
        b = W.prng_tensor_numpy(1234, name, shape, cfg)
        if name.endswith("head.4.weight") or name.endswith("head.4.bias"):
            continue
        np.testing.assert_array_equal(a, b, err_msg=name)
    bias = W.prng_tensor_numpy(1234, "downstream_head1.gaussian_dpt.dpt.head.4.bias", (14,), cfg)
    np.testing.assert_array_equal(bias[3:6], np.float32(-1.2))
    np.testing.assert_array_equal(bias[13], np.float32(0.0))


def _frames(img1, img2, ctx):
    import lietorch
    from splatt3r_amd.frame import create_frame
    T = lietorch.Sim3(torch.tensor(ctx, dtype=torch.float32, device="cuda").reshape(1, 8))
    f = create_frame(0, img1, T_WC=T, device="cuda")
    kf = create_frame(1, img2, device="cuda")
    return f, kf


def _render(model, f, kf, tgt):
    import lietorch
    from splatt3r_amd.splatt3r_utils import splatt3r_render
    Tt = lietorch.Sim3(torch.tensor(tgt, dtype=torch.float32, device="cuda").reshape(1, 8))
    out = splatt3r_render(model, f, kf, K=None, target_T_WC=Tt)
    assert out.shape[:3] == (1, 1, 3)
    return out[0, 0].float().cpu().numpy()


def _model(cfg, graphs):
    from splatt3r_amd.net import Splatt3RNet
    from splatt3r_amd.render import DecoderSplattingCUDA
    from splatt3r_amd.splatt3r_utils import Splatt3RModel
    net = Splatt3RNet(cfg, seed=1234, graphs=graphs)
    return Splatt3RModel(net, DecoderSplattingCUDA([0.0, 0.0, 0.0]).cuda())


def _check_image(parity, key, ours, ref, ref_t):
    o = ours.astype(np.float64)
    vals = dict(mean_l1=np.abs(o - ref).mean(), ours_vs_ref_tf32=np.abs(o - ref_t).mean(),
                ref_tf32_vs_fp32=np.abs(ref_t - ref).mean(), max_abs=np.abs(o - ref_t).max(),
                ref_mean=ref.mean())
    vals["rel_mean_l1"] = vals["ours_vs_ref_tf32"] / ref.mean()
    parity(key, **vals, tol=N1_TOL, rel_tol=REL_TOL, metric="mean_l1")
    assert vals["ours_vs_ref_tf32"] <= N1_TOL, (key, vals)
    assert vals["mean_l1"] <= N1_TOL, (key, vals)
    assert vals["rel_mean_l1"] < REL_TOL, (key, vals)


def _check_heads(parity, n1, tag, ours, sub):
    """Head outputs of the conditioned init vs the reference (max error
    relative to each output's scale, as tests/test_net.py)."""
    for i, r in ((1, ours[0]), (2, ours[1])):
        for k in ("scales", "opacities", "means"):
            ref = n1[f"{tag}_res{i}_{k}"].astype(np.float64)
            got = r[k][sub].float().cpu().numpy().astype(np.float64)
            assert got.shape == ref.shape, (tag, k, got.shape, ref.shape)
            err = np.abs(got - ref).max() / (np.abs(ref).max() + 1e-12)
            parity(f"n1_{tag}_res{i}_{k}", max_rel=err, tol=HEAD_TOL, metric="max_rel")
            assert err <= HEAD_TOL, (tag, i, k, err)
        sc = r["scales"].float()
        assert float(sc.log().std()) > 0.02, (tag, "scales are constant")


def _run_case(parity, tag, model, glue):
    from splatt3r_amd.splatt3r_utils import _extract_gaussian_params
    n1 = _load()
    _, _, H, Wd = CASES[tag]
    img1, img2 = _normalise(n1[f"{tag}_u8img1"]), _normalise(n1[f"{tag}_u8img2"])
    net = model.encoder
    f1, p1, _ = net._encode_image(img1.cuda(), None)
    f2, p2, _ = net._encode_image(img2.cuda(), None)
    r1, r2, _ = net.infer_pair(f1, p1, f2, p2, (H, Wd))
    gp, gc = _extract_gaussian_params(r1), _extract_gaussian_params(r2)
    sub = (slice(None), slice(None, None, 8), slice(None, None, 8)) if H > 64 else (slice(None),)
    _check_heads(parity, n1, tag, (r1, r2), sub)
    refs = None
    if glue:
        refs = tuple({k: torch.from_numpy(n1[f"{tag}_res{i}_{k}"]).cuda() for k in KEYS}
                     for i in (1, 2))
    for pose in POSES:
        ref, ref_t = _ref_images(n1, tag, pose)
        f, kf = _frames(img1, img2, n1[f"{tag}_{pose}_ctx"])
        f.gaussian_pred, f.gaussian_pred_cross = gp, gc
        _check_image(parity, f"n1_{tag}_{pose}_network", _render(model, f, kf,
                                                                  n1[f"{tag}_{pose}_tgt"]),
                     ref, ref_t)
        if refs is not None:
            f, kf = _frames(img1, img2, n1[f"{tag}_{pose}_ctx"])
            f.gaussian_pred, f.gaussian_pred_cross = refs
            img = _render(model, f, kf, n1[f"{tag}_{pose}_tgt"]).astype(np.float64)
            d = np.abs(img - ref)
            parity(f"n1_{tag}_{pose}_glue", mean_l1=d.mean(), max_abs=d.max(), tol=GLUE_TOL,
                   metric="mean_l1")
            assert d.mean() <= GLUE_TOL, (tag, pose, d.mean())


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["small_off", "small_nooff"])
def test_n1_small_network_render_vs_reference(tag, parity):
    n1 = _load()
    _run_case(parity, tag, _model(_cfg(n1, tag), graphs=False), glue=True)


@pytest.mark.gpu
def test_n1_full_network_render_vs_reference(parity):
    """Full architecture at 384x512 (C2) and 320x512 (C4): HIP network +
    render vs the reference network + glue + oracle raster."""
    n1 = _load()
    model = _model(_cfg(n1, "full_384x512"), graphs=True)
    for tag in ("full_384x512", "full_320x512"):
        _run_case(parity, tag, model, glue=False)
