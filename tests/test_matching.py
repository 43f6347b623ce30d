"""Dense matching (include/s3m.h) vs the oracle restatement of
matching_kernels.cu / matching.py, pinned by the reference-importable
img_gradient fixture and by known-answer cases."""
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN


def smooth_pointmap(b, h, w, rng, z=2.0):
    """A smooth surface seen by a pinhole camera (well-posed for iter_proj)."""
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    f = max(h, w)
    x = (u - w / 2) / f
    y = (v - h / 2) / f
    out = []
    for _ in range(b):
        a = rng.normal(size=3) * 0.2
        depth = z + a[0] * np.sin(3 * x) + a[1] * np.cos(2 * y) + a[2] * x * y
        out.append(np.stack([x * depth, y * depth, depth], -1))
    return np.stack(out).astype(np.float32)


def unit_desc(b, h, w, f, rng):
    d = rng.normal(size=(b, h, w, f)).astype(np.float32)
    return d / np.linalg.norm(d, axis=-1, keepdims=True)


# ------------------------------------------------------------- CPU: oracle
def test_oracle_prep_matches_reference_img_gradient():
    g = np.load(os.path.join(GOLDEN, "matching_prep.npz"))
    rays, pts, p_init = oracle.prep_iter_proj(g["X11"], g["X21"])
    # reference uses torch conv2d (summation order unspecified): fp32 tolerance
    np.testing.assert_allclose(rays, g["rays_with_grad"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(pts, g["pts3d_norm"], rtol=1e-6, atol=1e-7)
    b, h, w, _ = g["X11"].shape
    assert p_init[0, w + 3].tolist() == [3.0, 1.0]


def test_oracle_self_match_is_identity():
    rng = np.random.default_rng(0)
    X = smooth_pointmap(1, 24, 32, rng)
    D = unit_desc(1, 24, 32, 24, rng)
    idx, valid = oracle.match(X, X, D, D)
    # border pixels are clamped into [1, w-2] x [1, h-2] by iter_proj
    # (matching_kernels.cu:141-142) and the greedy dilated search then drifts
    # with random descriptors; interior pixels map to themselves except where
    # the LM estimate lands a hair below the integer (x.9999983) and `.long()`
    # (matching.py:68) truncates it, exactly as the reference does.
    ys, xs = np.meshgrid(np.arange(24), np.arange(32), indexing="ij")
    inner = ((ys > 0) & (ys < 23) & (xs > 0) & (xs < 31)).ravel()
    assert (idx[0][inner] == np.arange(24 * 32)[inner]).mean() > 0.95
    assert valid[0, inner, 0].mean() > 0.9


def test_oracle_iter_proj_recovers_planted_shift():
    rng = np.random.default_rng(1)
    h, w = 24, 32
    X11 = smooth_pointmap(1, h, w, rng)
    X21 = np.roll(X11, shift=(2, -3), axis=(1, 2))  # pixel (y,x) sees X11[y-2, x+3]
    rays, pts, p_init = oracle.prep_iter_proj(X11, X21)
    p, conv = oracle.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
    p = p.reshape(h, w, 2)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    inner = (ys >= 4) & (ys < h - 2) & (xs >= 2) & (xs < w - 5)
    np.testing.assert_allclose(p[..., 0][inner], (xs + 3)[inner], atol=0.05)
    np.testing.assert_allclose(p[..., 1][inner], (ys - 2)[inner], atol=0.05)


def test_oracle_refine_finds_best_descriptor():
    rng = np.random.default_rng(2)
    h, w, f = 20, 20, 24
    D11 = unit_desc(1, h, w, f, rng).astype(np.float16)
    D21 = D11[:, 10:11, 13:14].reshape(1, 1, f)  # query = descriptor at (u=13, v=10)
    p1 = np.array([[[11, 9]]], np.int64)          # start 2 px off
    out = oracle.refine_matches(D11, D21, p1, 3, 5)
    assert out[0, 0].tolist() == [13, 10]


def test_oracle_refine_all_negative_scores_keep_start():
    h, w, f = 10, 10, 4
    D11 = np.full((1, h, w, f), 0.5, np.float16)
    D21 = np.full((1, 1, f), -0.5, np.float16)
    out = oracle.refine_matches(D11, D21, np.array([[[4, 5]]], np.int64), 3, 5)
    assert out[0, 0].tolist() == [4, 5]


# -------------------------------------------------------------- GPU: HIP
def _to(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@pytest.mark.gpu
def test_hip_prep_bitexact_vs_oracle_and_golden():
    from splatt3r_amd.matching import prep_for_iter_proj
    g = np.load(os.path.join(GOLDEN, "matching_prep.npz"))
    rays, pts, p_init = prep_for_iter_proj(_to(g["X11"]), _to(g["X21"]), None)
    r_o, p_o, pi_o = oracle.prep_iter_proj(g["X11"], g["X21"])
    np.testing.assert_array_equal(rays.cpu().numpy(), r_o)
    np.testing.assert_array_equal(pts.cpu().numpy(), p_o)
    np.testing.assert_array_equal(p_init.cpu().numpy(), pi_o)
    np.testing.assert_allclose(rays.cpu().numpy(), g["rays_with_grad"], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("b,h,w", [(1, 24, 32), (2, 48, 64), (1, 384, 512)])
def test_hip_iter_proj_bitexact_vs_oracle(b, h, w):
    import mast3r_slam_backends as be
    rng = np.random.default_rng(h)
    X11 = smooth_pointmap(b, h, w, rng)
    X21 = smooth_pointmap(b, h, w, rng) + rng.normal(size=(b, h, w, 3)).astype(np.float32) * 1e-3
    rays, pts, p_init = oracle.prep_iter_proj(X11, X21)
    p_ref, c_ref = oracle.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
    p, c = be.iter_proj(_to(rays), _to(pts), _to(p_init), 10, 1e-8, 1e-6)
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref)
    np.testing.assert_array_equal(c.cpu().numpy(), c_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("f", [24, 16])
def test_hip_refine_bitexact_vs_oracle(f):
    import mast3r_slam_backends as be
    rng = np.random.default_rng(f)
    b, h, w = 2, 40, 56
    D11 = unit_desc(b, h, w, f, rng).astype(np.float16)
    D21 = unit_desc(b, h, w, f, rng).astype(np.float16).reshape(b, h * w, f)
    p1 = np.stack([rng.integers(0, w, size=(b, h * w)), rng.integers(0, h, size=(b, h * w))], -1)
    ref = oracle.refine_matches(D11, D21, p1, 3, 5)
    (out,) = be.refine_matches(_to(D11), _to(D21), _to(p1.astype(np.int64)), 3, 5)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("sort", [0, 0x33])
@pytest.mark.parametrize("lanes,pf", [(1, 4), (1, 6), (2, 2), (2, 4), (3, 4), (4, 3), (16, 3)])
@pytest.mark.parametrize("f,radius,dil", [(24, 3, 5), (24, 2, 3), (32, 1, 2), (24, 4, 2), (8, 3, 5)])
def test_hip_refine_ties_and_windows_vs_oracle(f, radius, dil, lanes, pf, sort):
    """Quantised descriptors make many equal fp16 scores: every kernel must
    keep the first candidate in the reference's scan order.  lanes 1 / 2 / 4
    = k_refine_lane with 1 / 2 / 4 lanes per query (radius 3, f 24; pf its
    load distance), 3 = k_refine_px (3 lanes per pixel, the fp16 chain
    handed lane to lane), 16 = k_refine_coop; radius 4 (81
    candidates) and fdim 8 take the generic per-lane kernel.  Query points
    up to 3 pixels off the image exercise the masked window slots.  sort:
    queries visited in window-centre tile order (8 x 8 tiles) or pixel order."""
    import mast3r_slam_backends as be
    from splatt3r_amd import _lib
    rng = np.random.default_rng(100 + f + radius)
    b, h, w = 2, 33, 47
    D11 = (rng.integers(-2, 3, size=(b, h, w, f)) * 0.125).astype(np.float16)
    D21 = (rng.integers(-2, 3, size=(b, h * w, f)) * 0.125).astype(np.float16)
    p1 = np.stack([rng.integers(-3, w + 3, size=(b, h * w)),
                   rng.integers(-3, h + 3, size=(b, h * w))], -1).astype(np.int64)
    ref = oracle.refine_matches(D11, D21, p1, radius, dil)
    _lib.lib().s3m_refine_set_lanes(lanes)
    _lib.lib().s3m_refine_set_prefetch(pf)
    _lib.lib().s3m_refine_set_sort(sort)
    try:
        (out,) = be.refine_matches(_to(D11), _to(D21), _to(p1), radius, dil)
    finally:
        _lib.lib().s3m_refine_set_lanes(-1)
        _lib.lib().s3m_refine_set_prefetch(4)
        _lib.lib().s3m_refine_set_sort(-1)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("sort", [0x11, 0x60, 0x06, 0x42, 0x66])
@pytest.mark.parametrize("lanes", [1, 3, 4, 16])
def test_hip_refine_tile_orders_vs_oracle(sort, lanes):
    """Window-centre binning with lopsided tiles (2x2, 64x1, 1x64, 16x4,
    64x64: one tile per image), three batches of different query spread
    (one batch's centres all in one tile), off-image centres clamped into
    the edge tiles, and a second call on the same stream (the scan re-zeroes
    the tile counts): every order gives the oracle's bits."""
    import mast3r_slam_backends as be
    from splatt3r_amd import _lib
    rng = np.random.default_rng(sort + lanes)
    b, h, w, f = 3, 37, 61, 24
    D11 = (rng.integers(-2, 3, size=(b, h, w, f)) * 0.125).astype(np.float16)
    D21 = (rng.integers(-2, 3, size=(b, h * w, f)) * 0.125).astype(np.float16)
    p1 = np.stack([rng.integers(-3, w + 3, size=(b, h * w)),
                   rng.integers(-3, h + 3, size=(b, h * w))], -1).astype(np.int64)
    p1[1] = (5, 7)                                  # batch 1: one window centre
    ref = oracle.refine_matches(D11, D21, p1, 3, 5)
    _lib.lib().s3m_refine_set_lanes(lanes)
    _lib.lib().s3m_refine_set_sort(sort)
    try:
        for _ in range(2):
            (out,) = be.refine_matches(_to(D11), _to(D21), _to(p1), 3, 5)
            np.testing.assert_array_equal(out.cpu().numpy(), ref)
    finally:
        _lib.lib().s3m_refine_set_lanes(-1)
        _lib.lib().s3m_refine_set_sort(-1)


@pytest.mark.gpu
def test_hip_match_end_to_end_vs_oracle():
    from splatt3r_amd.matching import match
    rng = np.random.default_rng(7)
    b, h, w = 2, 48, 64
    X11 = smooth_pointmap(b, h, w, rng)
    X21 = np.roll(X11, 1, axis=2) + rng.normal(size=X11.shape).astype(np.float32) * 1e-3
    D11 = unit_desc(b, h, w, 24, rng)
    D21 = unit_desc(b, h, w, 24, rng)
    init = rng.integers(0, h * w, size=(b, h * w)).astype(np.int64)
    for idx_init in (None, init):
        idx_ref, valid_ref = oracle.match(X11, X21, D11, D21, idx_init)
        idx, valid = match(_to(X11), _to(X21), _to(D11), _to(D21),
                           None if idx_init is None else _to(idx_init))
        np.testing.assert_array_equal(idx.cpu().numpy(), idx_ref)
        np.testing.assert_array_equal(valid.cpu().numpy(), valid_ref)


def _tracker_like_init(h, w, rng, shift=(1, 2), jitter=2):
    """The tracker's idx_f2k init (the previous frame's match, tracker.py:
    31-36): a near-identity map, shifted by the inter-frame motion, with a
    few pixels of disagreement (matching_kernels.cu:24-80 starts each
    refine window there)."""
    v, u = np.divmod(np.arange(h * w), w)
    u2 = np.clip(u + shift[1] + rng.integers(-jitter, jitter + 1, h * w), 0, w - 1)
    v2 = np.clip(v + shift[0] + rng.integers(-jitter, jitter + 1, h * w), 0, h - 1)
    return (v2 * w + u2).astype(np.int64)


@pytest.mark.gpu
@pytest.mark.parametrize("lanes,sort", [(None, None), (16, 0), (3, 0), (3, 0x33), (1, 0x33),
                                        (2, 0x42)])
@pytest.mark.parametrize("h,w", [(384, 512), (320, 512)])
def test_hip_refine_full_size_tracker_init_vs_oracle(h, w, lanes, sort):
    """refine_matches at the C2 / C4 frame sizes the tracker runs every
    frame, from tracker-like starting pixels (f = 24, radius 3, dilation 5):
    the default kernel and order (None), and other lanes / window-centre
    tile orders."""
    from splatt3r_amd import _lib
    if lanes is not None:
        _lib.lib().s3m_refine_set_lanes(lanes)
        _lib.lib().s3m_refine_set_sort(sort)
    try:
        _refine_full_size(h, w)
    finally:
        _lib.lib().s3m_refine_set_lanes(-1)
        _lib.lib().s3m_refine_set_sort(-1)


def _refine_full_size(h, w):
    import mast3r_slam_backends as be
    rng = np.random.default_rng(h + w)
    D11 = unit_desc(1, h, w, 24, rng)
    D21 = np.roll(D11, (1, 2), axis=(1, 2)) + rng.normal(size=D11.shape).astype(np.float32) * 0.3
    D21 /= np.linalg.norm(D21, axis=-1, keepdims=True)
    D11h, D21h = D11.astype(np.float16), D21.astype(np.float16).reshape(1, h * w, 24)
    idx0 = _tracker_like_init(h, w, rng)
    p1 = np.stack([idx0 % w, idx0 // w], -1)[None].astype(np.int64)
    ref = oracle.refine_matches(D11h, D21h, p1, 3, 5)
    (out,) = be.refine_matches(_to(D11h), _to(D21h), _to(p1), 3, 5)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(384, 512), (320, 512)])
def test_hip_match_full_size_tracker_init_vs_oracle(h, w):
    """The end-to-end match (prep, iter_proj, occlusion, refine, pixel_to_lin)
    at C2 / C4 size, with and without the tracker-like idx init."""
    from splatt3r_amd.matching import match
    rng = np.random.default_rng(3 * h + w)
    X11 = smooth_pointmap(1, h, w, rng)
    X21 = np.roll(X11, (1, 2), axis=(1, 2)) + rng.normal(size=X11.shape).astype(np.float32) * 1e-3
    D11 = unit_desc(1, h, w, 24, rng)
    D21 = np.roll(D11, (1, 2), axis=(1, 2)) + rng.normal(size=D11.shape).astype(np.float32) * 0.3
    D21 /= np.linalg.norm(D21, axis=-1, keepdims=True)
    for idx_init in (None, _tracker_like_init(h, w, rng)[None]):
        idx_ref, valid_ref = oracle.match(X11, X21, D11, D21, idx_init)
        idx, valid = match(_to(X11), _to(X21), _to(D11), _to(D21),
                           None if idx_init is None else _to(idx_init))
        np.testing.assert_array_equal(idx.cpu().numpy(), idx_ref)
        np.testing.assert_array_equal(valid.cpu().numpy(), valid_ref)
        assert valid_ref.mean() > 0.5


@pytest.mark.gpu
def test_backends_reject_non_contiguous():
    import mast3r_slam_backends as be
    rays = torch.zeros(1, 8, 8, 9, device="cuda")
    pts = torch.zeros(1, 3, 64, device="cuda").transpose(1, 2)
    with pytest.raises(RuntimeError, match="contiguous"):
        be.iter_proj(rays, pts, torch.zeros(1, 64, 2, device="cuda"), 10, 1e-8, 1e-6)


@pytest.mark.gpu
def test_matching_is_exact_while_a_gemm_runs_on_another_stream():
    """The frame loop overlaps the encoder's GEMMs (side stream) with the
    tracker's matching (main stream).  Packed-FP32 VALU instructions return
    wrong values while MFMAs of another kernel share the CU (csrc/build.py
    NO_PACKED_FP32): with them, 30-93 % of the matching launches overlapped
    by a GEMM came out different (tools/stress_bd_concurrency.py).  Here a
    library GEMM replays on a side stream while the dense matching runs
    again and again on the main stream: every result must equal the result
    on an idle device, bit for bit."""
    import time
    from splatt3r_amd import _lib, ops
    from splatt3r_amd.matching import match
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    h, w = 384, 512
    yy, xx = torch.meshgrid(torch.arange(h, device=dev, dtype=torch.float32),
                            torch.arange(w, device=dev, dtype=torch.float32), indexing="ij")
    X11 = torch.stack((xx / w - 0.5, yy / h - 0.5, torch.ones_like(xx)), -1)[None]
    X21 = X11 + 0.002 * torch.randn(X11.shape, device=dev, generator=g)
    D11 = torch.randn(1, h, w, 24, device=dev, generator=g).half()
    D21 = D11 + 0.05 * torch.randn(D11.shape, device=dev, generator=g).half()
    M, N, K = 1536, 4096, 1024
    A = torch.randn(M, K, device=dev, generator=g).half()
    Bw = torch.randn(N, K, device=dev, generator=g).half() * 0.03
    C = torch.empty(M, N, device=dev).half()
    gemm = ops.gemm([A], [Bw], [C], M, N, K, lda=K, bias=[torch.zeros(N, device=dev)],
                    act="gelu", tile=25, split_k=1)
    torch.cuda.synchronize()
    ref = match(X11, X21, D11, D21)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    outs = []
    t_end = time.time() + 3.0
    while time.time() < t_end:
        with torch.cuda.stream(side):
            for _ in range(16):
                gemm(_lib.stream(dev))
        for _ in range(8):
            outs.append(match(X11, X21, D11, D21))
        if len(outs) >= 64:
            torch.cuda.synchronize()
            bad = sum(not (torch.equal(i, ref[0]) and torch.equal(v, ref[1])) for i, v in outs)
            assert bad == 0, f"{bad} of {len(outs)} overlapped matching calls differ"
            outs = []
    torch.cuda.synchronize()
    bad = sum(not (torch.equal(i, ref[0]) and torch.equal(v, ref[1])) for i, v in outs)
    assert bad == 0, f"{bad} of {len(outs)} overlapped matching calls differ"
