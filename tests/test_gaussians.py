"""gaussians_to_world: HIP pass (include/s3w.h) vs the torch-CPU oracle
(oracle/gaussians_ref.py, restating splatt3r_utils.py:180-328).
Selection and order are bit-exact (same mask, same compaction order);
float outputs within 1e-5 relative (matmul summation order)."""
import numpy as np
import pytest
import torch

import oracle.gaussians_ref as GR


def _pred(H, W, seed, nan_frac=0.0):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(1, H, W, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    means = torch.randn(1, H, W, 3, generator=g) * 0.5
    means[..., 2] = torch.rand(1, H, W, generator=g) * 4 - 0.5      # some z <= depth_min
    p = dict(means=means,
             scales=torch.exp(torch.randn(1, H, W, 3, generator=g) - 2.5),
             rotations=q, sh=torch.randn(1, H, W, 3, 1, generator=g) * 0.3,
             opacities=torch.rand(1, H, W, 1, generator=g),
             conf=1 + torch.rand(1, H, W, generator=g) * 2)
    img = torch.rand(1, 3, H, W, generator=g) * 2.2 - 1.1
    return p, img


def _pose():
    th = 0.3
    M = torch.eye(4)
    R = torch.tensor([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]],
                     dtype=torch.float32)
    M[:3, :3] = R * 1.3
    M[:3, 3] = torch.tensor([0.2, -0.1, 0.5])
    return M


def test_oracle_quantile_filter_semantics():
    p, img = _pred(16, 24, 0)
    out = GR.gaussians_to_world([p], img, _pose(), 1, 0.05, 0.98, 0.5, 1.5)
    z = p["means"][0, ..., 2].reshape(-1)
    zv = z[z > 0.05]
    zu = np.quantile(zv.numpy().astype(np.float64), 0.98)
    keep = (z > 0.05) & (z.double() <= zu + 1e-6) & (p["scales"][0].reshape(-1, 3).max(-1).values < 0.5) \
        & (p["conf"][0].reshape(-1) >= 1.5)
    assert out[0].shape[0] == int(keep.sum())


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,stride,q,maxs,minc", [
    (384, 512, 4, 0.98, 1.0, 1.5), (384, 512, 1, 0.98, 0.5, 1.5), (48, 64, 3, 1.0, 0.5, 0.0),
    (50, 70, 4, 0.5, 10.0, 2.0)])
def test_gaussians_to_world_gpu_vs_oracle(H, W, stride, q, maxs, minc):
    import lietorch
    from splatt3r_amd.frame import Frame
    from splatt3r_amd.splatt3r_utils import gaussians_to_world
    p, img = _pred(H, W, H * W + stride)
    M = _pose()
    want = GR.gaussians_to_world([p], img, M, stride, 0.05, q, maxs, minc)
    # a Sim3 whose matrix is M: rotation about y by 0.3, scale 1.3
    T = torch.tensor([[0.2, -0.1, 0.5, 0.0, np.sin(0.15), 0.0, np.cos(0.15), 1.3]],
                     dtype=torch.float32).cuda()
    fr = Frame(0, img.cuda(), None, None, T_WC=lietorch.Sim3(T))
    fr.gaussian_pred = {k: v.cuda() for k, v in p.items()}
    got = gaussians_to_world(fr, include_cross=False, spatial_stride=stride,
                             depth_max_percentile=q, max_scale=maxs, min_confidence=minc)
    assert got[0].shape[0] == want[0].shape[0]
    for g, w, tol in zip(got, want, (2e-5, 1e-4, 1e-5, 0)):
        np.testing.assert_allclose(g.cpu().numpy(), w.numpy(), rtol=tol, atol=tol * 1e-2)


@pytest.mark.gpu
def test_gaussians_to_world_all_filtered_returns_none():
    import lietorch
    from splatt3r_amd.frame import Frame
    from splatt3r_amd.splatt3r_utils import gaussians_to_world
    p, img = _pred(32, 32, 5)
    p["means"][..., 2] = -1.0
    fr = Frame(0, img.cuda(), None, None, T_WC=lietorch.Sim3.Identity(1, device="cuda"))
    fr.gaussian_pred = {k: v.cuda() for k, v in p.items()}
    assert gaussians_to_world(fr, include_cross=False, spatial_stride=2) is None


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,stride,q,maxs,minc,dmin", [
    (384, 512, 4, 0.98, 1.0, 1.5, 0.05), (96, 128, 1, 0.98, 0.5, 1.5, 0.05),
    (48, 64, 3, 1.0, 0.5, 0.0, 0.05), (50, 70, 4, 0.5, 10.0, 2.0, 0.05),
    (175, 175, 1, 0.3, 10.0, 0.0, float("-inf")), (1, 1, 1, 0.98, 10.0, 0.0, 0.05),
    (256, 256, 2, 0.98, 10.0, 0.0, 5.0)])
def test_single_launch_path_equals_multi_pass(H, W, stride, q, maxs, minc, dmin):
    """s3w_gaussians_to_world's two-launch path (n <= 30720: one workgroup
    radix-selects the two quantile order statistics in LDS and block-scans
    the filter flags, then a chip-wide emit) returns the multi-pass path's
    records and count bit for bit: the tracker's stride-4 view, stride 1,
    no quantile, n0 = 0 (every z below depth_min), depth_min = -inf
    (negative z, 30625 Gaussians), n = 1."""
    from splatt3r_amd import _lib
    from splatt3r_amd.splatt3r_utils import world_records
    p, img = _pred(H, W, 7 * H + W)
    if dmin == float("-inf"):
        p["means"][..., 2] -= 1.0
    view = {k: v[0].cuda() for k, v in p.items()}
    T = _pose().cuda()
    lib = _lib.lib()
    outs = []
    try:
        for path in (1, 2):
            lib.s3w_set_path(path)
            rec, cnt = world_records(view, img[0].cuda(), T, stride, dmin, q, maxs, minc)
            torch.cuda.synchronize()
            outs.append((rec[:int(cnt.item())].cpu(), int(cnt.item())))
    finally:
        lib.s3w_set_path(0)
    (r1, c1), (r2, c2) = outs
    assert c1 == c2
    assert torch.equal(r1, r2)
