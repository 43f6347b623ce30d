"""World-space Gaussian map (SharedGaussians, frame.py:357-463) and the
full-map render (visualization.py:467-600).

Append: HIP (include/s3w.h s3w_map_append) vs the numpy restatement
oracle/gaussians_ref.MapRef -- bit-exact (pure copies and selection).
Full-map render: tests/golden/viz_render.npz holds the reference's own
_render_gs_interactive driven on a synthetic map with a stub rasterizer
(settings + inputs captured) and oracle.raster's image; our camera math,
scale-invariant copies and HIP raster must reproduce them (settings 1e-6,
inputs and image bit-exact).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.gaussians_ref import MapRef


def _batch(rng, n):
    return (rng.normal(size=(n, 3)).astype(np.float32), rng.normal(size=(n, 6)).astype(np.float32),
            rng.uniform(0, 1, (n, 3)).astype(np.float32), rng.uniform(0, 1, n).astype(np.float32))


def test_oracle_map_eviction_and_truncation():
    m = MapRef(10)
    rng = np.random.default_rng(0)
    a = _batch(rng, 8)
    m.append(*a, kf_idx=0, thr=-1.0)
    assert m.n == 8
    b = _batch(rng, 5)
    m.append(*b, kf_idx=1, thr=-1.0)         # space 2 -> truncated to 2, no eviction
    assert m.n == 10 and list(m.kf) == [0] * 8 + [1] * 2
    np.testing.assert_array_equal(m.means[8:10], b[0][:2])
    c = _batch(rng, 3)
    m.append(*c, kf_idx=2, thr=-1.0)         # full: newest half to the front, then append
    assert m.n == 8
    np.testing.assert_array_equal(m.means[:3], a[0][5:8])
    np.testing.assert_array_equal(m.means[3:5], b[0][:2])
    np.testing.assert_array_equal(m.means[5:8], c[0])
    m.append(*_batch(rng, 4), kf_idx=3, thr=2.0)   # everything filtered: no-op
    assert m.n == 8


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [1000, 1001])
def test_hip_map_append_matches_oracle(cap):
    from splatt3r_amd.gaussian_map import SharedGaussians
    rng = np.random.default_rng(cap)
    gm = SharedGaussians(max_gaussians=cap, device="cuda")
    ref = MapRef(cap)
    for step, n in enumerate([300, 0, 450, 700, 120, 999, 1, 640, 333, 0, 800]):
        b = _batch(rng, n)
        thr = 0.3 if step % 3 else 0.05
        ref.append(*b, kf_idx=step, thr=thr)
        if n:
            gm.append(*(torch.from_numpy(x).cuda() for x in b), kf_idx=step,
                      opacity_threshold=thr)
        assert gm.n_gaussians == ref.n, step
        k = ref.n
        np.testing.assert_array_equal(gm.means[:k].cpu().numpy(), ref.means[:k])
        np.testing.assert_array_equal(gm.cov_triu[:k].cpu().numpy(), ref.cov[:k])
        np.testing.assert_array_equal(gm.colors[:k].cpu().numpy(), ref.colors[:k])
        np.testing.assert_array_equal(gm.opacities[:k].cpu().numpy(), ref.opac[:k])
        np.testing.assert_array_equal(gm.kf_id[:k].cpu().numpy(), ref.kf[:k])
    gm.clear()
    assert gm.get_all() is None


@pytest.mark.gpu
def test_hip_map_append_from_world_records_respects_device_count():
    """append_records reads the valid row count from the device (the output
    of s3w_gaussians_to_world): rows past it are ignored."""
    from splatt3r_amd.gaussian_map import SharedGaussians
    rng = np.random.default_rng(5)
    rec = rng.uniform(0, 1, (500, 13)).astype(np.float32)
    gm = SharedGaussians(max_gaussians=4096, device="cuda")
    cnt = torch.tensor([321], dtype=torch.int64, device="cuda")
    gm.append_records(torch.from_numpy(rec).cuda(), cnt, kf_idx=7, opacity_threshold=0.3)
    ref = MapRef(4096)
    r = rec[:321]
    ref.append(r[:, :3], r[:, 3:9], r[:, 9:12], r[:, 12], 7, 0.3)
    assert gm.n_gaussians == ref.n
    np.testing.assert_array_equal(gm.means[:ref.n].cpu().numpy(), ref.means[:ref.n])
    np.testing.assert_array_equal(gm.opacities[:ref.n].cpu().numpy(), ref.opac[:ref.n])


@pytest.mark.gpu
def test_hip_map_empty_batch_on_full_map_is_a_noop():
    """frame.py:414-416: an append whose batch is empty after the opacity
    filter returns before the FIFO eviction.  Full map + (a) every record
    below the threshold, (b) a device count of 0, (c) then a real batch
    (evicts once, exactly like MapRef)."""
    from splatt3r_amd.gaussian_map import SharedGaussians
    rng = np.random.default_rng(17)
    cap = 600
    gm = SharedGaussians(max_gaussians=cap, device="cuda")
    ref = MapRef(cap)
    b = _batch(rng, cap)
    ref.append(*b, kf_idx=0, thr=-1.0)
    gm.append(*(torch.from_numpy(x).cuda() for x in b), kf_idx=0, opacity_threshold=-1.0)
    assert gm.n_gaussians == ref.n == cap

    def check():
        k = ref.n
        assert gm.n_gaussians == k
        np.testing.assert_array_equal(gm.means[:k].cpu().numpy(), ref.means[:k])
        np.testing.assert_array_equal(gm.opacities[:k].cpu().numpy(), ref.opac[:k])
        np.testing.assert_array_equal(gm.kf_id[:k].cpu().numpy(), ref.kf[:k])

    low = _batch(rng, 50)
    low = low[:3] + (low[3] * 0.2,)                    # all opacities < 0.3
    ref.append(*low, kf_idx=1, thr=0.3)
    gm.append(*(torch.from_numpy(x).cuda() for x in low), kf_idx=1, opacity_threshold=0.3)
    check()
    rec = torch.from_numpy(rng.uniform(0.5, 1, (40, 13)).astype(np.float32)).cuda()
    gm.append_records(rec, torch.zeros(1, dtype=torch.int64, device="cuda"), kf_idx=2,
                      opacity_threshold=0.3)          # device count 0
    check()
    c = _batch(rng, 70)
    ref.append(*c, kf_idx=3, thr=0.3)
    gm.append(*(torch.from_numpy(x).cuda() for x in c), kf_idx=3, opacity_threshold=0.3)
    check()
    assert ref.n < cap


def test_viz_camera_matches_reference_capture():
    """Camera math of _render_gs_interactive (CPU): settings vs the capture."""
    from splatt3r_amd.gaussian_map import gl_to_cv_T_WC, viz_camera
    g = np.load(os.path.join(GOLDEN, "viz_render.npz"))
    vw, vh = (int(v) for v in g["viewport"])
    s = float(g["res_scale"])
    rw, rh = max(64, int(vw * s)), max(64, int(vh * s))
    assert (rh, rw) == (int(g["settings_image_height"]), int(g["settings_image_width"]))
    tx, ty, view_t, proj, campos, sc, sc2 = viz_camera(gl_to_cv_T_WC(g["T_CW_gl"]), rw, rh,
                                                      float(g["hfov"]) / 2.0)
    assert abs(tx - float(g["settings_tanfovx"])) <= 1e-7
    assert abs(ty - float(g["settings_tanfovy"])) <= 1e-7
    np.testing.assert_allclose(view_t.numpy(), g["settings_viewmatrix"], atol=1e-6)
    np.testing.assert_allclose(proj.numpy(), g["settings_projmatrix"], atol=1e-5)
    np.testing.assert_allclose(campos.numpy(), g["settings_campos"], atol=1e-6)
    np.testing.assert_array_equal(g["means"] * np.float32(sc), g["in_means3D"])


@pytest.mark.gpu
def test_hip_full_map_render_matches_reference_viz(parity):
    """Bit-exact with the captured camera; with this host's own camera math
    (torch CPU ops: tanfovy / matrices can differ in the last bit from the
    capturing host) within 1e-6 mean-L1."""
    from splatt3r_amd.gaussian_map import SharedGaussians, gl_to_cv_T_WC, render_map
    g = np.load(os.path.join(GOLDEN, "viz_render.npz"))
    n = g["means"].shape[0]
    gm = SharedGaussians(max_gaussians=1 << 16, device="cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    gm.append(t(g["means"]), t(g["cov6"]), t(g["colors"]), t(g["opacities"]), kf_idx=0,
              opacity_threshold=0.0)
    assert gm.n_gaussians == n
    vw, vh = (int(v) for v in g["viewport"])
    s = float(g["res_scale"])
    rw, rh = max(64, int(vw * s)), max(64, int(vh * s))
    T = gl_to_cv_T_WC(g["T_CW_gl"])
    cam = (float(g["settings_tanfovx"]), float(g["settings_tanfovy"]),
           torch.from_numpy(g["settings_viewmatrix"]), torch.from_numpy(g["settings_projmatrix"]),
           torch.from_numpy(g["settings_campos"]), 20.0, 400.0)
    ours = render_map(gm, T, rw, rh, float(g["hfov"]) / 2.0, camera=cam).permute(1, 2, 0)
    ours = ours.cpu().numpy()
    d = np.abs(ours.astype(np.float64) - g["image_hwc"])
    parity("viz_full_map_render_captured_camera", max_abs=d.max(), mean_l1=d.mean(), tol=0.0)
    np.testing.assert_array_equal(ours, g["image_hwc"])
    own = render_map(gm, T, rw, rh, float(g["hfov"]) / 2.0).permute(1, 2, 0).cpu().numpy()
    d = np.abs(own.astype(np.float64) - g["image_hwc"])
    parity("viz_full_map_render_own_camera", max_abs=d.max(), mean_l1=d.mean(), tol=1e-6)
    assert d.mean() <= 1e-6


@pytest.mark.gpu
def test_hip_c5_map_8m_append_evict_and_render_bitexact(parity):
    """C5 at its own size: the 8,388,608-Gaussian map of bench.py bench_map
    built through s3w_map_append in 1M keyframe batches (== the numpy
    restatement MapRef, bit-exact), rendered full-map at 960x540 with the
    viz camera == oracle.raster on the same scaled inputs (bit-exact), then
    one more keyframe batch: FIFO half-eviction at capacity (== MapRef)."""
    from splatt3r_amd.gaussian_map import SharedGaussians, VIZ_BG, render_map, viz_camera
    from splatt3r_amd.synthetic import c5_map_batches
    import oracle
    n = 8_388_608
    gm = SharedGaussians(max_gaussians=n, device="cuda")
    ref = MapRef(n)
    batches = list(c5_map_batches(n + (1 << 20), seed=0, device="cuda"))
    h = lambda t: t.cpu().numpy()

    def check(tag):
        k = ref.n
        assert gm.n_gaussians == k, tag
        for name, a, b in (("means", gm.means, ref.means), ("cov", gm.cov_triu, ref.cov),
                           ("colors", gm.colors, ref.colors), ("opac", gm.opacities, ref.opac),
                           ("kf", gm.kf_id, ref.kf)):
            np.testing.assert_array_equal(h(a[:k]), b[:k], err_msg=f"{tag} {name}")

    for k, b in enumerate(batches[:-1]):
        gm.append(*b, kf_idx=k, opacity_threshold=0.3)
        ref.append(*(h(x) for x in b), kf_idx=k, thr=0.3)
    check("filled")
    T = np.eye(4, dtype=np.float32)
    W_, H_ = 960, 540
    cam = viz_camera(T, W_, H_, 45.0)
    img = render_map(gm, T, W_, H_, 45.0, camera=cam, clamp=False).cpu().numpy()
    tx, ty, view_t, proj, campos, s, s2 = cam
    sd = dict(image_height=H_, image_width=W_, tanfovx=tx, tanfovy=ty,
              bg=np.asarray(VIZ_BG, np.float32), scale_modifier=1.0,
              viewmatrix=view_t.numpy().ravel(), projmatrix=proj.numpy().ravel(), sh_degree=0,
              campos=campos.numpy().ravel())
    out = oracle.raster(sd, ref.means[:n] * np.float32(s), ref.opac[:n].reshape(-1, 1),
                        colors_precomp=ref.colors[:n], cov3D_precomp=ref.cov[:n] * np.float32(s2),
                        nthreads=16)
    import diff_gaussian_rasterization as dgr
    parity("c5_full_map_render_8m", mismatched_px=float((img != out["color"]).sum()),
           instances=dgr.last_num_rendered, oracle_instances=out["num_rendered"], tol=0.0)
    np.testing.assert_array_equal(img, out["color"])
    # one more keyframe at capacity: newest half to the front, then append
    gm.append(*batches[-1], kf_idx=len(batches) - 1, opacity_threshold=0.3)
    ref.append(*(h(x) for x in batches[-1]), kf_idx=len(batches) - 1, thr=0.3)
    assert ref.n == n // 2 + (1 << 20)
    check("evicted")
