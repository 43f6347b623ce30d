"""Tile rasterizer (include/gsr.h, drop-in diff_gaussian_rasterization).

Oracle: oracle/raster_ref.c (canonical graphdeco algorithm; parity vs the
reference's CUDA binary is unpinned: the submodule is absent).  The
boundary inputs are pinned by tests/golden/render_boundary.npz, captured
from the reference glue with a stub rasterizer (oracle/gen_golden.py).
Forward bar: bit-exact vs the oracle (same operation order, fixed exp);
backward: float atomics reorder sums -> max error <= BWD_TOL x max |ref|.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN

BWD_TOL = 2e-5   # measured worst 4.4e-6 (1M splats, C3 resolution)
from splatt3r_amd.synthetic import (identity_camera_settings, raster_grad,
                                    raster_microbench_scene, settings_to_dict)


def small_scene(P, seed, H=48, W=64, fx=60.0):
    K = np.array([[fx, 0, W / 2], [0, fx, H / 2], [0, 0, 1]], np.float32)
    return raster_microbench_scene(P, H=H, W=W, K=K, seed=seed)


def cpu_settings(sc):
    rs, scale = identity_camera_settings(sc["K"], sc["H"], sc["W"], "cpu")
    return settings_to_dict(rs), scale


# ------------------------------------------------------------- CPU: oracle
def test_oracle_single_gaussian_centre_value():
    sc = small_scene(1, 0)
    sd, scale = cpu_settings(sc)
    H, W = sc["H"], sc["W"]
    # a splat exactly on pixel (20, 30): invert the projection
    z = 3.0
    x = (30 - (W / 2 - 0.5)) / 60.0 * z
    y = (20 - (H / 2 - 0.5)) / 60.0 * z
    means = np.array([[x, y, z]], np.float32) * scale
    cov = np.array([[4e-4, 0, 0, 4e-4, 0, 4e-4]], np.float32) * scale * scale
    out = oracle.raster(sd, means, [[0.7]], colors_precomp=[[1.0, 0.5, 0.25]], cov3D_precomp=cov)
    c = out["color"][:, 20, 30]
    assert out["radii"][0] > 0
    # power ~ 0 at the centre -> alpha = 0.7, T = 1, bg = 0
    np.testing.assert_allclose(c, np.array([1.0, 0.5, 0.25]) * 0.7, rtol=1e-3)


def test_oracle_front_splat_occludes_back():
    sc = small_scene(1, 0)
    sd, scale = cpu_settings(sc)
    means = np.array([[0, 0, 2.0], [0, 0, 4.0]], np.float32) * scale
    cov = np.array([[1e-2, 0, 0, 1e-2, 0, 1e-2]] * 2, np.float32) * scale * scale
    out = oracle.raster(sd, means, [[0.99], [0.99]], colors_precomp=[[1, 0, 0], [0, 1, 0]],
                        cov3D_precomp=cov)
    c = out["color"][:, 23, 31]
    # the splat centre sits half a pixel off (31.5, 23.5): alpha just under 0.99
    assert c[0] > 0.9 and c[1] < 0.05 and c[0] > 20 * c[1]


def test_oracle_culls_behind_near_plane():
    sc = small_scene(1, 0)
    sd, scale = cpu_settings(sc)
    means = np.array([[0, 0, 0.01]], np.float32) * scale  # view z = 0.1 <= 0.2
    out = oracle.raster(sd, means, [[0.9]], colors_precomp=[[1, 1, 1]],
                        cov3D_precomp=np.array([[1e-2, 0, 0, 1e-2, 0, 1e-2]], np.float32))
    assert out["radii"][0] == 0 and out["num_rendered"] == 0
    assert np.all(out["color"] == 0)


def test_oracle_backward_colour_grad_is_exact_and_opacity_grad_matches_fd():
    sc = small_scene(40, 3)
    sd, scale = cpu_settings(sc)
    m = sc["means"] * scale
    cov = sc["cov6"] * scale * scale
    op = sc["opacities"]
    col = np.clip(sc["shs"][:, 0, :] + 0.5, 0, 1).astype(np.float32)
    g = raster_grad(sc["H"], sc["W"], seed=4)
    out = oracle.raster(sd, m, op, colors_precomp=col, cov3D_precomp=cov, dL_dout=g)
    L = lambda o: float((o["color"] * g).sum())
    # colours enter linearly: finite difference is exact up to rounding
    k = int(np.argmax(out["radii"]))
    for ch in range(3):
        c2 = col.copy(); c2[k, ch] += 1e-2
        fd = (L(oracle.raster(sd, m, op, colors_precomp=c2, cov3D_precomp=cov)) - L(out)) / 1e-2
        np.testing.assert_allclose(out["dL_dcolors"][k, ch], fd, rtol=2e-3, atol=2e-3)
    o2 = op.copy(); o2[k] += 1e-3
    o3 = op.copy(); o3[k] -= 1e-3
    fd = (L(oracle.raster(sd, m, o2, colors_precomp=col, cov3D_precomp=cov)) -
          L(oracle.raster(sd, m, o3, colors_precomp=col, cov3D_precomp=cov))) / 2e-3
    np.testing.assert_allclose(out["dL_dopacity"][k], fd, rtol=5e-2, atol=5e-3)


def test_oracle_fexp_ulp_bound():
    """The blend's fixed-sequence exponential (raster_math.hpp fexp, restated
    in the oracle) against the correctly rounded exp (float64 exp rounded to
    float32) over the blend's domain [-87, 0]: at most 3 ulp (VERDICT r04:
    max 3 ulp, ~13 % of values differ; the old header claimed 2)."""
    f = oracle.lib().oracle_fexp
    import ctypes
    f.restype, f.argtypes = ctypes.c_float, [ctypes.c_float]
    rng = np.random.default_rng(5)
    xs = np.concatenate([np.linspace(-87.0, 0.0, 150_001, dtype=np.float32),
                         -rng.exponential(3.0, 50_000).astype(np.float32).clip(0, 87)])
    got = np.array([f(float(x)) for x in xs], np.float32)
    ref = np.exp(xs.astype(np.float64)).astype(np.float32)
    ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 3, ulp.max()
    assert 0.0 < (ulp > 0).mean() < 0.25


def test_tile_mask_rows_keeps_every_hit(tmp_path):
    """The preprocess's row-run tile mask (raster_math.hpp tile_mask_rows)
    holds every tile the per-tile edge-minimum test (tile_hit) keeps, over
    400k random ellipses / opacities / rects of 2..64 tiles, and keeps at
    most 1 % more (the culling is conservative either way; images do not
    depend on it, only num_rendered does).  Host code built by hipcc."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(here, "..", "splatt3r-slam_amd", "csrc")
    exe = str(tmp_path / "tile_mask_check")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", csrc, os.path.join(here, "native", "tile_mask_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=600)
    out = subprocess.run([exe, "400000"], check=True, capture_output=True, text=True, timeout=300)
    n, hits, kept, miss = map(int, out.stdout.split())
    assert n == 400000 and hits > 0
    assert miss == 0, out.stdout
    assert kept <= hits * 1.01, out.stdout


def test_oracle_libm_exp_option_changes_only_low_bits():
    """oracle.raster(exp='libm') runs glibc expf in the blend: the image moves
    by rounding only (the exponential differs by <= 3 ulp)."""
    sc = small_scene(1500, 9)
    sd, scale = cpu_settings(sc)
    kw = dict(shs=sc["shs"], cov3D_precomp=sc["cov6"] * scale * scale)
    a = oracle.raster(sd, sc["means"] * scale, sc["opacities"], **kw)
    b = oracle.raster(sd, sc["means"] * scale, sc["opacities"], exp="libm", **kw)
    np.testing.assert_array_equal(a["radii"], b["radii"])
    d = np.abs(a["color"] - b["color"])
    assert d.max() < 1e-5 and d.mean() < 1e-7
    with pytest.raises(ValueError):
        oracle.raster(sd, sc["means"] * scale, sc["opacities"], exp="fast", **kw)


def test_render_glue_settings_match_reference_boundary():
    from splatt3r_amd.render import camera_settings, normalize_intrinsics
    g = np.load(os.path.join(GOLDEN, "render_boundary.npz"))
    h, w = int(g["settings_image_height"]), int(g["settings_image_width"])
    ctx = torch.from_numpy(g["head_ctx_pose"])
    tgt = torch.from_numpy(g["head_tgt_pose"])
    K = torch.from_numpy(g["head_K"])
    ext = torch.inverse(ctx) @ tgt
    intr = normalize_intrinsics(K, (h, w))
    st, scale = camera_settings(ext, intr, torch.full((1,), 0.1), torch.full((1,), 1000.0),
                                (h, w), torch.zeros(1, 3), 0)
    rs = st[0]
    np.testing.assert_allclose(rs.tanfovx, g["settings_tanfovx"], rtol=1e-6)
    np.testing.assert_allclose(rs.tanfovy, g["settings_tanfovy"], rtol=1e-6)
    np.testing.assert_allclose(rs.viewmatrix.numpy(), g["settings_viewmatrix"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rs.projmatrix.numpy(), g["settings_projmatrix"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rs.campos.numpy(), g["settings_campos"], rtol=1e-6, atol=1e-6)


# -------------------------------------------------------------- GPU: HIP
def _to(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def _gpu_render(sc, mode="shs", grad=None, P=None):
    from diff_gaussian_rasterization import GaussianRasterizer
    rs, scale = identity_camera_settings(sc["K"], sc["H"], sc["W"], "cuda")
    m = _to(sc["means"] * scale).requires_grad_(grad is not None)
    cov = _to(sc["cov6"] * scale * scale).requires_grad_(grad is not None)
    op = _to(sc["opacities"]).requires_grad_(grad is not None)
    m2 = torch.zeros_like(m, requires_grad=True)
    kw = dict(means3D=m, means2D=m2, opacities=op, cov3D_precomp=cov)
    if mode == "shs":
        shs = _to(sc["shs"]).requires_grad_(grad is not None)
        kw["shs"] = shs
    else:
        col = _to(np.clip(sc["shs"][:, 0, :] + 0.5, 0, 1)).requires_grad_(grad is not None)
        kw["colors_precomp"] = col
    img, radii = GaussianRasterizer(rs)(**kw)
    if grad is not None:
        (img * _to(grad)).sum().backward()
    return rs, scale, img, radii, kw


@pytest.mark.gpu
@pytest.mark.parametrize("P,seed,mode", [(2000, 0, "shs"), (5000, 1, "colors"), (1, 2, "shs")])
def test_hip_forward_bitexact_vs_oracle(P, seed, mode):
    sc = small_scene(P, seed)
    rs, scale, img, radii, kw = _gpu_render(sc, mode)
    sd = settings_to_dict(rs)
    ref = oracle.raster(sd, sc["means"] * scale, sc["opacities"],
                        shs=sc["shs"] if mode == "shs" else None,
                        colors_precomp=None if mode == "shs" else np.clip(sc["shs"][:, 0, :] + 0.5, 0, 1),
                        cov3D_precomp=sc["cov6"] * scale * scale)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref["radii"])
    np.testing.assert_array_equal(img.detach().cpu().numpy(), ref["color"])


@pytest.mark.gpu
@pytest.mark.parametrize("P,seed,mode", [(2000, 0, "shs"), (5000, 1, "colors")])
def test_hip_forward_vs_libm_exp_oracle(P, seed, mode):
    """The HIP image against the oracle with the canonical graphdeco
    exponential (libm expf), not the kernel's own fixed-sequence exp: equal
    radii, image within 1e-6 mean / 1e-4 max absolute."""
    sc = small_scene(P, seed)
    rs, scale, img, radii, kw = _gpu_render(sc, mode)
    ref = oracle.raster(settings_to_dict(rs), sc["means"] * scale, sc["opacities"],
                        shs=sc["shs"] if mode == "shs" else None,
                        colors_precomp=None if mode == "shs" else np.clip(sc["shs"][:, 0, :] + 0.5, 0, 1),
                        cov3D_precomp=sc["cov6"] * scale * scale, exp="libm")
    np.testing.assert_array_equal(radii.cpu().numpy(), ref["radii"])
    d = np.abs(img.detach().cpu().numpy() - ref["color"])
    assert d.mean() <= 1e-6 and d.max() <= 1e-4, (d.mean(), d.max())


def _restage(sc, z):
    """Move every Gaussian to depth z along its own ray (same pixel)."""
    sc = dict(sc)
    m = sc["means"].copy()
    r = (z / m[:, 2]).astype(np.float32)
    sc["means"] = (m * r[:, None]).astype(np.float32)
    sc["cov6"] = (sc["cov6"] * (r * r)[:, None]).astype(np.float32)
    return sc


@pytest.mark.gpu
@pytest.mark.parametrize("binning", ["tile", "global"])
@pytest.mark.parametrize("case", ["plane", "two_depths", "wide_range", "all_culled", "tail_4097",
                                  "tail_8193", "tiles_3600", "tiles_8160", "tiles_8832",
                                  "big_splats", "ragged_1x1", "one_tile_20k", "one_tile_20k_plane"])
def test_hip_binning_edge_cases_bitexact_vs_oracle(case, binning):
    """Both forward binnings (the global depth + tile sorts of raster.hip
    "sorting", the default, and "per-tile binning"): equal depths (ties resolved
    by Gaussian index: the per-tile sort's index passes), a 1-2 pass key
    width, a 4-pass key width, nothing visible (R = 0), segment tails (4096
    and 8192 items), tile ids of 12, 13 and 14 bits (8,832 tiles: past the
    per-tile path's 8,192, so the global path runs), splats whose rect
    exceeds the 64-tile mask (plain rect enumeration), a ragged 1-tile image,
    and ~20k instances in one tile (past the 16,384 sorted in LDS: the
    chunked passes), with distinct and with equal depths -- bit-exact against
    the oracle."""
    from splatt3r_amd import _lib
    rng = np.random.default_rng(7)
    P, H, W, fx = 3000, 48, 64, 60.0
    if case.startswith("one_tile_20k"):
        P, H, W, fx = 20000, 16, 16, 15.0
    if case == "tail_4097":
        P = 4097
    if case == "tail_8193":
        P = 8193
    if case == "tiles_3600":
        H, W, fx = 720, 1280, 900.0
    if case == "tiles_8160":
        H, W, fx = 1088, 1920, 1300.0
    if case == "tiles_8832":
        H, W, fx = 1104, 2048, 1400.0
    if case == "big_splats":
        P, H, W, fx = 2000, 540, 960, 700.0
    if case == "ragged_1x1":
        H, W, fx = 13, 9, 12.0
    sc = small_scene(P, 11, H=H, W=W, fx=fx)
    if case == "big_splats":
        # sigma x 12: rects of ~10 x 10 tiles and more (> 64: no tile mask)
        sc = dict(sc)
        sc["cov6"] = (sc["cov6"] * 144.0).astype(np.float32)
    if case == "plane":
        sc = _restage(sc, np.full(P, 3.0, np.float32))
    elif case == "two_depths":
        sc = _restage(sc, np.where(rng.random(P) < 0.5, 3.0, 3.0001).astype(np.float32))
    elif case == "wide_range":
        sc = _restage(sc, np.exp(rng.uniform(np.log(0.3), np.log(500.0), P)).astype(np.float32))
    elif case == "all_culled":
        # in front of the 0.2 near-plane cull even after the settings'
        # scale-invariant rescale of the means
        sc = _restage(sc, np.full(P, 1e-5, np.float32))
    elif case == "one_tile_20k_plane":
        sc = _restage(sc, np.full(P, 3.0, np.float32))
    _lib.lib().gsr_set_binning(1 if binning == "tile" else 0)
    try:
        rs, scale, img, radii, kw = _gpu_render(sc, "colors")
    finally:
        _lib.lib().gsr_set_binning(-1)
    sd = settings_to_dict(rs)
    ref = oracle.raster(sd, sc["means"] * scale, sc["opacities"],
                        colors_precomp=np.clip(sc["shs"][:, 0, :] + 0.5, 0, 1),
                        cov3D_precomp=sc["cov6"] * scale * scale)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref["radii"])
    np.testing.assert_array_equal(img.detach().cpu().numpy(), ref["color"])
    if case == "all_culled":
        assert int(radii.max()) == 0
    if case.startswith("one_tile_20k"):
        import diff_gaussian_rasterization as dgr
        assert dgr.last_num_rendered > 16384


@pytest.mark.gpu
def test_hip_forward_c3_resolution_vs_oracle():
    sc = raster_microbench_scene(200_000, seed=0)
    rs, scale, img, radii, _ = _gpu_render(sc, "shs")
    ref = oracle.raster(settings_to_dict(rs), sc["means"] * scale, sc["opacities"], shs=sc["shs"],
                        cov3D_precomp=sc["cov6"] * scale * scale, nthreads=16)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref["radii"])
    np.testing.assert_array_equal(img.detach().cpu().numpy(), ref["color"])
    # tile culling (raster_math.hpp tile_cull/tile_hit) drops only (Gaussian,
    # tile) pairs the blend skips at every pixel: same image, fewer instances
    import diff_gaussian_rasterization as dgr
    assert 0 < dgr.last_num_rendered < ref["num_rendered"]


@pytest.mark.gpu
def test_hip_forward_c3_full_size_bitexact_vs_oracle(parity):
    """The exact C3 microbench case bench.py times (4,194,304 splats @
    960x540, seed 0): radii and image bit-exact vs the canonical oracle."""
    from splatt3r_amd.synthetic import C3_P
    sc = raster_microbench_scene(C3_P, seed=0)
    rs, scale, img, radii, _ = _gpu_render(sc, "shs")
    ref = oracle.raster(settings_to_dict(rs), sc["means"] * scale, sc["opacities"], shs=sc["shs"],
                        cov3D_precomp=sc["cov6"] * scale * scale, nthreads=16)
    import diff_gaussian_rasterization as dgr
    parity("c3_full_forward", mismatched_px=float((img.detach().cpu().numpy() != ref["color"]).sum()),
           mismatched_radii=float((radii.cpu().numpy() != ref["radii"]).sum()),
           instances=dgr.last_num_rendered, oracle_instances=ref["num_rendered"], tol=0.0)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref["radii"])
    np.testing.assert_array_equal(img.detach().cpu().numpy(), ref["color"])
    assert 0 < dgr.last_num_rendered < ref["num_rendered"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["1M", "c3_full"])
def test_hip_backward_1m_splats_c3_resolution_vs_oracle(parity, case):
    """Backward at C3 resolution (960x540): 2^20 splats, and the full C3
    microbench case (4,194,304 splats, scene seed 0, dL/dimage seed 1 as
    SURVEY §8(d) C3 and bench.py's raster_c3 leg)."""
    from splatt3r_amd.synthetic import C3_P
    if case == "1M":
        sc = raster_microbench_scene(1 << 20, seed=2)
        g = raster_grad(sc["H"], sc["W"], seed=3)
    else:
        sc = raster_microbench_scene(C3_P, seed=0)
        g = raster_grad(sc["H"], sc["W"], seed=1)
    rs, scale, img, radii, kw = _gpu_render(sc, "shs", grad=g)
    ref = oracle.raster(settings_to_dict(rs), sc["means"] * scale, sc["opacities"], shs=sc["shs"],
                        cov3D_precomp=sc["cov6"] * scale * scale, dL_dout=g, nthreads=16)
    np.testing.assert_array_equal(img.detach().cpu().numpy(), ref["color"])
    for name, a, b in (("means2D", kw["means2D"].grad[:, :2], ref["dL_dmeans2D"][:, :2]),
                       ("opacity", kw["opacities"].grad, ref["dL_dopacity"].reshape(-1, 1)),
                       ("sh", kw["shs"].grad, ref["dL_dsh"]),
                       ("cov3D", kw["cov3D_precomp"].grad, ref["dL_dcov3D"]),
                       ("means3D", kw["means3D"].grad, ref["dL_dmeans3D"])):
        a = a.detach().cpu().numpy().reshape(b.shape).astype(np.float64)
        d = np.abs(a - b)
        sc_ = np.abs(b).max() + 1e-12
        parity(f"c3_bwd_{case}_{name}", max_rel=d.max() / sc_, p999_rel=np.percentile(d, 99.9) / sc_,
               tol=BWD_TOL)
        assert d.max() <= BWD_TOL * sc_ + 1e-6, (name, d.max() / sc_)


@pytest.mark.gpu
def test_hip_backward_vs_oracle():
    sc = small_scene(3000, 5)
    g = raster_grad(sc["H"], sc["W"], seed=6)
    rs, scale, img, radii, kw = _gpu_render(sc, "shs", grad=g)
    ref = oracle.raster(settings_to_dict(rs), sc["means"] * scale, sc["opacities"], shs=sc["shs"],
                        cov3D_precomp=sc["cov6"] * scale * scale, dL_dout=g)

    def close(a, b, name):
        a = a.detach().cpu().numpy().reshape(b.shape)
        tol = 1e-4 * (np.abs(b).max() + 1e-12)
        err = np.abs(a - b).max()
        assert err <= tol + 1e-6, f"{name}: max err {err} > {tol}"

    close(kw["means2D"].grad[:, :2], ref["dL_dmeans2D"][:, :2], "means2D")
    close(kw["opacities"].grad, ref["dL_dopacity"].reshape(-1, 1), "opacity")
    close(kw["shs"].grad, ref["dL_dsh"], "sh")
    close(kw["cov3D_precomp"].grad, ref["dL_dcov3D"], "cov3D")
    close(kw["means3D"].grad, ref["dL_dmeans3D"], "means3D")


@pytest.mark.gpu
def test_hip_api_contract():
    from diff_gaussian_rasterization import GaussianRasterizer
    sc = small_scene(10, 0)
    rs, scale = identity_camera_settings(sc["K"], sc["H"], sc["W"], "cuda")
    m = _to(sc["means"])
    with pytest.raises(Exception, match="excatly one of either SHs"):
        GaussianRasterizer(rs)(means3D=m, means2D=m, opacities=_to(sc["opacities"]),
                               cov3D_precomp=_to(sc["cov6"]))
    with pytest.raises(Exception, match="scale/rotation pair"):
        GaussianRasterizer(rs)(means3D=m, means2D=m, opacities=_to(sc["opacities"]),
                               shs=_to(sc["shs"]))
    # empty input: image of zeros, empty radii (reference: P == 0 -> no render)
    img, radii = GaussianRasterizer(rs)(means3D=m[:0], means2D=m[:0], opacities=_to(sc["opacities"])[:0],
                                        shs=_to(sc["shs"])[:0], cov3D_precomp=_to(sc["cov6"])[:0])
    assert img.shape == (3, sc["H"], sc["W"]) and radii.shape == (0,)
    assert float(img.abs().sum()) == 0.0
    vis = GaussianRasterizer(rs).markVisible(_to(sc["means"] * scale))
    assert vis.dtype == torch.bool and bool(vis.all())
    # inference_mode + requires_grad means2D (cuda_splatting.py:94)
    with torch.inference_mode():
        img, radii = GaussianRasterizer(rs)(means3D=_to(sc["means"] * scale), means2D=m,
                                            opacities=_to(sc["opacities"]), shs=_to(sc["shs"]),
                                            cov3D_precomp=_to(sc["cov6"] * scale * scale))
    assert img.shape == (3, sc["H"], sc["W"])


@pytest.mark.gpu
def test_hip_scale_rotation_path_matches_precomputed_cov():
    from diff_gaussian_rasterization import GaussianRasterizer
    rng = np.random.default_rng(0)
    sc = small_scene(500, 7)
    rs, scale = identity_camera_settings(sc["K"], sc["H"], sc["W"], "cuda")
    s3 = np.exp(rng.uniform(np.log(0.005), np.log(0.03), (500, 3))).astype(np.float32) * scale
    q = rng.normal(size=(500, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)  # (r, x, y, z) order on this path
    R = oracle_rot_wxyz(q)
    cov = np.einsum("nik,nk,njk->nij", R, s3 * s3, R)
    iu = np.triu_indices(3)
    m = _to(sc["means"] * scale)
    base = dict(means3D=m, means2D=torch.zeros_like(m), opacities=_to(sc["opacities"]),
                shs=_to(sc["shs"]))
    a, _ = GaussianRasterizer(rs)(**base, scales=_to(s3), rotations=_to(q))
    b, _ = GaussianRasterizer(rs)(**base, cov3D_precomp=_to(cov[:, iu[0], iu[1]].astype(np.float32)))
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=2e-4)


def oracle_rot_wxyz(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)],
                    -1).reshape(-1, 3, 3)


@pytest.mark.gpu
def test_hip_render_glue_boundary_vs_reference_capture():
    """Our fused packing + settings reproduce what the reference glue hands
    the rasterizer (render_boundary.npz), then the HIP render matches the
    oracle on exactly the captured inputs."""
    from splatt3r_amd.render import pack_splats
    g = np.load(os.path.join(GOLDEN, "render_boundary.npz"))
    hw = g["head_m1"].shape[1] * g["head_m1"].shape[2]
    views = []
    for v in ("1", "2"):
        views.append(dict(means=_to(g["head_m" + v].reshape(hw, 3)),
                          scales=_to(g["head_s" + v].reshape(hw, 3)),
                          rotations=_to(g["head_r" + v].reshape(hw, 4)),
                          sh=_to(g["head_sh" + v].reshape(hw, 3, 1)),
                          opacities=_to(g["head_o" + v].reshape(hw, 1)),
                          img=_to(g["head_img" + v].reshape(3, hw))))
    scale = float(1.0 / torch.tensor(0.1, dtype=torch.float32))
    from splatt3r_amd import _lib
    means, cov6, shs, opac = [], [], [], []
    P = 2 * hw
    means = torch.empty(P, 3, device="cuda"); cov6 = torch.empty(P, 6, device="cuda")
    shs = torch.empty(P, 1, 3, device="cuda"); opac = torch.empty(P, 1, device="cuda")
    for i, v in enumerate(views):
        o = i * hw
        _lib.call("s3r_pack_splats", v["means"].data_ptr(), v["scales"].data_ptr(),
                  v["rotations"].data_ptr(), v["sh"].data_ptr(), v["opacities"].data_ptr(),
                  v["img"].data_ptr(), hw, 1, scale, 1, means[o:].data_ptr(), cov6[o:].data_ptr(),
                  shs[o:].data_ptr(), opac[o:].data_ptr(), _lib.stream())
    np.testing.assert_allclose(means.cpu().numpy(), g["in_means3D"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(cov6.cpu().numpy(), g["in_cov3D_precomp"], rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(shs.cpu().numpy(), g["in_shs"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(opac.cpu().numpy(), g["in_opacities"])
    del pack_splats


def _mat_to_sim3(M):
    """[sR | t] 4x4 -> lietorch Sim3 data (t, q xyzw, s)."""
    M = np.asarray(M, np.float64).reshape(4, 4)
    s = np.cbrt(np.linalg.det(M[:3, :3]))
    R = M[:3, :3] / s
    w = np.sqrt(max(1e-12, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    q = np.array([(R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w),
                  (R[1, 0] - R[0, 1]) / (4 * w), w])
    return np.concatenate([M[:3, 3], q / np.linalg.norm(q), [s]]).astype(np.float32)


@pytest.mark.gpu
def test_hip_camera_settings_from_sim3_vs_reference_capture():
    """camera_settings_sim3 (cached intrinsics + one fp64 s3r_camera thread)
    reproduces the settings the reference decoder glue built for the
    captured poses/intrinsics (render_boundary.npz)."""
    from splatt3r_amd.render import camera_settings_sim3
    g = np.load(os.path.join(GOLDEN, "render_boundary.npz"))
    Tc = torch.from_numpy(_mat_to_sim3(g["head_ctx_pose"])).cuda()
    Tt = torch.from_numpy(_mat_to_sim3(g["head_tgt_pose"])).cuda()
    K = torch.from_numpy(g["head_K"].reshape(3, 3))
    h, w = int(g["settings_image_height"]), int(g["settings_image_width"])
    (st,), scale = camera_settings_sim3(Tc, Tt, K, (h, w), torch.zeros(3, device="cuda"))
    assert abs(st.tanfovx - float(g["settings_tanfovx"])) < 1e-6
    assert abs(st.tanfovy - float(g["settings_tanfovy"])) < 1e-6
    np.testing.assert_allclose(st.viewmatrix.cpu().numpy(), g["settings_viewmatrix"], atol=2e-6)
    np.testing.assert_allclose(st.projmatrix.cpu().numpy(), g["settings_projmatrix"], atol=1e-5)
    np.testing.assert_allclose(st.campos.cpu().numpy(), g["settings_campos"], atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("P,seed,mode,hw", [(2000, 0, "shs", (48, 64)), (5000, 1, "colors", (48, 64)),
                                            (1, 2, "shs", (48, 64)), (60000, 3, "shs", (384, 512))])
def test_hip_deferred_forward_equals_two_call_forward(P, seed, mode, hw):
    """gsr_forward_deferred (no host read; instance count and depth-key range
    on the device) == gsr_preprocess + gsr_render bit for bit when the frame
    fits; too small a capacity or key width raises the status bits (memory
    safe, image not used) and reports the sizes for the next call."""
    import diff_gaussian_rasterization as dgr
    H, W = hw
    sc = small_scene(P, seed, H=H, W=W, fx=60.0 * W / 64)
    rs, scale, img, radii, kw = _gpu_render(sc, mode)
    R = dgr.last_num_rendered
    args = dict(means3D=kw["means3D"].detach(), opacities=kw["opacities"].detach(),
                cov3D_precomp=kw["cov3D_precomp"].detach())
    if mode == "shs":
        args["shs"] = kw["shs"].detach()
    else:
        args["colors_precomp"] = kw["colors_precomp"].detach()
    for cap, bits in ((R + 1000, 32), (max(R, 1), 32), (2 * R + 1, 24)):
        c, r, info = dgr.rasterize_deferred(rs, capacity=cap, key_bits=bits, **args)
        st, tot, live = info.tolist()
        assert tot == R and live <= 32
        if live <= bits:
            assert st == 0, (cap, bits, st)
            assert torch.equal(c, img.detach()) and torch.equal(r, radii)
    if R > 1:
        _, _, info = dgr.rasterize_deferred(rs, capacity=R // 2, key_bits=32, **args)
        assert info.tolist()[0] & 1
    _, _, info = dgr.rasterize_deferred(rs, capacity=R + 10, key_bits=1, **args)
    st, tot, live = info.tolist()
    assert (st & 2) == (2 if live > 1 else 0)
