"""Host-side Python of the path pinned to the reference's own code.

tests/golden/host_glue.npz is produced by oracle/gen_golden.py `host`, which
AST-extracts the reference functions (their modules need lietorch /
mast3r_slam_backends / cv2, absent here) and runs them on synthetic inputs:
gaussians_to_world (splatt3r_utils.py:180-328), the geometry helpers
(geometry.py:5-128), one tracker normal-equation step in ray and calibrated
mode (tracker.py:129-270, lietorch's Sim3 in matrix form), add_factors'
Q-weighting and edge acceptance (global_opt.py:30-99) and the
match_iterative_proj glue (matching.py:8-90, with the oracle kernels in
place of the uncompilable CUDA ones).

CPU tests pin the oracle restatements (oracle/tracker_ref.py,
oracle/gaussians_ref.py, oracle.match) and the product's host code
(FactorGraph.add_factors, geometry.constrain_points_to_ray) to those
outputs; GPU tests hold the HIP paths to them.  Tolerances: selections,
orders, indices and masks bit-exact; fp32 geometry 1e-5..1e-4 relative;
normal equations 1e-3 relative (fp32 per-point terms vs the float64 run).
"""
import os

import numpy as np
import pytest
import torch

import oracle
import oracle.gaussians_ref as GR
import oracle.tracker_ref as TR
from conftest import GOLDEN


def _g():
    return np.load(os.path.join(GOLDEN, "host_glue.npz"))


def _g2w_case(g, c):
    pre = f"g2w{c}_"
    H, W, stride, cross, q, maxs, minc = g[pre + "args"]
    p1 = {k[len(pre) + 3:]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre + "p1_")}
    p2 = {k[len(pre) + 3:]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre + "p2_")}
    want = tuple(g[pre + "out_" + k] for k in ("means", "cov", "colors", "opacities"))
    return (p1, p2, torch.from_numpy(g[pre + "img"]), g[pre + "T"], int(stride), bool(cross),
            float(q), float(maxs), float(minc), want)


def _check_g2w(got, want):
    assert got[0].shape[0] == want[0].shape[0]
    for a, b, tol in zip(got, want, (2e-5, 1e-4, 1e-5, 0)):
        np.testing.assert_allclose(np.asarray(a), b, rtol=tol, atol=tol * 1e-2)


@pytest.mark.parametrize("c", range(4))
def test_oracle_gaussians_to_world_vs_reference(c):
    p1, p2, img, T, stride, cross, q, maxs, minc, want = _g2w_case(_g(), c)
    M = torch.from_numpy(_sim3_matrix(T))
    # include_cross: both views, each filtered on its own quantile, concatenated
    got = GR.gaussians_to_world([p1, p2] if cross else [p1], img, M, stride, 0.05, q, maxs, minc)
    _check_g2w([x.numpy() for x in got], want)


def _sim3_matrix(T):
    T = np.asarray(T, np.float64)
    x, y, z, w = T[3:7] / np.linalg.norm(T[3:7])
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    M = np.eye(4)
    M[:3, :3] = R * T[7]
    M[:3, 3] = T[:3]
    return M.astype(np.float32)


def test_oracle_geometry_vs_reference():
    g = _g()
    X = g["geo_X"]
    rd, J = TR.point_to_ray_dist(X, jacobian=True)
    np.testing.assert_allclose(rd, g["geo_rd"], rtol=1e-12)
    np.testing.assert_allclose(J, g["geo_rd_J"], rtol=1e-10, atol=1e-14)
    p = TR.act_sim3(g["geo_T"].astype(np.float64), X)
    np.testing.assert_allclose(p, g["geo_act"], rtol=1e-6, atol=1e-7)
    dXdT = np.concatenate([np.broadcast_to(np.eye(3), (X.shape[0], 3, 3)), -TR.skew(p),
                           p[:, :, None]], -1)
    np.testing.assert_allclose(dXdT, g["geo_act_J"], rtol=1e-6, atol=1e-7)
    pz, D, valid = TR.project_calib(g["geo_P"], g["geo_K"], (240, 320), border=-10, z_eps=1e-6)
    np.testing.assert_array_equal(valid, g["geo_pz_valid"][:, 0])
    v = g["geo_pz_valid"][:, 0]
    np.testing.assert_allclose(pz[v], g["geo_pz"][v], rtol=1e-12)
    np.testing.assert_allclose(D, g["geo_pz_J"], rtol=1e-10, atol=1e-14)


def test_oracle_tracker_normal_equations_vs_reference():
    from splatt3r_amd.config import config
    c = config["tracking"]
    g = _g()
    H, gg, _ = TR.normal_equations(g["trk_ray_T"], g["trk_ray_Xf"], g["trk_ray_Xk"],
                                   g["trk_ray_Q"], g["trk_ray_valid"], c["sigma_ray"],
                                   c["sigma_dist"], c["huber"])
    np.testing.assert_allclose(H, g["trk_ray_H"], rtol=1e-6, atol=1e-9 * np.abs(H).max())
    np.testing.assert_allclose(gg, g["trk_ray_g"], rtol=1e-5, atol=1e-8 * np.abs(gg).max())
    h, w = (int(v) for v in g["trk_cal_hw"])
    H, gg, _ = TR.normal_equations_calib(g["trk_cal_T"], g["trk_cal_Xf_c"], g["trk_cal_Xk_c"],
                                         g["trk_cal_Q"], g["trk_cal_valid"], g["trk_cal_K"], (h, w),
                                         c["pixel_border"], c["depth_eps"], c["sigma_pixel"],
                                         c["sigma_depth"], c["huber"])
    np.testing.assert_allclose(H, g["trk_cal_H"], rtol=1e-6, atol=1e-9 * np.abs(H).max())
    np.testing.assert_allclose(gg, g["trk_cal_g"], rtol=1e-5, atol=1e-8 * np.abs(gg).max())
    meas, ok = TR.calib_measurements(g["trk_cal_Xk_c"], (h, w), c["depth_eps"])
    np.testing.assert_allclose(meas, g["trk_cal_meas"], rtol=1e-12)
    np.testing.assert_array_equal(ok, g["trk_cal_vmeas"][:, 0])


def test_constrain_points_to_ray_vs_reference():
    from splatt3r_amd.geometry import constrain_points_to_ray
    g = _g()
    h, w = (int(v) for v in g["trk_cal_hw"])
    K = torch.from_numpy(g["trk_cal_K"])
    Xk = constrain_points_to_ray((h, w), torch.from_numpy(g["trk_cal_Xk"])[None], K)[0]
    np.testing.assert_array_equal(Xk.numpy(), g["trk_cal_Xk_c"])
    Xf = constrain_points_to_ray((h, w), torch.from_numpy(g["trk_cal_Xf"])[None], K)[0]
    np.testing.assert_array_equal(Xf.numpy()[g["trk_cal_idx"]], g["trk_cal_Xf_c"])


def test_add_factors_vs_reference():
    """The product FactorGraph.add_factors (host torch; the pair decode is
    injected) == the reference's add_factors text on the same matches."""
    from splatt3r_amd.config import config
    from splatt3r_amd.global_opt import FactorGraph
    g = _g()
    m = tuple(torch.from_numpy(g["af_m_" + k]) for k in
              ("idx_i2j", "idx_j2i", "valid_j", "valid_i", "Qii", "Qjj", "Qji", "Qij"))

    class KF:
        feat = torch.zeros(1, 2, 4)
        pos = torch.zeros(1, 2, 2)
        img_true_shape = torch.tensor([[12, 16]])

    ii, jj = g["af_ii"].tolist(), g["af_jj"].tolist()
    for case, reloc in (("add", False), ("reloc", True)):
        fg = FactorGraph(None, [KF()] * 5, device="cpu", match_fn=lambda *a: m)
        ret = fg.add_factors(ii, jj, config["local_opt"]["min_match_frac"], is_reloc=reloc)
        assert bool(ret) == bool(g[f"af_{case}_ret"])
        for k in ("ii", "jj", "idx_ii2jj", "idx_jj2ii", "valid_match_j", "valid_match_i"):
            np.testing.assert_array_equal(getattr(fg, k).numpy(), g[f"af_{case}_{k}"], err_msg=k)
        # Q = sqrt(Qa * Qb) in host torch: exact on the generating machine,
        # within 1 ulp on another CPU's vector sqrt (measured on the GPU box)
        for k in ("Q_ii2jj", "Q_jj2ii"):
            np.testing.assert_array_max_ulp(getattr(fg, k).numpy(), g[f"af_{case}_{k}"], maxulp=1)


@pytest.mark.parametrize("c", [0, 1])
def test_oracle_match_vs_reference_glue(c):
    g = _g()
    pre = f"mt{c}_"
    init = g[pre + "idx_init"] if pre + "idx_init" in g.files else None
    idx, valid = oracle.match(g[pre + "X11"], g[pre + "X21"], g[pre + "D11"], g[pre + "D21"],
                              init)
    np.testing.assert_array_equal(idx, g[pre + "idx"])
    np.testing.assert_array_equal(valid.reshape(g[pre + "valid"].shape), g[pre + "valid"])


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("c", range(4))
def test_hip_gaussians_to_world_vs_reference(c):
    import lietorch
    from splatt3r_amd.frame import Frame
    from splatt3r_amd.splatt3r_utils import gaussians_to_world
    p1, p2, img, T, stride, cross, q, maxs, minc, want = _g2w_case(_g(), c)
    fr = Frame(0, img.cuda(), None, None,
               T_WC=lietorch.Sim3(torch.from_numpy(T).reshape(1, 8).cuda()))
    fr.gaussian_pred = {k: v.cuda() for k, v in p1.items()}
    fr.gaussian_pred_cross = {k: v.cuda() for k, v in p2.items()}
    got = gaussians_to_world(fr, include_cross=cross, spatial_stride=stride,
                             depth_max_percentile=q, max_scale=maxs, min_confidence=minc)
    _check_g2w([x.cpu().numpy() for x in got], want)


@pytest.mark.gpu
def test_hip_tracker_normal_equations_vs_reference(parity):
    from splatt3r_amd.config import config
    from splatt3r_amd.tracker import NormalEquations
    c = config["tracking"]
    g = _g()
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)
                                   if a.dtype != bool else np.ascontiguousarray(a)).cuda()
    ne = NormalEquations("cuda")
    H, gg, _ = ne(g["trk_ray_T"], d(g["trk_ray_Xf"]), d(g["trk_ray_Xk"]), d(g["trk_ray_Q"]),
                  d(g["trk_ray_valid"]), c["sigma_ray"], c["sigma_dist"], c["huber"])
    for key, a, b in (("ray_H", H, g["trk_ray_H"]), ("ray_g", gg, g["trk_ray_g"])):
        err = np.abs(a - b).max() / np.abs(b).max()
        parity("tracker_ne_" + key, max_rel=err, tol=1e-3)
        assert err <= 1e-3, (key, err)
    h, w = (int(v) for v in g["trk_cal_hw"])
    ne = NormalEquations("cuda")
    ne.set_pose_host(g["trk_cal_T"])
    ne.launch_calib(d(g["trk_cal_Xf_c"]), d(g["trk_cal_Xk_c"]), d(g["trk_cal_Q"]),
                    d(g["trk_cal_valid"]), g["trk_cal_K"].astype(np.float32).reshape(9).copy(),
                    (h, w), c)
    H, gg, _ = ne.fetch()
    for key, a, b in (("calib_H", H, g["trk_cal_H"]), ("calib_g", gg, g["trk_cal_g"])):
        err = np.abs(a - b).max() / np.abs(b).max()
        parity("tracker_ne_" + key, max_rel=err, tol=1e-3)
        assert err <= 1e-3, (key, err)


@pytest.mark.gpu
@pytest.mark.parametrize("c", [0, 1])
def test_hip_match_vs_reference_glue(c):
    from splatt3r_amd.matching import match
    g = _g()
    pre = f"mt{c}_"
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    init = d(g[pre + "idx_init"]) if pre + "idx_init" in g.files else None
    idx, valid = match(d(g[pre + "X11"]), d(g[pre + "X21"]), d(g[pre + "D11"]),
                       d(g[pre + "D21"]), init)
    np.testing.assert_array_equal(idx.cpu().numpy(), g[pre + "idx"])
    np.testing.assert_array_equal(valid.cpu().numpy(), g[pre + "valid"])
