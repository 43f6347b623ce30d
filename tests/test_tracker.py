"""Tracker Gauss-Newton (include/s3t.h, splatt3r_amd/tracker.py) vs the numpy
oracle (oracle/tracker_ref.py, restating tracker.py:156-214).  The oracle's
Jacobian is pinned by finite differences of its own residual under the left
retraction Exp(d)*T (the parametrisation lietorch's retr uses)."""
import numpy as np
import pytest
import torch

import oracle
import oracle.tracker_ref as TR

CFG = dict(sigma_ray=0.003, sigma_dist=10.0, k=1.345)


def _scene(n, seed, noise=0.0):
    rng = np.random.default_rng(seed)
    Xk = np.concatenate([rng.uniform(-1, 1, (n, 2)), rng.uniform(1, 4, (n, 1))], 1)
    T_true = np.array([0.05, -0.02, 0.03, 0.02, -0.01, 0.015, 0.0, 1.02])
    T_true[6] = np.sqrt(1 - np.sum(T_true[3:6] ** 2))
    # Xf such that T_true . Xf = Xk
    Tinv = oracle.sim3_inv(T_true.astype(np.float32)[None])[0].astype(np.float64)
    Xf = TR.act_sim3(Tinv, Xk) + rng.normal(size=(n, 3)) * noise
    Q = rng.uniform(1.0, 3.0, (n, 1))
    valid = rng.uniform(size=(n, 1)) > 0.1
    return (Xf.astype(np.float32), Xk.astype(np.float32), Q.astype(np.float32), valid,
            T_true.astype(np.float32))


def _residual(T, Xf, Xk):
    return (TR.point_to_ray_dist(Xk.astype(np.float64)) -
            TR.point_to_ray_dist(TR.act_sim3(T, Xf.astype(np.float64))))


def test_oracle_jacobian_matches_finite_differences():
    Xf, Xk, Q, valid, _ = _scene(64, 0, noise=0.01)
    T = np.array([0.1, 0.0, -0.05, 0.0, 0.0, 0.0, 1.0, 1.1], np.float64)
    p = TR.act_sim3(T, Xf.astype(np.float64))
    dXdT = np.concatenate([np.broadcast_to(np.eye(3), (64, 3, 3)), -TR.skew(p), p[:, :, None]], -1)
    _, D = TR.point_to_ray_dist(p, jacobian=True)
    J = -D @ dXdT
    eps = 1e-4
    for j in range(7):
        d = np.zeros((1, 7), np.float32)
        d[0, j] = eps
        Tp = oracle.sim3_retr(T.astype(np.float32)[None], d)[0].astype(np.float64)
        d[0, j] = -eps
        Tm = oracle.sim3_retr(T.astype(np.float32)[None], d)[0].astype(np.float64)
        fd = (_residual(Tp, Xf, Xk) - _residual(Tm, Xf, Xk)) / (2 * eps)
        np.testing.assert_allclose(J[:, :, j], fd, rtol=2e-2, atol=2e-3, err_msg=f"col {j}")


def test_oracle_gn_recovers_pose():
    Xf, Xk, Q, valid, T_true = _scene(2000, 1)
    T = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    for _ in range(20):
        H, g, _ = TR.normal_equations(T, Xf, Xk, Q, valid, **CFG)
        tau = np.linalg.solve(H, g)
        T = oracle.sim3_retr(T[None], tau.astype(np.float32)[None])[0]
    np.testing.assert_allclose(TR.act_sim3(T, Xf), Xk, atol=1e-4)


def test_solve_normal_eqs_raises_like_cholesky():
    from splatt3r_amd.tracker import CholeskyError, solve_normal_eqs
    with pytest.raises(CholeskyError):
        solve_normal_eqs(-np.eye(7), np.ones(7))
    with pytest.raises(CholeskyError):
        solve_normal_eqs(np.full((7, 7), np.nan), np.ones(7))
    H = np.diag(np.arange(1.0, 8.0))
    np.testing.assert_allclose(solve_normal_eqs(H, np.ones(7)), 1 / np.arange(1.0, 8.0))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 196608])
def test_normal_equations_gpu_vs_oracle(n):
    from splatt3r_amd.tracker import NormalEquations
    Xf, Xk, Q, valid, _ = _scene(n, 2, noise=0.02)
    T = np.array([0.01, 0.02, -0.01, 0.01, 0.0, -0.01, 0.9999, 0.98], np.float32)
    T[3:7] /= np.linalg.norm(T[3:7])
    ne = NormalEquations("cuda")
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    H, g, cost = ne(T, d(Xf), d(Xk), d(Q), d(valid), CFG["sigma_ray"], CFG["sigma_dist"], CFG["k"])
    Hr, gr, cr = TR.normal_equations(T, Xf, Xk, Q, valid, **CFG)
    # fp32 per-point terms summed in fp32 per block / fp64 across blocks
    scale = np.abs(Hr).max()
    np.testing.assert_allclose(H, Hr, rtol=1e-3, atol=1e-5 * scale)
    np.testing.assert_allclose(g, gr, rtol=1e-3, atol=1e-5 * np.abs(gr).max())
    np.testing.assert_allclose(cost, cr, rtol=1e-3)


@pytest.mark.gpu
def test_invalid_points_contribute_nothing():
    from splatt3r_amd.tracker import NormalEquations
    Xf, Xk, Q, valid, _ = _scene(4096, 3, noise=0.02)
    valid[:] = False
    ne = NormalEquations("cuda")
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    H, g, cost = ne(np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32), d(Xf), d(Xk), d(Q), d(valid),
                    0.003, 10.0, 1.345)
    assert np.all(H == 0) and np.all(g == 0) and cost == 0


@pytest.mark.gpu
def test_opt_pose_ray_dist_sim3_recovers_pose():
    import lietorch
    from splatt3r_amd.tracker import FrameTracker
    Xf, Xk, Q, valid, T_true = _scene(196608, 4)
    tr = FrameTracker(None, None, "cuda")
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    T_WCk = lietorch.Sim3.Identity(1, device="cuda")
    T_WCf = lietorch.Sim3.Identity(1, device="cuda")
    T_WCf_new, T_CkCf = tr.opt_pose_ray_dist_sim3(d(Xf), d(Xk), T_WCf, T_WCk, d(Q), d(valid))
    got = T_CkCf.act(d(Xf)).cpu().numpy()
    np.testing.assert_allclose(got, Xk, atol=2e-4)
    assert 1 <= tr.last_iters < 50


@pytest.mark.gpu
def test_device_gn_loop_matches_host_loop():
    """s3t_gn_iterations (Cholesky/retr/convergence on the device) follows
    the host-driven loop: same iteration count, same pose to fp32 noise."""
    import lietorch
    from splatt3r_amd.tracker import FrameTracker
    Xf, Xk, Q, valid, _ = _scene(196608, 5, noise=0.01)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    I = lietorch.Sim3.Identity(1, device="cuda")
    tr = FrameTracker(None, None, "cuda")
    _, T_dev = tr.opt_pose_ray_dist_sim3(d(Xf), d(Xk), I, I, d(Q), d(valid))
    it_dev = tr.last_iters
    _, T_host = tr.opt_pose_ray_dist_sim3_host(d(Xf), d(Xk), I, I, d(Q), d(valid))
    assert abs(tr.last_iters - it_dev) <= 1
    np.testing.assert_allclose(T_dev.data.cpu().numpy(), T_host.data.cpu().numpy(), atol=2e-5)


@pytest.mark.gpu
def test_device_gn_reports_cholesky_failure():
    import lietorch
    from splatt3r_amd.tracker import CholeskyError, FrameTracker
    Xf, Xk, Q, valid, _ = _scene(4096, 6)
    valid[:] = False                       # H = 0: not positive definite
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    I = lietorch.Sim3.Identity(1, device="cuda")
    tr = FrameTracker(None, None, "cuda")
    with pytest.raises(CholeskyError):
        tr.opt_pose_ray_dist_sim3(d(Xf), d(Xk), I, I, d(Q), d(valid))


# ------------------------------------------------- calibrated (use_calib)
CAL = dict(pixel_border=-10.0, depth_eps=1e-6, sigma_pixel=1.0, sigma_depth=10.0, k=1.345)


def _calib_scene(h, w, seed, noise=0.0):
    """Keyframe pointmap on its pixel rays (constrain_points_to_ray) and a
    frame pointmap with T_true . Xf = Xk, so the calibrated residuals
    (tracker.py:216-270) vanish at T_true."""
    rng = np.random.default_rng(seed)
    f = 0.9 * max(h, w)
    K = np.array([[f, 0, w / 2], [0, f, h / 2], [0, 0, 1]], np.float32)
    v, u = np.divmod(np.arange(h * w), w)
    z = rng.uniform(1, 4, h * w)
    Xk = np.stack([(u - K[0, 2]) / K[0, 0] * z, (v - K[1, 2]) / K[1, 1] * z, z], 1)
    T_true = np.array([0.03, -0.02, 0.02, 0.01, -0.015, 0.01, 0.0, 1.03])
    T_true[6] = np.sqrt(1 - np.sum(T_true[3:6] ** 2))
    Tinv = oracle.sim3_inv(T_true.astype(np.float32)[None])[0].astype(np.float64)
    Xf = TR.act_sim3(Tinv, Xk) + rng.normal(size=(h * w, 3)) * noise
    Q = rng.uniform(1.0, 3.0, (h * w, 1))
    valid = rng.uniform(size=(h * w, 1)) > 0.1
    return (Xf.astype(np.float32), Xk.astype(np.float32), Q.astype(np.float32), valid,
            T_true.astype(np.float32), K)


def _calib_ne(T, Xf, Xk, Q, valid, K, hw):
    return TR.normal_equations_calib(T, Xf, Xk, Q, valid, K, hw, CAL["pixel_border"],
                                     CAL["depth_eps"], CAL["sigma_pixel"], CAL["sigma_depth"],
                                     CAL["k"])


def test_oracle_calib_jacobian_matches_finite_differences():
    h, w = 8, 8
    Xf, Xk, Q, valid, _, K = _calib_scene(h, w, 10, noise=0.01)
    T = np.array([0.05, 0.0, -0.03, 0.0, 0.0, 0.0, 1.0, 1.05], np.float64)

    def res(Tx):
        pz, _, _ = TR.project_calib(TR.act_sim3(Tx, Xf.astype(np.float64)), K, (h, w))
        return TR.calib_measurements(Xk, (h, w), 1e-6)[0] - pz

    p = TR.act_sim3(T, Xf.astype(np.float64))
    dXdT = np.concatenate([np.broadcast_to(np.eye(3), (h * w, 3, 3)), -TR.skew(p),
                           p[:, :, None]], -1)
    _, D, _ = TR.project_calib(p, K, (h, w))
    J = -D @ dXdT
    eps = 1e-4
    for j in range(7):
        d = np.zeros((1, 7), np.float32)
        d[0, j] = eps
        Tp = oracle.sim3_retr(T.astype(np.float32)[None], d)[0].astype(np.float64)
        d[0, j] = -eps
        Tm = oracle.sim3_retr(T.astype(np.float32)[None], d)[0].astype(np.float64)
        fd = (res(Tp) - res(Tm)) / (2 * eps)
        scale = np.abs(J[:, :, j]).max() + 1e-9
        np.testing.assert_allclose(J[:, :, j], fd, rtol=3e-2, atol=3e-2 * scale, err_msg=f"col {j}")


def test_oracle_calib_gn_recovers_pose():
    h, w = 24, 32
    Xf, Xk, Q, valid, T_true, K = _calib_scene(h, w, 11)
    T = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    for _ in range(20):
        H, g, _ = _calib_ne(T, Xf, Xk, Q, valid, K, (h, w))
        T = oracle.sim3_retr(T[None], np.linalg.solve(H, g).astype(np.float32)[None])[0]
    np.testing.assert_allclose(TR.act_sim3(T, Xf), Xk, atol=1e-3)


def test_oracle_calib_masks():
    """Points behind the camera, outside image+border and keyframe depths
    <= depth_eps contribute nothing (valid_proj & valid_meas, tracker.py:234)."""
    h, w = 4, 4
    Xf, Xk, Q, valid, _, K = _calib_scene(h, w, 12)
    valid[:] = True
    I = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    Xf2 = Xf.copy()
    Xf2[:, 2] = -1.0                   # every point behind the camera
    H, g, c = _calib_ne(I, Xf2, Xk, Q, valid, K, (h, w))
    assert np.all(H == 0) and np.all(g == 0) and c == 0
    Xk2 = Xk.copy()
    Xk2[:, 2] = 0.0                    # no valid keyframe depth
    H, g, c = _calib_ne(I, Xf, Xk2, Q, valid, K, (h, w))
    assert np.all(H == 0) and c == 0


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(1, 1), (24, 32), (384, 512)])
def test_calib_normal_equations_gpu_vs_oracle(hw):
    from splatt3r_amd.config import config
    from splatt3r_amd.tracker import NormalEquations
    h, w = hw
    Xf, Xk, Q, valid, _, K = _calib_scene(h, w, 13, noise=0.01)
    # a ring of points pushed outside the border and one behind the camera
    Xf[:: 7, 0] += 50.0
    if h * w > 1:
        Xf[1, 2] = -2.0
    T = np.array([0.01, 0.02, -0.01, 0.01, 0.0, -0.01, 0.9999, 0.98], np.float32)
    T[3:7] /= np.linalg.norm(T[3:7])
    ne = NormalEquations("cuda")
    ne.set_pose_host(T)
    cfg = dict(config["tracking"], **{k: v for k, v in CAL.items() if k != "k"}, huber=CAL["k"])
    ne.launch_calib(_dev(Xf), _dev(Xk), _dev(Q), _dev(valid), K.reshape(9).copy(), (h, w), cfg)
    H, g, cost = ne.fetch()
    Hr, gr, cr = _calib_ne(T, Xf, Xk, Q, valid, K, (h, w))
    scale = np.abs(Hr).max() + 1e-30
    np.testing.assert_allclose(H, Hr, rtol=2e-3, atol=2e-5 * scale)
    np.testing.assert_allclose(g, gr, rtol=2e-3, atol=2e-5 * (np.abs(gr).max() + 1e-30))
    np.testing.assert_allclose(cost, cr, rtol=2e-3, atol=1e-6)


@pytest.mark.gpu
def test_opt_pose_calib_sim3_recovers_pose():
    import lietorch
    from splatt3r_amd.tracker import FrameTracker
    h, w = 384, 512
    Xf, Xk, Q, valid, _, K = _calib_scene(h, w, 14)
    tr = FrameTracker(None, None, "cuda")
    I = lietorch.Sim3.Identity(1, device="cuda")
    _, T_CkCf = tr.opt_pose_calib_sim3(_dev(Xf), _dev(Xk), I, I, _dev(Q), _dev(valid),
                                       _dev(K), (h, w))
    got = T_CkCf.act(_dev(Xf)).cpu().numpy()
    np.testing.assert_allclose(got, Xk, atol=2e-3)
    assert 1 <= tr.last_iters < 50


@pytest.mark.gpu
def test_calib_device_gn_matches_oracle_loop():
    """Each device iteration (normal equations + fp64 Cholesky + retr) tracks
    the float64 oracle's loop from the same start: same pose after 3 steps."""
    import lietorch
    from splatt3r_amd.tracker import FrameTracker
    h, w = 96, 128
    Xf, Xk, Q, valid, _, K = _calib_scene(h, w, 15, noise=0.005)
    T = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    for _ in range(3):
        H, g, _ = _calib_ne(T, Xf, Xk, Q, valid, K, (h, w))
        T = oracle.sim3_retr(T[None], np.linalg.solve(H, g).astype(np.float32)[None])[0]
    tr = FrameTracker(None, None, "cuda")
    tr.cfg = dict(tr.cfg, max_iters=3, rel_error=0.0, delta_norm=0.0)
    I = lietorch.Sim3.Identity(1, device="cuda")
    _, T_dev = tr.opt_pose_calib_sim3(_dev(Xf), _dev(Xk), I, I, _dev(Q), _dev(valid),
                                      _dev(K), (h, w))
    assert tr.last_iters == 3
    np.testing.assert_allclose(T_dev.data.cpu().numpy().reshape(8), T, atol=5e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(196608, 0), (1000, 1), (63, 2)])
def test_track_prep_matches_torch_reference_expressions(n, seed):
    """s3t_track_prep == the reference's torch expressions (tracker.py:
    28-91): gathers and masks exact, Qk = sqrt(Qff[idx] * Qkf) within one
    ulp (device sqrt), the three decision counts exact (incl. the unique
    count of hit keyframe pixels, with many duplicate matches)."""
    from splatt3r_amd.tracker import track_prep
    g = torch.Generator(device="cuda").manual_seed(seed)
    r = lambda *s: torch.rand(*s, device="cuda", generator=g)
    idx = torch.randint(0, n, (n,), device="cuda", generator=g)
    idx[: n // 3] = idx[0]                                   # duplicate hits
    vm = r(n, 1) > 0.3
    Xf = torch.randn(n, 3, device="cuda", generator=g)
    Cf, Ck = r(n, 1) * 3, r(n, 1) * 3
    Qff, Qkf = r(n, 1) * 4, r(n, 1) * 4
    C_conf, Q_conf = 1.0, 1.5
    Xo, Qo, vo, cnt = track_prep(idx, vm, Xf, Cf, Ck, Qff, Qkf, C_conf, Q_conf)
    Qk = torch.sqrt(Qff[idx] * Qkf)
    torch.testing.assert_close(Qo, Qk, rtol=2e-7, atol=0)
    assert torch.equal(Xo, Xf[idx])
    vq = Qo > Q_conf                                        # masks from the kernel's own Qk
    vopt = vm & (Cf[idx] > C_conf) & (Ck > C_conf) & vq
    assert torch.equal(vo, vopt)
    ref = [int(vopt.sum()), int((vm & vq).sum()), int(torch.unique(idx[vm[:, 0]]).numel())]
    assert cnt.cpu().tolist() == ref
