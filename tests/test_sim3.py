"""Sim3 group ops (lietorch replacement, include/s3lie.h) vs the oracle
restatement of gn_kernels.cu:171-452.  Parity vs lietorch itself is unpinned
(submodule absent); the oracle is pinned by group identities below."""
import ctypes

import numpy as np
import pytest
import torch

import oracle


def rand_sim3(n, rng, tscale=1.0):
    t = rng.normal(size=(n, 3)) * tscale
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    s = np.exp(rng.normal(size=(n, 1)) * 0.3)
    return np.concatenate([t, q, s], 1).astype(np.float32)


def sim3_matrix_np(T):
    T = T.astype(np.float64)
    x, y, z, w = T[:, 3], T[:, 4], T[:, 5], T[:, 6]
    R = np.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
        2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
        2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
    M = np.zeros((T.shape[0], 4, 4))
    M[:, :3, :3] = R * T[:, 7, None, None]
    M[:, :3, 3] = T[:, :3]
    M[:, 3, 3] = 1
    return M


def xi_cases(rng, n):
    xi = rng.normal(size=(n, 7)).astype(np.float32) * 0.5
    # small-angle / small-scale branches (gn_kernels.cu:303-311, :341-358)
    xi[0, 3:6] = 0.0
    xi[1, 6] = 0.0
    xi[2, 3:7] = 0.0
    xi[3, 3:6] = 1e-5
    xi[4, 6] = 1e-7
    return xi


# ------------------------------------------------------------- CPU: oracle
def test_oracle_exp_zero_is_identity():
    E = oracle.sim3_exp(np.zeros((1, 7), np.float32))
    np.testing.assert_array_equal(E[0], [0, 0, 0, 0, 0, 0, 1, 1])


def test_oracle_act_matches_matrix_form():
    rng = np.random.default_rng(0)
    T = rand_sim3(64, rng)
    X = rng.normal(size=(64, 3)).astype(np.float32)
    Y = np.stack([oracle.sim3_act(T[i], X[i])[0] for i in range(64)])
    M = sim3_matrix_np(T)
    Yr = np.einsum("nij,nj->ni", M[:, :3, :3], X) + M[:, :3, 3]
    np.testing.assert_allclose(Y, Yr, rtol=1e-5, atol=1e-5)


def test_oracle_mul_inv_roundtrip():
    rng = np.random.default_rng(1)
    T = rand_sim3(32, rng)
    I = oracle.sim3_mul(T, oracle.sim3_inv(T))
    np.testing.assert_allclose(I[:, :3], 0, atol=1e-5)
    np.testing.assert_allclose(np.abs(I[:, 6]), 1, atol=1e-6)
    np.testing.assert_allclose(I[:, 7], 1, rtol=1e-6)


def test_oracle_mul_is_matrix_product():
    rng = np.random.default_rng(2)
    A, B = rand_sim3(16, rng), rand_sim3(16, rng)
    C = oracle.sim3_mul(A, B)
    np.testing.assert_allclose(sim3_matrix_np(C), sim3_matrix_np(A) @ sim3_matrix_np(B),
                               rtol=1e-5, atol=1e-5)


def test_oracle_exp_branches_continuous():
    # exp near the small-angle thresholds agrees with exp at tiny offsets
    xi = np.zeros((2, 7), np.float32)
    xi[:, 0:3] = [0.3, -0.2, 0.1]
    xi[1, 3:6] = 2e-3   # theta^2 = 1.2e-5 > EPS: regular branch
    xi[0, 3:6] = 5e-4   # theta^2 = 7.5e-7 < EPS: Taylor branch
    E = oracle.sim3_exp(xi)
    np.testing.assert_allclose(E[0, :3], E[1, :3], atol=2e-3)
    np.testing.assert_allclose(E[:, 6], 1.0, atol=1e-5)


def test_oracle_retr_is_exp_times_T():
    rng = np.random.default_rng(3)
    T = rand_sim3(16, rng)
    xi = xi_cases(rng, 16)
    R = oracle.sim3_retr(T, xi)
    M = sim3_matrix_np(oracle.sim3_exp(xi)) @ sim3_matrix_np(T)
    np.testing.assert_allclose(sim3_matrix_np(R), M, rtol=1e-5, atol=1e-5)


def test_native_host_helpers_match_oracle_bitwise():
    from splatt3r_amd import _lib
    lib = _lib.lib()
    rng = np.random.default_rng(4)
    T = rand_sim3(8, rng)
    xi = xi_cases(rng, 8)
    for i in range(8):
        out = np.zeros(8, np.float32)
        lib.s3lie_sim3_retr_host(T[i].ctypes.data, xi[i].ctypes.data, out.ctypes.data)
        np.testing.assert_array_equal(out, oracle.sim3_retr(T[i], xi[i])[0])
        lib.s3lie_sim3_mul_host(T[i].ctypes.data, T[(i + 1) % 8].ctypes.data, out.ctypes.data)
        np.testing.assert_array_equal(out, oracle.sim3_mul(T[i], T[(i + 1) % 8])[0])
        lib.s3lie_sim3_inv_host(T[i].ctypes.data, out.ctypes.data)
        np.testing.assert_array_equal(out, oracle.sim3_inv(T[i])[0])


def test_lietorch_shim_cpu_group_ops():
    import lietorch
    rng = np.random.default_rng(5)
    T = lietorch.Sim3(torch.from_numpy(rand_sim3(4, rng)))
    I = (T * T.inv()).data.numpy()
    np.testing.assert_allclose(I[:, :3], 0, atol=1e-5)
    ident = lietorch.Sim3.Identity(1)
    assert ident.data.tolist() == [[0, 0, 0, 0, 0, 0, 1, 1]]
    assert lietorch.Sim3.embedded_dim == 8
    M = T.matrix().numpy()
    np.testing.assert_allclose(M, sim3_matrix_np(T.data.numpy()), rtol=1e-5, atol=1e-6)


# -------------------------------------------------------------- GPU: HIP
@pytest.mark.gpu
def test_hip_sim3_ops_vs_oracle():
    import lietorch
    rng = np.random.default_rng(10)
    n = 4096
    Tn, Un = rand_sim3(n, rng), rand_sim3(n, rng)
    xin = xi_cases(rng, n)
    Xn = rng.normal(size=(n, 3)).astype(np.float32) * 3
    T = lietorch.Sim3(torch.from_numpy(Tn).cuda())
    U = lietorch.Sim3(torch.from_numpy(Un).cuda())
    # act, mul, inv: pure +,-,*,/ and sqrt -> bit-exact vs the strict oracle
    np.testing.assert_array_equal(T.act(torch.from_numpy(Xn).cuda()).cpu().numpy(),
                                  oracle.sim3_act(Tn, Xn))
    np.testing.assert_array_equal((T * U).data.cpu().numpy(), oracle.sim3_mul(Tn, Un))
    np.testing.assert_array_equal(T.inv().data.cpu().numpy(), oracle.sim3_inv(Tn))
    # exp / retr go through sinf/cosf/expf (libm vs device ocml, ~1 ulp); the
    # W coefficients (C - ...)/theta^2 (gn_kernels.cu:367-370) cancel, which
    # amplifies that to ~1e-5 absolute on the translation.
    xi = torch.from_numpy(xin).cuda()
    np.testing.assert_allclose(lietorch.Sim3.exp(xi).data.cpu().numpy(), oracle.sim3_exp(xin),
                               rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(T.retr(xi).data.cpu().numpy(), oracle.sim3_retr(Tn, xin),
                               rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_hip_sim3_broadcast_act_and_log_roundtrip():
    import lietorch
    rng = np.random.default_rng(11)
    Tn = rand_sim3(1, rng)
    Xn = rng.normal(size=(1, 5000, 3)).astype(np.float32)
    T = lietorch.Sim3(torch.from_numpy(Tn).cuda())
    Y = T.act(torch.from_numpy(Xn).cuda())
    assert Y.shape == (1, 5000, 3)
    np.testing.assert_array_equal(Y[0].cpu().numpy(), oracle.sim3_act(Tn, Xn[0]))
    xi = torch.from_numpy(xi_cases(rng, 256)).cuda()
    back = lietorch.Sim3.exp(xi).log()
    np.testing.assert_allclose(back.cpu().numpy(), xi.cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_hip_pose_retr_in_place():
    from splatt3r_amd import _lib
    rng = np.random.default_rng(12)
    P = rand_sim3(37, rng)
    dx = rng.normal(size=(36, 7)).astype(np.float32) * 0.1
    Pd = torch.from_numpy(P).cuda()
    _lib.call("s3lie_pose_retr", Pd.data_ptr(), torch.from_numpy(dx).cuda().data_ptr(), 37, 1,
              _lib.stream())
    np.testing.assert_allclose(Pd.cpu().numpy(), oracle.pose_retr(P, dx, 1), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(Pd.cpu().numpy()[0], P[0])  # pinned pose untouched


@pytest.mark.gpu
def test_hip_matrix():
    import lietorch
    rng = np.random.default_rng(13)
    Tn = rand_sim3(100, rng)
    M = lietorch.Sim3(torch.from_numpy(Tn).cuda()).matrix().cpu().numpy()
    np.testing.assert_allclose(M, sim3_matrix_np(Tn), rtol=1e-5, atol=1e-6)
    S = lietorch.SE3(torch.from_numpy(Tn[:, :7]).cuda()).matrix().cpu().numpy()
    Tn1 = Tn.copy()
    Tn1[:, 7] = 1
    np.testing.assert_allclose(S, sim3_matrix_np(Tn1), rtol=1e-5, atol=1e-6)
