"""Keyframe-pair sharding and the map all-gather (splatt3r_amd/pairs.py),
world_size 2 over gloo on the CPU, plus the world transform vs numpy."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_partitions_pairs():
    from splatt3r_amd.pairs import shard
    pairs = [(i, j) for j in range(1, 9) for i in range(max(0, j - 4), j)]
    for ws in (1, 2, 3, 8):
        parts = [shard(pairs, ws, r) for r in range(ws)]
        flat = [p for part in parts for p in part]
        assert sorted(flat) == sorted(pairs)
        assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from splatt3r_amd.pairs import GAUSS_FLOATS, gather_map
    n = 5 + 3 * rank                       # unequal shards
    recs = torch.full((n, GAUSS_FLOATS), float(rank)) + torch.arange(n)[:, None] * 0.01
    out = gather_map(recs, ws)
    q.put((rank, out.numpy()))
    dist.destroy_process_group()


def test_gather_map_world_size_2_gloo():
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.concatenate([np.full((5 + 3 * r, 13), float(r)) + np.arange(5 + 3 * r)[:, None] * 0.01
                           for r in range(ws)]).astype(np.float32)
    for r in range(ws):
        np.testing.assert_array_equal(res[r], want)


@pytest.mark.gpu
def test_world_gaussians_matches_numpy():
    from splatt3r_amd.pairs import world_gaussians
    rng = np.random.default_rng(0)
    h, w = 4, 6
    q = rng.normal(size=(1, h, w, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    res = dict(means=torch.from_numpy(rng.normal(size=(1, h, w, 3)).astype(np.float32)),
               scales=torch.from_numpy(rng.uniform(0.01, 0.1, (1, h, w, 3)).astype(np.float32)),
               rotations=torch.from_numpy(q),
               sh=torch.from_numpy(rng.normal(size=(1, h, w, 3, 1)).astype(np.float32) * 0.1),
               opacities=torch.from_numpy(rng.uniform(size=(1, h, w, 1)).astype(np.float32)))
    T = torch.tensor([0.1, -0.2, 0.3, 0.0, 0.0, np.sin(0.2), np.cos(0.2), 1.5])
    img = torch.from_numpy(rng.uniform(-1, 1, (1, 3, h, w)).astype(np.float32))
    out = world_gaussians({k: v[0].cuda() for k, v in res.items()}, T.cuda(), img.cuda())
    out = out.cpu().numpy()
    # numpy restatement of splatt3r_utils.py:290-312
    c, s_ = np.cos(0.4), np.sin(0.4)
    R = np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1]]) * 1.5
    t = np.array([0.1, -0.2, 0.3])
    m = res["means"].numpy().reshape(-1, 3)
    np.testing.assert_allclose(out[:, :3], m @ R.T + t, rtol=1e-5, atol=1e-5)
    from splatt3r_amd.synthetic import quat_xyzw_to_rot
    Rq = quat_xyzw_to_rot(q.reshape(-1, 4))
    sc = res["scales"].numpy().reshape(-1, 3)
    cov = np.einsum("nij,nj,nkj->nik", Rq, sc * sc, Rq)
    cw = R @ cov @ R.T
    iu = np.triu_indices(3)
    np.testing.assert_allclose(out[:, 3:9], cw[:, iu[0], iu[1]], rtol=1e-4, atol=1e-7)
    rgb = np.clip(img[0].numpy().transpose(1, 2, 0).reshape(-1, 3) * 0.5 + 0.5, 0, 1)
    C0 = 0.28209479177387814
    sh0 = res["sh"].numpy().reshape(-1, 3) + (rgb - 0.5) / C0
    np.testing.assert_allclose(out[:, 9:12], np.clip(sh0 * C0 + 0.5, 0, 1), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(out[:, 12], res["opacities"].numpy().reshape(-1))
