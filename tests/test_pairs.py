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


def fake_match_dir(feat_a, pos_a, feat_b, pos_b, shape_a, shape_b):
    """Deterministic stand-in for splatt3r_match_directed (no network on the
    CPU): (idx_a2b, valid, Q_aa, Q_ba) with its shapes and dtypes, values
    derived from the keyframe features so every ordered pair differs."""
    H, W = (int(v) for v in shape_a[0].reshape(-1)[:2])
    hw = H * W
    ka = feat_a[:, 0, 0].round().long()
    kb = feat_b[:, 0, 0].round().long()
    ar = torch.arange(hw)
    idx = (ar[None] * (ka[:, None] + 1) + kb[:, None] * 7) % hw
    valid = ((ar[None] + ka[:, None] + 2 * kb[:, None]) % 3 != 0)[..., None]
    q = lambda s: (1.0 + ((ar[None] * (s[:, None] + 2)) % 11).float() * (s[:, None] + 1).float()
                   / 5.0)[..., None]
    return idx, valid, q(ka), q(ka * 2 + kb)


def fake_match(feat_i, pos_i, feat_j, pos_j, shape_i, shape_j):
    """The symmetric 8-tuple (splatt3r_match_symmetric's order) of the two
    directed stand-ins, as the network's symmetric call is its two
    directions."""
    a = fake_match_dir(feat_i, pos_i, feat_j, pos_j, shape_i, shape_j)
    b = fake_match_dir(feat_j, pos_j, feat_i, pos_i, shape_j, shape_i)
    return a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3]


def _kf_frames(n, H=32, W=48):
    from splatt3r_amd.frame import Frame
    from splatt3r_amd.net import positions
    frames = []
    for k in range(n):
        f = Frame(k, torch.zeros(1, 3, H, W), torch.tensor([[H, W]]), torch.tensor([[H, W]]),
                  T_WC=object())
        f.feat = torch.full((1, (H // 16) * (W // 16), 8), float(k))
        f.pos = positions(1, H // 16, W // 16, "cpu")
        frames.append(f)
    return frames


PAIRS = [[(0, 1), (1, 2), (0, 2), (2, 3), (1, 3), (0, 3), (3, 4)], [(4, 5), (2, 5), (1, 5)]]


def _edges(fg):
    return {k: getattr(fg, k).clone() for k in ("ii", "jj", "idx_ii2jj", "idx_jj2ii",
                                                "valid_match_j", "valid_match_i", "Q_ii2jj",
                                                "Q_jj2ii")}


def _shard_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from splatt3r_amd.global_opt import FactorGraph
    from splatt3r_amd.pairs import PairShard
    sh = PairShard(None, "cpu", match_fn=fake_match, match_dir_fn=fake_match_dir)
    if rank == 0:
        frames = _kf_frames(6)
        for k, f in enumerate(frames):
            sh.broadcast_keyframe(k, f)
        fg = FactorGraph(None, frames, device="cpu", shard=sh)
        accepted = [fg.add_factors([p[0] for p in ps], [p[1] for p in ps], 0.5) for ps in PAIRS]
        sh.stop()
        q.put((rank, (accepted, {k: v.numpy() for k, v in _edges(fg).items()}, sh.stats)))
    else:
        sh.serve()
        q.put((rank, sh.stats))
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_add_factors_matches_single_rank_gloo(ws):
    """FactorGraph.add_factors with the pair shard over ws gloo ranks (pair p
    on rank p mod ws, keyframe features broadcast at creation, idx/valid/Q
    gathered to rank 0) builds exactly the single-rank edges."""
    from splatt3r_amd.global_opt import FactorGraph
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    accepted, edges, st0 = res[0]
    fg = FactorGraph(None, _kf_frames(6), device="cpu", match_fn=fake_match)
    want_acc = [fg.add_factors([p[0] for p in ps], [p[1] for p in ps], 0.5) for ps in PAIRS]
    assert accepted == want_acc
    for k, v in _edges(fg).items():
        np.testing.assert_array_equal(edges[k], v.numpy(), err_msg=k)
    assert len(edges["ii"]) > 0
    # every rank received every keyframe and ran its share of the pairs'
    # directed units (two per pair: no rank idles on a small batch)
    n_pairs = sum(len(ps) for ps in PAIRS)
    assert sum(res[r]["units"] if r else st0["units"] for r in range(ws)) == 2 * n_pairs
    assert st0["pairs"] == n_pairs
    assert all((res[r] if r else st0)["keyframes"] == 6 for r in range(ws))


@pytest.mark.gpu
def test_world_records_matches_numpy():
    """world_records (the map records of refresh_map, include/s3w.h) with its
    filters off: the world transform of gaussians_to_world vs numpy."""
    import lietorch
    from splatt3r_amd.splatt3r_utils import world_records
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
    M = lietorch.Sim3(T.cuda().reshape(1, 8)).matrix()[0]
    out, cnt = world_records({k: v[0].cuda() for k, v in res.items()}, img.cuda()[0], M)
    assert int(cnt) == h * w
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


def _beat(rank, msg):
    import time
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "progress.log"), "a") as f:
        f.write(f"{time.time():.1f} rank {rank}: {msg}\n")


def _gpu_shard_worker(rank, ws, port, q):
    # static GEMM launch policy: the per-process tuner times candidates and
    # may pick other tiles in another process (same math, other rounding)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), S3_GEMM_TUNE="0")
    _beat(rank, "init")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from dist_util import init_gpu_group
    dev = init_gpu_group(rank, ws, 240)
    _beat(rank, f"process group up ({dist.get_backend()})")
    try:
        from splatt3r_amd.frame import Keyframes, create_frame
        from splatt3r_amd.pairs import PairShard, q_weighted
        from splatt3r_amd.splatt3r_utils import load_splatt3r, splatt3r_match_symmetric
        from splatt3r_amd.synthetic import tum_like_sequence
        from splatt3r_amd.weights import FULL
        model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
        _beat(rank, "model loaded")
        sh = PairShard(model, dev)
        pairs = [(0, 1), (1, 2), (0, 2), (2, 3), (1, 3)]
        if rank == 0:
            imgs = tum_like_sequence(4, 384, 512, seed=5, step_px=3.0, device=dev)
            kfs = Keyframes()
            for k in range(4):
                f = create_frame(k, imgs[k], device=dev)
                f.feat, f.pos, _ = model.encoder._encode_image(f.img, f.img_true_shape)
                kfs.append(f)
                sh.broadcast_keyframe(k, f)
            _beat(rank, "keyframes broadcast")
            got = sh.match_pairs([p[0] for p in pairs], [p[1] for p in pairs])
            _beat(rank, "pairs gathered")
            # the single-rank answer: one symmetric decode of every pair (the
            # batch-invariant backend plans make the rank split irrelevant)
            cat = lambda ks, a: torch.cat([getattr(kfs[k], a) for k in ks])
            ii, jj = [p[0] for p in pairs], [p[1] for p in pairs]
            m = splatt3r_match_symmetric(model, cat(ii, "feat"), cat(ii, "pos"), cat(jj, "feat"),
                                         cat(jj, "pos"), [kfs[0].img_true_shape] * len(pairs),
                                         [kfs[0].img_true_shape] * len(pairs))
            want = q_weighted(m, sh.Q_conf)
            ok = all(torch.equal(got[k], want[k]) for k in range(6))
            # the global-map refresh: keyframe k re-inferred against partner
            # k+1 (k-1 for the last) on rank k mod 2, world records at its
            # pose, all-gathered into both ranks' maps
            from splatt3r_amd.gaussian_map import SharedGaussians, render_map
            import lietorch
            poses = torch.stack([lietorch.Sim3.Identity(1, device=dev).data.reshape(8)] * 4)
            poses[:, 0] = torch.arange(4, device=dev) * 0.05
            edges_i, edges_j = [0, 1, 2, 3], [1, 2, 3, 2]
            sh.gmap = SharedGaussians(max_gaussians=1 << 20, device=dev)
            # (portable-PRNG opacities sit near 0.12: threshold 0 keeps them)
            sh.refresh_map(edges_i, edges_j, poses, spatial_stride=4, opacity_threshold=0.0)
            _beat(rank, "map refreshed")
            sh.stop()
            local = PairShard(model, dev, gmap=SharedGaussians(max_gaussians=1 << 20, device=dev),
                              local=True)
            for k in range(4):
                local.register_local(k, kfs[k])
            local.refresh_map(edges_i, edges_j, poses, spatial_stride=4, opacity_threshold=0.0)
            n = sh.gmap.n_gaussians
            map_ok = n == local.gmap.n_gaussians and n > 0 and all(
                torch.equal(getattr(sh.gmap, a)[:n], getattr(local.gmap, a)[:n])
                for a in ("means", "cov_triu", "colors", "opacities", "kf_id"))
            T = np.eye(4, dtype=np.float32)
            T[2, 3] = -1.0
            img0 = render_map(sh.gmap, T, 256, 192, 60.0)
            img1 = render_map(local.gmap, T, 256, 192, 60.0)
            q.put((rank, (ok, map_ok, bool(torch.equal(img0, img1)), n,
                          sh.gmap.means[:n].double().sum().item())))
        else:
            from splatt3r_amd.gaussian_map import SharedGaussians
            sh.gmap = SharedGaussians(max_gaussians=1 << 20, device=dev)
            sh.serve()
            _beat(rank, "served")
            n = sh.gmap.n_gaussians
            q.put((rank, (sh.stats["units"], n, sh.gmap.means[:n].double().sum().item())))
    except Exception as e:           # report instead of leaving the peer blocked
        q.put((rank, f"error: {e!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_pairs_two_ranks_on_gpu_match_local_decode():
    """Two ranks on the GPU (gloo transport staged through the host): keyframe
    features broadcast from rank 0, each pair's two directions decoded as
    units on ranks u mod 2 with the real network, idx/valid/Q gathered back
    in pair order -- bit-identical to one symmetric decode of all pairs on a
    single rank (batch-invariant backend plans).  Then the global-map refresh
    (PairShard.refresh_map): edges re-inferred across the ranks, filtered
    world records all-gathered into both ranks' SharedGaussians -- both maps
    equal the single-rank map and render_map of it is bit-identical."""
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_shard_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = {}
    try:
        while len(res) < ws:
            r, v = q.get(timeout=300)
            res[r] = v
            assert not (isinstance(v, str) and v.startswith("error")), (r, v)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    ok, map_ok, render_ok, n0, sum0 = res[0]
    pairs1, n1, sum1 = res[1]
    assert ok is True
    assert pairs1 == 5          # units 1, 3, .., 9: the (j, i) direction of every pair
    # refresh_map: both ranks hold the same map, equal to the single-rank map,
    # and its render is bit-identical
    assert map_ok and render_ok
    assert n0 == n1 and sum0 == sum1


FAKE_CAP = 10


def fake_map(pairs, poses, params):
    """Deterministic stand-in for PairShard._map_records (no network on the
    CPU): a variable number of records per edge (3..9 of FAKE_CAP rows, the
    rest garbage that must never reach the map), valued from the edge, the
    keyframe pose and the filter parameters."""
    buf = torch.full((len(pairs), FAKE_CAP, 13), -7.0)
    cnt = torch.zeros(len(pairs), dtype=torch.int64)
    for p, (i, j) in enumerate(pairs):
        n = 3 + (5 * i + j) % 7
        base = poses[i].sum() + float(params[1]) + 10 * i + j
        buf[p, :n] = base + torch.arange(n * 13, dtype=torch.float32).reshape(n, 13) * 0.5
        cnt[p] = n
    return buf, cnt


def fake_records(pairs, poses, params):
    """fake_map's records, compacted (the single-rank expectation)."""
    buf, cnt = fake_map(pairs, poses, params)
    return [buf[p, :int(cnt[p])] for p in range(len(pairs))]


MAP_EDGES = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (0, 2), (1, 3)]


def _map_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from splatt3r_amd.pairs import PairShard
    sh = PairShard(None, "cpu", match_fn=fake_match, map_fn=fake_map, match_dir_fn=fake_match_dir,
                   map_cap=lambda pairs, hp: FAKE_CAP)
    poses = torch.arange(6 * 8, dtype=torch.float32).reshape(6, 8) * 0.1
    if rank == 0:
        for k, f in enumerate(_kf_frames(6)):
            sh.broadcast_keyframe(k, f)
        recs = sh.refresh_map([e[0] for e in MAP_EDGES], [e[1] for e in MAP_EDGES], poses,
                              spatial_stride=4, depth_max_percentile=0.9)
        sh.stop()
    else:
        sh.serve()
        recs = sh.last_map
    q.put((rank, [r.numpy() for r in recs]))
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_map_refresh_matches_single_rank_gloo(ws):
    """refresh_map over ws gloo ranks: edge e re-inferred on rank e mod ws,
    variable-length record sets padded to a fixed capacity and all-gathered
    with their counts -- every rank holds exactly the single-rank records,
    in edge order, and no padding row leaks."""
    from splatt3r_amd.pairs import PairShard
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_map_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sh = PairShard(None, "cpu", map_fn=fake_map, map_cap=lambda pairs, hp: FAKE_CAP)
    poses = torch.arange(6 * 8, dtype=torch.float32).reshape(6, 8) * 0.1
    single = sh.refresh_map([e[0] for e in MAP_EDGES], [e[1] for e in MAP_EDGES], poses,
                            spatial_stride=4, depth_max_percentile=0.9)
    want = fake_records(MAP_EDGES, poses, (4.0, 0.9, 1.0, 1.5, 0.3))
    assert [w.shape[0] for w in want] == [int(c) for c in single.counts]
    for got, w in zip(single, want):
        np.testing.assert_array_equal(got.numpy(), w.numpy())
    for r in range(ws):
        assert len(res[r]) == len(MAP_EDGES)
        for got, w in zip(res[r], want):
            np.testing.assert_array_equal(got, w.numpy())


def test_shard_check_detects_a_corrupted_unit():
    """PairShard.check_units / check_map (bench.py --gpus N shard_check):
    the local re-decode equals an intact gathered batch, and a single
    flipped index, valid flag, Q bit or map record is reported unequal."""
    from splatt3r_amd.pairs import PairShard
    sh = PairShard(None, "cpu", match_fn=fake_match, match_dir_fn=fake_match_dir,
                   map_fn=fake_map, map_cap=lambda pairs, hp: FAKE_CAP)
    for k, f in enumerate(_kf_frames(5)):
        sh.register_local(k, f)
    ii, jj = [0, 1, 0, 2, 1], [1, 2, 2, 3, 3]
    got = sh.match_pairs(ii, jj)
    assert sh.check_units(ii, jj, got, max_units=10)["equal"] is True
    assert sh.stats["units"] == 0                     # the check is not counted as work
    for k, tamper in ((0, lambda t: t.view(-1)[17].add_(1)),
                      (3, lambda t: t.view(-1)[5].logical_not_()),
                      (5, lambda t: t.view(-1)[9].add_(1e-6))):
        bad = [t.clone() for t in got]
        tamper(bad[k])
        assert sh.check_units(ii, jj, bad, max_units=10)["equal"] is False
    poses = torch.arange(6 * 8, dtype=torch.float32).reshape(6, 8) * 0.1
    mi, mj = [0, 1, 2, 3], [1, 2, 3, 2]
    hp = (4.0, 0.98, 1.0, 1.5, 0.0)
    recs = sh.refresh_map(mi, mj, poses, spatial_stride=4, opacity_threshold=0.0)
    assert sh.check_map(mi, mj, poses, hp, recs, max_pairs=4)["equal"] is True
    recs.buffers[2, 1, 4] += 1.0
    assert sh.check_map(mi, mj, poses, hp, recs, max_pairs=4)["equal"] is False
