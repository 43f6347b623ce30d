"""The sharded backend inside a SLAM run (VERDICT r04 missing 1): rank 0's
Backend with a PairShard on its worker thread, ranks 1..W-1 in
pairs.serve_backend, against the single-thread single-rank backend.

CPU (gloo, world_size 2 and 3): the frontend's side of the protocol
(keyframe appended -> on_keyframe -> queue_global_optimization, then wait /
refresh / stop) with the network, retrieval and GN replaced by deterministic
stand-ins (tests/test_pairs.py fake_match / fake_match_dir, a fixed
retrieval rule, an edge-driven pose update written through
FactorGraph._publish): the worker issues every rank-0 collective in task
order while the 'frontend' thread keeps appending keyframes, and the
factor-graph edges and poses equal the single-thread run exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_pairs import _kf_frames, fake_match, fake_match_dir

N_KF = 9


class _FakeRetrieval:
    """RetrievalDatabase.update stand-in: keyframe k retrieves k - 2 and
    k - 3 (main.py:153-173 adds them to the consecutive edge)."""

    def update(self, frame, add_after_query=True, k=3, min_thresh=0.0):
        i = int(frame.frame_id)
        return [j for j in (i - 2, i - 3) if j >= 0]


def _fake_solve(fg):
    """An edge-driven 'GN step' on the CPU: every keyframe of the graph moves
    by its edge count and the Q mass of its edges, written back through
    FactorGraph._publish (the deferred-pose path on a worker thread)."""
    unique = fg.get_unique_kf_idx()
    if unique.numel() <= 1:
        return
    poses = torch.cat([fg.frames[int(i)].T_WC.data.reshape(1, 8) for i in unique]).clone()
    for r, u in enumerate(unique.tolist()):
        on = (fg.ii == u) | (fg.jj == u)
        qm = float(fg.Q_ii2jj[fg.ii == u].sum() + fg.Q_jj2ii[fg.jj == u].sum())
        vm = float(fg.valid_match_j[fg.ii == u].sum())
        poses[r, 0] += 0.01 * float(on.sum()) + 1e-6 * qm
        poses[r, 1] += 1e-7 * vm
    fg._publish(unique, poses, 1)


def _make_backend(shard):
    from splatt3r_amd.backend import Backend
    from splatt3r_amd.frame import Keyframes

    class _CpuBackend(Backend):
        def _solve(self):
            _fake_solve(self.factor_graph)

    be = _CpuBackend(None, Keyframes(), device="cpu", retrieval=_FakeRetrieval(), shard=shard)
    be.factor_graph.match_fn = fake_match
    return be


def _frames():
    import lietorch
    frames = _kf_frames(N_KF)
    for f in frames:
        f.T_WC = lietorch.Sim3.Identity(1)
    return frames


def _drive(be, worker: bool):
    """The frontend's calls for N_KF keyframes (slam.Frontend._kf_added)."""
    if worker:
        be.start_worker()
    try:
        for k, f in enumerate(_frames()):
            be.keyframes.append(f)
            be.on_keyframe(k, f)
            be.queue_global_optimization(k)
        be.wait()
    finally:
        be.stop()
    fg = be.factor_graph
    poses = torch.cat([be.keyframes[k].T_WC.data.reshape(1, 8) for k in range(N_KF)])
    out = {k: getattr(fg, k).clone().numpy() for k in ("ii", "jj", "idx_ii2jj", "idx_jj2ii",
                                                        "valid_match_j", "valid_match_i",
                                                        "Q_ii2jj", "Q_jj2ii")}
    out["poses"] = poses.numpy()
    out["optimized"] = be.stats["optimized"]
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from splatt3r_amd.pairs import PairShard, serve_backend
        if rank == 0:
            sh = PairShard(None, "cpu", match_fn=fake_match, match_dir_fn=fake_match_dir)
            out = _drive(_make_backend(sh), worker=True)
            out["shard_stats"] = dict(sh.stats)
            q.put((rank, out))
        else:
            sh = serve_backend(None, "cpu", match_dir_fn=fake_match_dir)
            q.put((rank, dict(sh.stats)))
    except Exception as e:       # report instead of leaving the peers blocked
        q.put((rank, f"error: {e!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_backend_worker_matches_single_thread_gloo(ws):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = {}
    try:
        while len(res) < ws:
            r, v = q.get(timeout=180)
            assert not (isinstance(v, str) and v.startswith("error")), (r, v)
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    want = _drive(_make_backend(None), worker=False)          # single thread, single rank
    got = res[0]
    assert got["optimized"] == want["optimized"] == N_KF
    for k in ("ii", "jj", "idx_ii2jj", "idx_jj2ii", "valid_match_j", "valid_match_i",
              "Q_ii2jj", "Q_jj2ii", "poses"):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    assert len(want["ii"]) >= 2 * N_KF - 4
    assert np.abs(want["poses"][:, 0]).max() > 0            # the solves moved the poses
    # every worker rank received every keyframe and ran a share of the
    # directed units (<= 3 pairs per keyframe = <= 6 units: all ranks busy)
    n_units = 2 * sum(1 + len(_FakeRetrieval().update(f)) for f in _frames()[1:])
    assert sum(res[r]["units"] for r in range(1, ws)) + got["shard_stats"]["units"] == n_units
    for r in range(1, ws):
        assert res[r]["keyframes"] == N_KF and res[r]["units"] > 0


def test_keyframe_broadcast_is_a_worker_task():
    """With the worker running, on_keyframe queues the broadcast ahead of the
    keyframe's optimisation instead of issuing a collective on the calling
    (frontend) thread."""
    calls = []

    class _Shard:
        ws, rank = 2, 0

        def broadcast_keyframe(self, idx, frame):
            import threading
            calls.append(("kf", idx, threading.current_thread().name))

        def stop(self):
            calls.append(("stop",))

    be = _make_backend(None)
    be.shard = _Shard()
    be.global_optimization = lambda idx: calls.append(("opt", idx))
    be.start_worker()
    f = _frames()[0]
    be.on_keyframe(0, f)
    be.queue_global_optimization(0)
    be.wait()
    be.stop()
    import threading
    assert calls[0][:2] == ("kf", 0) and calls[0][2] != threading.current_thread().name
    assert calls[1] == ("opt", 0) and calls[-1] == ("stop",)


# ------------------------------------------------------------------ GPU ----
def _slam_run(model, frames, dev, shard, gmap):
    """Frontend + Backend (worker thread, lockstep: the frontend waits for
    each keyframe task, the schedule of single_thread) over the frames, then
    the global-map refresh into gmap."""
    from splatt3r_amd.backend import Backend
    from splatt3r_amd.frame import Keyframes
    from splatt3r_amd.slam import Frontend
    be = Backend(model, Keyframes(), device=dev, shard=shard)
    if shard is not None:
        be.start_worker()
    fe = Frontend(model, device=dev, spatial_stride=4, render=False, backend=be)
    try:
        for i in range(frames.shape[0]):
            fe.step(i, frames[i])
            be.wait()
        be.refresh_map(gmap, opacity_threshold=0.0)
    finally:
        be.stop()
        fe.close()
    torch.cuda.synchronize()
    fg = be.factor_graph
    n = gmap.n_gaussians
    # numpy / python values only: tensors sent through the multiprocessing
    # queue would be shared by file descriptor and vanish with the sender
    np_ = lambda t: t.detach().cpu().numpy()
    return dict(kf=list(fe.new_kf_frames), ii=fg.ii.tolist(), jj=fg.jj.tolist(),
                idx=np_(fg.idx_ii2jj), Q=np_(fg.Q_ii2jj),
                poses=np_(torch.cat([fe.keyframes[k].T_WC.data.reshape(1, 8)
                                     for k in range(len(fe.keyframes))])),
                n=int(n), means=np_(gmap.means[:n]), cov=np_(gmap.cov_triu[:n]),
                opac=np_(gmap.opacities[:n]))


def _gpu_rank(rank, ws, port, q):
    # static GEMM policy in both processes (batch-invariant, no per-process
    # timing choices)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), S3_GEMM_TUNE="0")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from dist_util import init_gpu_group
    dev = init_gpu_group(rank, ws, 300)
    try:
        from splatt3r_amd.gaussian_map import SharedGaussians
        from splatt3r_amd.pairs import PairShard, serve_backend
        from splatt3r_amd.splatt3r_utils import load_splatt3r
        from splatt3r_amd.synthetic import tum_like_sequence
        from splatt3r_amd.weights import FULL
        model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
        if rank > 0:
            sh = serve_backend(model, dev, gmap=SharedGaussians(max_gaussians=1 << 21, device=dev))
            q.put((rank, (int(sh.stats["units"]), int(sh.gmap.n_gaussians))))
            return
        frames = tum_like_sequence(12, 384, 512, seed=3, step_px=4.0, device=dev)
        a = _slam_run(model, frames, dev, PairShard(model, dev),
                      SharedGaussians(max_gaussians=1 << 21, device=dev))
        b = _slam_run(model, frames, dev, None, SharedGaussians(max_gaussians=1 << 21, device=dev))
        q.put((rank, (a, b)))
    except Exception as e:           # report instead of leaving the peer blocked
        q.put((rank, f"error: {e!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_slam_with_sharded_backend_equals_single_rank_on_gpu():
    """A whole SLAM run (Frontend + Backend on its worker thread) with the
    backend's keyframe-pair batches sharded over 2 ranks (gloo, both on the
    one GPU; rank 1 in serve_backend) equals the single-rank single-thread
    run: same keyframes and factor-graph edges, bit-identical match indices,
    Q and keyframe poses, and the same refreshed global map (batch-invariant
    backend plans: the rank split changes no bit)."""
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_rank, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = {}
    try:
        while len(res) < ws:
            r, v = q.get(timeout=600)
            assert not (isinstance(v, str) and v.startswith("error")), (r, v)
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    a, b = res[0]
    units1, n1 = res[1]
    assert len(b["kf"]) >= 3 and a["kf"] == b["kf"]
    assert (a["ii"], a["jj"]) == (b["ii"], b["jj"]) and len(a["ii"]) >= 2
    for k in ("idx", "Q", "poses", "means", "cov", "opac"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert a["n"] == b["n"] == n1 > 0          # rank 1 holds the same map
    assert units1 > 0


def test_backend_worker_stream_is_lowest_priority(monkeypatch):
    """The backend worker's HIP stream takes the lowest priority the device
    offers (torch's range is (lowest, highest)): the frontend's high-priority
    main chain and its encoder keep their rate while keyframe tasks drain.
    It is the library's dedicated "backend" stream (_lib.frame_stream)."""
    from splatt3r_amd import _lib
    from splatt3r_amd import backend as B
    assert B.worker_stream_priority((0, -1)) == 0
    assert B.worker_stream_priority((0, -5)) == 0
    made = []

    class FakeStream:
        @staticmethod
        def priority_range():
            return (0, -3)

    monkeypatch.setattr(B.torch.cuda, "Stream", FakeStream)
    monkeypatch.setattr(B.torch.cuda, "set_device", lambda d: None)
    monkeypatch.setattr(_lib, "_FRAME_STREAMS", {})
    monkeypatch.setattr(_lib, "_FRAME_ORDER", [])
    monkeypatch.setattr(_lib, "_make_stream", lambda dev, prio: made.append(prio) or object())
    be = B.Backend.__new__(B.Backend)          # no retrieval database / factor graph needed
    be.device = torch.device("cuda", 0)
    be._q = be._thread = be._stream = be._err = None
    be.start_worker()
    try:
        assert be._stream is _lib._FRAME_STREAMS[(0, "backend", 0)]
        assert (0, "backend", 0) in _lib._FRAME_ORDER
    finally:
        be._q.put(None)
        be._thread.join(timeout=30)
    assert not be._thread.is_alive()
