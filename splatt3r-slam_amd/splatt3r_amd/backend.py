"""The SLAM backend's task bodies (main.py:76-190), in-process.

  Backend.global_optimization(idx)  run_backend's loop body (main.py:142-190):
      consecutive keyframe + retrieval candidates (RetrievalDatabase.update,
      k = 3, min_thresh 5e-3) -> FactorGraph.add_factors -> solve_GN_rays /
      solve_GN_calib
  Backend.relocalization(frame)     relocalization (main.py:76-119): retrieval
      query without adding -> tentative keyframe -> strict add_factors ->
      on success add to the database, copy the pose of the best match and
      solve; on failure pop the keyframe

The reference runs these in a second process sharing the GPU
(config base.yaml single_thread: False) and polls a task queue.  Here the
frontend calls them directly (single_thread) or hands keyframe tasks to a
worker thread that issues them on its own HIP stream (`start_worker`), so
backend kernels run concurrently with the tracker's on the same device.
With a pairs.PairShard over W ranks, keyframe features are broadcast at
keyframe creation and add_factors' pair batches run across the ranks
(ranks 1..W-1 run pairs.serve_backend).  With the worker running, rank 0's
collectives are all issued by the worker thread, in task order: the
frontend's keyframe broadcast is queued as a task ahead of the keyframe's
optimisation, so the frontend thread never blocks on a collective and never
interleaves one with the worker's pair batches (PairShard.lock guards the
remaining frontend-thread tasks: relocalisation, map refresh, stop).  The
worker runs on the CPU too (no streams), for the gloo protocol tests.
"""
from __future__ import annotations

import contextlib
import queue
import threading

import torch

import lietorch
from splatt3r_amd.config import config
from splatt3r_amd.global_opt import FactorGraph


def worker_stream_priority(priority_range=None) -> int:
    """HIP stream priority of the backend worker: the LOWEST the device
    offers (torch numbers priorities so that the range is (lowest, highest),
    e.g. (0, -1)).  The frontend's main chain runs at high priority and its
    encoder at normal; the keyframe tasks then fill what those leave and the
    frontend keeps its frame rate while the queue drains (main.py:122-190
    runs the backend as a separate process that shares the GPU)."""
    lo, _hi = priority_range if priority_range is not None else torch.cuda.Stream.priority_range()
    return int(lo)


class Backend:
    def __init__(self, model, keyframes, K=None, device="cuda", retrieval=None, shard=None):
        from splatt3r_amd.retrieval_database import (RetrievalDatabase,
                                                     synthetic_retrieval_weights)
        self.model = model
        self.keyframes = keyframes
        self.device = torch.device(device)
        self.shard = shard
        self.factor_graph = FactorGraph(model, keyframes, K, device, shard=shard)
        # the retrieval checkpoint is not available offline: synthetic
        # weights of its shapes unless a database is passed in
        self.retrieval = retrieval if retrieval is not None else RetrievalDatabase(
            synthetic_retrieval_weights(self.device), device=self.device)
        self.stats = dict(optimized=0, edges=0, reloc_attempts=0, reloc_success=0,
                          retrieval_candidates=0, last_reloc_candidates=[])
        self._q = None
        self._thread = None
        self._stream = None
        self._err = None

    # ------------------------------------------------------ keyframes ----
    def on_keyframe(self, idx: int, frame):
        """A keyframe was appended on the frontend: broadcast its features to
        the pair-shard ranks (the reference shares them through
        SharedKeyframes' shared memory).  With the worker running the
        broadcast is its next task (issued on the worker thread and stream,
        before the keyframe's optimisation, which is queued after it)."""
        if self.shard is not None and self.shard.ws > 1:
            if self._q is not None:
                self._q.put(("kf", idx, frame, self._ready_event()))
            else:
                self.shard.broadcast_keyframe(idx, frame)

    def _solve(self):
        if config["use_calib"]:
            return self.factor_graph.solve_GN_calib()
        return self.factor_graph.solve_GN_rays()

    def global_optimization(self, idx: int):
        """main.py:142-190 for the queued keyframe idx."""
        kf_idx = [idx - 1 - j for j in range(min(1, idx))]
        frame = self.keyframes[idx]
        retrieval_inds = self.retrieval.update(frame, add_after_query=True,
                                               k=config["retrieval"]["k"],
                                               min_thresh=config["retrieval"]["min_thresh"])
        self.stats["retrieval_candidates"] += len(retrieval_inds)
        kf_idx += retrieval_inds
        kf_idx = set(kf_idx)
        kf_idx.discard(idx)
        kf_idx = list(kf_idx)
        frame_idx = [idx] * len(kf_idx)
        if kf_idx:
            self.factor_graph.add_factors(kf_idx, frame_idx, config["local_opt"]["min_match_frac"])
        self.stats["edges"] = int(self.factor_graph.ii.numel())
        self._solve()
        self.stats["optimized"] += 1

    def relocalization(self, frame) -> bool:
        """main.py:76-119."""
        self.stats["reloc_attempts"] += 1
        kf_idx = list(self.retrieval.update(frame, add_after_query=False,
                                            k=config["retrieval"]["k"],
                                            min_thresh=config["retrieval"]["min_thresh"]))
        self.stats["last_reloc_candidates"] = list(kf_idx)
        success = False
        if kf_idx:
            self.keyframes.append(frame)
            n_kf = len(self.keyframes)
            # synchronous broadcast: relocalisation runs on the calling
            # thread after wait(), and its add_factors needs the keyframe on
            # every rank
            if self.shard is not None and self.shard.ws > 1:
                self.shard.broadcast_keyframe(n_kf - 1, frame)
            frame_idx = [n_kf - 1] * len(kf_idx)
            if self.factor_graph.add_factors(frame_idx, kf_idx, config["reloc"]["min_match_frac"],
                                             is_reloc=config["reloc"]["strict"]):
                self.retrieval.update(frame, add_after_query=True, k=config["retrieval"]["k"],
                                      min_thresh=config["retrieval"]["min_thresh"])
                success = True
                self.keyframes[n_kf - 1].T_WC = lietorch.Sim3(
                    self.keyframes[kf_idx[0]].T_WC.data.clone())
            else:
                self.keyframes.pop_last()
        if success:
            self.stats["reloc_success"] += 1
            self._solve()
        return success

    # ------------------------------------------------------------ map -----
    def refresh_map(self, gmap, spatial_stride: int = 4, depth_max_percentile: float = 0.98,
                    max_scale: float = 1.0, min_confidence: float = 1.5,
                    opacity_threshold: float = 0.3):
        """The global-map refresh after optimisation (north star C5: batched
        re-inference + full-map render): every keyframe of the factor graph
        is re-inferred against its first edge partner -- sharded over the
        ranks (pair p on rank p mod W) -- and its self-prediction becomes
        world Gaussians at its optimised pose with gaussians_to_world's
        filters (splatt3r_utils.py:180-328; the defaults are main.py's map
        arguments); one all-gather rebuilds `gmap` (and every worker's map)
        in keyframe order, the SharedGaussians.append semantics
        (frame.py:388-443, opacity > 0.3).  Call from the frontend thread
        after wait().  Returns the per-keyframe record tensors."""
        from splatt3r_amd.pairs import PairShard
        ii, jj = self.factor_graph.ii.tolist(), self.factor_graph.jj.tolist()
        partner: dict = {}
        for i, j in zip(ii, jj):
            partner.setdefault(i, j)
            partner.setdefault(j, i)
        ks = sorted(partner)
        if not ks:
            gmap.clear()
            return []
        poses = self.keyframes.get_poses().data.reshape(-1, 8)
        if self.shard is not None and self.shard.ws > 1:
            sh = self.shard
        else:
            sh = PairShard(self.model, self.device, local=True)
            for k in ks:
                sh.register_local(k, self.keyframes[k])
        sh.gmap = gmap
        return sh.refresh_map(ks, [partner[k] for k in ks], poses, spatial_stride,
                              depth_max_percentile, max_scale, min_confidence, opacity_threshold)

    # --------------------------------------------------------- worker ----
    def start_worker(self):
        """single_thread: False -- keyframe tasks run on a worker thread and
        its own HIP stream (no stream on the CPU), concurrently with the
        frontend."""
        self._q = queue.Queue()
        if self.device.type == "cuda":
            from splatt3r_amd import _lib
            self._stream = _lib.frame_stream(self.device, "backend", worker_stream_priority())
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    def _ready_event(self):
        """An event after the caller's queued work (None on the CPU)."""
        if self.device.type != "cuda":
            return None
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        return ready

    def _loop(self):
        if self._stream is not None:
            torch.cuda.set_device(self.device)
        while True:
            item = self._q.get()
            if item is None:
                self._q.task_done()
                return
            kind, idx, frame, ready = item
            # keyframe reads on this thread are stream-safe snapshots and pose
            # writes are handed to the frontend's stream (frame.Keyframes);
            # registered per task: the frontend may attach its keyframe list
            # after the worker started
            if self._stream is not None:
                self.keyframes.register_reader(self._stream)
            ctx = (torch.cuda.stream(self._stream) if self._stream is not None
                   else contextlib.nullcontext())
            try:
                with ctx, torch.inference_mode():
                    if ready is not None:
                        self._stream.wait_event(ready)
                    if kind == "kf":
                        if self._stream is not None:
                            for t in (frame.feat, frame.pos, frame.img):
                                t.record_stream(self._stream)
                        self.shard.broadcast_keyframe(idx, frame)
                    else:
                        self.global_optimization(idx)
            except Exception as e:   # surfaced by wait()/stop()
                self._err = e
            self._q.task_done()

    def queue_global_optimization(self, idx: int):
        """states.queue_global_optimization (main.py:409, 526): run now
        (single thread) or hand to the worker."""
        if self._q is None:
            self.global_optimization(idx)
            return
        self._q.put(("opt", idx, None, self._ready_event()))

    def wait(self):
        if self._q is not None:
            self._q.join()
            if self._stream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self._stream)
                self.keyframes.apply_pending(wait=True)
        if self._err is not None:
            e, self._err = self._err, None
            raise e

    def stop(self, stop_shard: bool = True):
        """End the worker; with a shard over W > 1 ranks (stop_shard) also
        release ranks 1..W-1 from serve_backend()."""
        if self._q is not None:
            self._q.put(None)
            self._q.join()
            self._thread.join()
            self._q = None
        if stop_shard and self.shard is not None and self.shard.ws > 1:
            self.shard.stop()
        if self._err is not None:
            e, self._err = self._err, None
            raise e
