"""The frontend of the SLAM loop: main.py:395-535 (one call of `step` = one
frame of the reference's `while True` body).  The backend (main.py:76-190)
is optional (`backend=backend.Backend(...)`): keyframe tasks run inline or
on a worker thread/stream, RELOC frames go through its retrieval-based
relocalization; its pair batches shard across GPUs (splatt3r_amd/pairs.py).
With `viz=True` the world map the viz process renders is kept on the device
(gaussian_map.SharedGaussians); the GUI itself is out of scope.

Per tracked frame this runs, as the reference does with --no-viz and
rendering on (the default):
  tracker.track                 encoder(frame) + fused decoder/heads vs the
                                last keyframe + dense matching + GN pose
  gaussians_to_world            when should_append_gaussians says so
  splatt3r_render               2*h*w splats into the frame's view, read
                                back to host (the reference writes a PNG)

Software pipelining: when the caller passes the next frame's image
(`step(i, img, next_img=...)`, as the reference's loop could with
dataset[i + 1]), the encoder of frame i + 1 is queued on a side HIP stream
before frame i's decoder, matching, GN and render are queued on the main
stream, so the two chains share the chip (the 768-token GEMMs fill only a
part of the 256 CUs) and the encoder also fills the host-sync gaps of the
tracker.  With a lookahead list (`next_img=[img_{i+1}, img_{i+2}, ...]`)
and `enc_batch=k`, frames i+1..i+k are encoded as one image batch when
frame i+1 is not queued yet (dataset playback; a live camera uses k = 1):
the encoder is per-image (no op mixes images), so every frame is still
encoded exactly once from its own image, with M = 768k-row GEMMs.
"""
from __future__ import annotations

import contextlib
import os
import queue
import threading
import time
import types

import torch

import lietorch
from splatt3r_amd import _lib
from splatt3r_amd.config import config
from splatt3r_amd.frame import Frame, Keyframes, Mode, create_frame
from splatt3r_amd.gaussian_map import SharedGaussians, should_append_gaussians
from splatt3r_amd.splatt3r_utils import (RasterSizing, _sim3_to_4x4, splatt3r_inference_mono,
                                         splatt3r_render, world_records)
from splatt3r_amd.tracker import FrameTracker

__all__ = ["Frontend", "should_append_gaussians", "lookahead_batches"]


def _shared_stream(device, priority, role):
    """One HIP stream per (device, priority, role) for the whole process:
    Frontends created one after another (bench legs, tests) reuse the same
    streams instead of creating two or three more each; every new stream is
    mapped onto one of the process's few hardware queues (GPU_MAX_HW_QUEUES),
    and a frontend whose streams came late in that assignment ran its
    frames ~1.6x slower (tools/live_ab.py, profiles/r04k_live_ab_before.log / _after.log).  The
    streams are the library's dedicated ones (_lib.frame_stream: created in
    a fixed order, each on a hardware queue of its own), not torch's pool."""
    return _lib.frame_stream(device, role, int(priority))


def _clear_ahead_slot(model):
    enc = getattr(model, "encoder", None)
    if enc is not None and getattr(enc, "_ahead_slot", None) is not None:
        enc._ahead_slot = None


def lookahead_batches(i: int, next_enc: int, n_next: int, enc_batch: int, enc_ahead=None):
    """The encoder batches frame i queues: [(first frame, count)].

    `next_enc` is the lowest frame index not yet queued, `n_next` the number
    of lookahead images handed to the step (frames i + 1 .. i + n_next).
    Frames are queued in batches of at most `enc_batch` until every frame up
    to i + enc_ahead (None: i + 1) is queued; the last batch is partial when
    fewer images are available.  Pure host logic: Frontend._step and the
    bench's timed-region plan (bench.py plan_encodes) share it."""
    kb = max(1, int(enc_batch))
    want = i + max(1, enc_ahead or 1)
    out = []
    while next_enc <= want:
        off = next_enc - (i + 1)
        c = min(kb, n_next - off)
        if off < 0 or c <= 0:
            break
        out.append((next_enc, c))
        next_enc += c
    return out



# diagnostic only (timeline A/B): S3_DIAG_SKIP="world,render" leaves the
# speculative world records / render out of the tracked frame
_DIAG_SKIP = set(filter(None, os.environ.get("S3_DIAG_SKIP", "").split(",")))

class _RenderTicket:
    """A render queued on the render worker: `keep(finish)` hands the image
    to `finish` (run on the worker, on its stream), `drop()` discards it.
    Every ticket gets exactly one decision; the worker waits for it."""

    def __init__(self):
        self.decided = threading.Event()
        self.finish = None
        self.done = threading.Event()

    def keep(self, finish):
        self.finish = finish
        self.decided.set()

    def drop(self):
        self.decided.set()


class _RenderWorker:
    """splatt3r_render off the tracking thread, on its own HIP stream.

    The rasterizer sizes its binning buffers from num_rendered, a host read
    (diff_gaussian_rasterization forward): on the tracking thread that read
    drained the main stream every frame and the host then issued the rest of
    the frame while the GPU idled (`profiles/r03k_timeline.txt`, 11 % idle in
    host-issue gaps; `profiles/r03l_host_profile.log`: 4.6 ms per frame of the
    tracking thread's 6.7 spent inside that forward).  Here the tracking
    thread records an event and queues the render; the worker's stream waits
    on the event, renders (the same kernels, so the same image bit for bit),
    waits for the tracker's keep / drop decision and then runs the frame's
    PNG write / read-back on its stream.  ctypes releases the GIL during the
    library's blocking calls, so the tracking thread keeps issuing the next
    frame meanwhile.  One daemon thread, FIFO: renders finish in frame order.
    Measured (profiles/r03m_ab.log, bench device path, one box): 152.6 /
    163.1 frames/s with the worker vs 167.0 / 167.6 inline -- the GPU was not
    idle during the tracking thread's wait, and the worker's Python competes
    for the GIL -- so it is opt-in (Frontend(render_async=True))."""

    DECISION_TIMEOUT_S = 60.0

    def __init__(self, device):
        self.stream = _shared_stream(device, 0, "render")
        self.q: queue.Queue = queue.Queue()
        self.error = None
        self.timeouts = 0          # renders dropped for want of a decision (drain raises)
        self.thread = threading.Thread(target=self._loop, name="s3-render", daemon=True)
        self.thread.start()

    def close(self):
        """Stop the worker thread after the queued renders."""
        self.q.put(None)
        self.thread.join()

    def _loop(self):
        while True:
            task = self.q.get()
            if task is None:
                return
            ev, fn, ticket = task
            try:
                with torch.cuda.stream(self.stream):
                    self.stream.wait_event(ev)
                    img = fn()
                    # the tracker decides right after its GN sync; a decision
                    # that never comes (an exception on the tracking thread)
                    # drops the render instead of blocking the queue, and is
                    # counted (Frontend.drain raises)
                    if not ticket.decided.wait(self.DECISION_TIMEOUT_S):
                        img = None
                        self.timeouts += 1
                    if ticket.finish is not None and img is not None:
                        ticket.finish(img)
            except BaseException as e:          # surfaced by drain()
                self.error = e
            finally:
                ticket.done.set()

    def submit(self, fn, tensors) -> _RenderTicket:
        ev = torch.cuda.Event()
        ev.record()                          # the tracking thread's stream position
        for t in tensors:                    # read on the worker stream: keep the blocks
            t.record_stream(self.stream)
        ticket = _RenderTicket()
        self.q.put((ev, fn, ticket))
        return ticket


class Frontend:
    _INFO_RING = 16
    _RB_RING = 4               # pinned read-back buffers of delivered renders
    def __init__(self, model, device="cuda", K=None, spatial_stride=4, render=True,
                 depth_max_percentile=0.98, max_scale=1.0, min_confidence=1.5,
                 readback=True, enc_batch=1, main_priority=None, late_prefetch=False,
                 viz=False, max_gaussians=4 * 1024 * 1024, backend=None, render_writer=None,
                 decode_ahead=False, enc_ahead=None, render_async=False, deferred_render=True):
        self.model = model
        # dataio.RenderWriter: the per-frame gs_init_* / gs_track_* PNG export
        # (main.py:436-446, 490-506), written off the tracking thread
        self.render_writer = render_writer
        # viz: the reference's enable_gs_viz (main.py:357, `not --no-viz`).
        # Only then does it record the last append (main.py:434-435,488-489);
        # under --no-viz last_gs_append_T_WC stays None, so should_append is
        # always true and gaussians_to_world runs on every tracked frame.
        self.viz = viz
        # the world map the viz process renders (frame.py:357-463); appended
        # to with opacity > 0.3 (main.py:426-433, 480-487)
        self.gmap = SharedGaussians(max_gaussians=max_gaussians, device=device) if viz else None
        self.map_opacity_threshold = 0.3
        self.device = device
        self.K = K
        self.late_prefetch = late_prefetch
        self.keyframes = Keyframes()
        if config["use_calib"]:
            if K is None:
                raise ValueError("use_calib needs the camera intrinsics K (main.py:310-318)")
            self.keyframes.set_intrinsics(K)   # main.py:314-318
        self.tracker = FrameTracker(model, self.keyframes, device)
        # backend.Backend (main.py:76-190) or None (frontend only, as the
        # headline bench); its factor graph shares this keyframe list
        self.backend = backend
        if backend is not None:
            backend.keyframes = self.keyframes
            backend.factor_graph.frames = self.keyframes
        self.mode = Mode.INIT
        self.render = render
        self.readback = readback
        self.gs_args = dict(include_cross=False, spatial_stride=spatial_stride,
                            depth_max_percentile=depth_max_percentile, max_scale=max_scale,
                            min_confidence=min_confidence)
        self.last_T_WC = None
        self.last_append_T_WC = None
        self.last_append_idx = -(10 ** 9)                       # main.py:341-342
        self.min_translation, self.min_frame_gap = 0.12, 3   # main.py:339-340
        self.new_kf_frames: list[int] = []
        self._gw_count = None   # device count of world records (no-viz path)
        self._stats = dict(frames=0, tracked=0, reloc=0, keyframes=0, gn_iters=0, f16_saturations=0,
                          gaussians_world=0, rendered=0, rerendered=0)
        self._last_render = None
        # host read-back of the render: double-buffered pinned images filled by
        # async D2H copies; `last_render` waits for the copy on access, so the
        # host is not stalled inside the frame (the reference writes the PNG
        # synchronously, main.py:501-506)
        self._rb_bufs = None
        self._rb_events = [None, None]
        self._rb_i = 0
        self._rb_event = None
        self.fps_timer = None
        self.enc_stream = _shared_stream(device, 0, "encoder") if torch.cuda.is_available() else None
        self._queue = {}           # frame index -> (Frame whose encoder is queued, done event)
        self.enc_batch = enc_batch # images per encoder replay when lookahead frames are given
        # frames kept queued ahead of the current one (None: queue the next
        # enc_batch frames only when frame i + 1 is not queued yet)
        self.enc_ahead = enc_ahead
        self._next_enc = 0         # lowest frame index not queued for encoding
        # decode-ahead (splatt3r_utils._decode_ahead): a frame whose decode
        # is issued also decodes the next queued frame against the same
        # keyframe in the same Bp = 2 replay; the result is used when that
        # frame is tracked against the same keyframe
        self.decode_ahead = decode_ahead
        # a decode-ahead slot left on the shared model by an earlier session
        # (frame ids restart, the allocator reuses addresses) is never valid
        # for this one
        _clear_ahead_slot(model)
        # render_async:splatt3r_render + its PNG write / read-back on a
        # worker thread and stream (_RenderWorker); drain() waits for them
        self._rworker = _RenderWorker(device) if render_async and render else None
        # sync-free renders (diff_gaussian_rasterization.rasterize_deferred):
        # the tracked frame's render never waits for the host; each image is
        # delivered (PNG writer / read-back) once its validity flag, copied
        # to the host behind it, shows it fitted the binning capacity
        # (re-rendered with the two-call path otherwise), in frame order
        self.sizing = RasterSizing() if deferred_render else None
        self._info_ring = None     # pinned {status, instances, key bits} mirrors
        self._info_i = 0
        self._pending: list = []
        self._tickets: list = []
        # min(match_frac_k, unique_frac_f) of the frames tracked against the
        # current keyframe, in order: the decode-ahead pairing predictor
        self._kf_fracs: list[float] = []
        # frames tracked / keyframes made at each distance (in frames) from
        # the last keyframe: the predictor's online keyframe-rate estimate
        self._kf_at_dist: dict[int, list[int]] = {}
        self._last_kf_i = 0
        self.spans = None          # list -> per-frame GPU events (encoder, main chain)
        self.wait_log = None       # list -> device time of the waits on encoder batches (diagnostic)
        # main chain on a stream of its own priority (the encoder side stream
        # keeps the default one): the dispatcher then prefers the frame's
        # critical path and the encoder fills the CUs it leaves idle
        self.main_stream = (_shared_stream(device, main_priority, "main")
                            if main_priority is not None and self.enc_stream is not None else None)
        # the no-viz gaussians_to_world records of every tracked frame (the
        # reference computes them and drops them, main.py:467-488) run on a
        # side stream once the pose is known, off the frame's main chain;
        # their consumers (stats, drain) wait for it
        self.aux_stream = _shared_stream(device, 0, "aux") if self.enc_stream is not None else None
        self._aux_used = False
        # the tracked frame's speculative sync-free render on the aux stream
        # too (S3_RENDER_AUX=0: on the main stream, behind the GN chunk)
        self.render_on_aux = (self.aux_stream is not None and self.sizing is not None
                              and os.environ.get("S3_RENDER_AUX", "1") != "0")

    def _prefetch(self, i, imgs):
        """Create frames i, i+1, ... for `imgs` and queue their encoder on
        the side stream as one image batch (one plan replay: the ViT-L
        GEMMs at M = 768 * len(imgs) fill the chip better than one image)."""
        main = torch.cuda.current_stream(self.device)
        frames = [create_frame(i + j, im, None, device=self.device) for j, im in enumerate(imgs)]
        ready = torch.cuda.Event()
        ready.record(main)                       # the image upload / producer
        with torch.cuda.stream(self.enc_stream):
            self.enc_stream.wait_event(ready)
            e0 = self._event()
            img = (frames[0].img if len(frames) == 1
                   else torch.cat([f.img for f in frames], 0))
            feat, pos, _ = self.model.encoder._encode_image(img, frames[0].img_true_shape)
            done = torch.cuda.Event(enable_timing=self.spans is not None)
            done.record(self.enc_stream)
        if self.spans is not None:
            self.spans.append(("enc", i, e0, done))
        # allocated on the side stream, read on the main one
        feat.record_stream(main)
        pos.record_stream(main)
        for j, f in enumerate(frames):
            f.feat, f.pos = feat[j:j + 1], pos[j:j + 1]
            f.img.record_stream(self.enc_stream)
            self._queue[i + j] = (f, done)

    def _pair_mode(self, i):
        """Which decode to pair with frame i's (decode-ahead): "same" --
        frame i + 1 against the current keyframe, used when frame i is NOT
        made a keyframe; "new" -- frame i + 1 against frame i itself, used
        when frame i IS made a keyframe (the next frame is then tracked
        against it, and its decoder inputs are already known: both frames'
        encoder features); None -- decode frame i alone.  Frame i becomes a
        keyframe when its min(match_frac_k, unique_frac_f) falls below
        match_frac_thresh (tracker.py:104-110).  Two estimates: the fraction
        decays as the camera leaves the keyframe, so frame i's is linearly
        extrapolated from the last two frames tracked against the same
        keyframe; and the sequence's own rate of keyframes at frame i's
        distance from the last keyframe (>= 4 samples).  A Bp = 2 replay
        costs ~1.56 Bp = 1 replays (profiles/r03f), so a pairing pays while
        its slot is used with probability > 0.56: "same" below a keyframe
        rate of 0.44 unless the extrapolation says keyframe, "new" above
        0.56, no pairing otherwise (the extrapolation alone, without a rate
        estimate, declines: it guesses keyframes too often to pair on).
        A wrong guess costs speed only, never results."""
        fr = self._kf_fracs
        made, seen = self._kf_at_dist.get(i - self._last_kf_i, (0, 0))
        rate = made / seen if seen >= 4 else None
        if len(fr) >= 2 and 2.0 * fr[-1] - fr[-2] < config["tracking"]["match_frac_thresh"]:
            return "new" if rate is not None and rate > 0.56 else None
        if rate is None or rate < 0.44:
            return "same"
        return "new" if rate > 0.56 else None

    def _ahead_source(self, i, frame):
        """decode-ahead: (the queued Frame i + 1 with its encoder ordered
        before the current stream, the frame to decode it against: None =
        the current keyframe, or Frame i), called only when a decode is
        issued; None when the predictor declines the pairing."""
        def ahead():
            q = self._queue.get(i + 1)
            if q is None:
                return None
            mode = self._pair_mode(i)
            if mode is None:
                self.model.encoder.ahead_counts["declined"] += 1
                return None
            self._wait_enc(q[1], "ahead", i + 1)
            return q[0], (frame if mode == "new" else None)
        return ahead

    def _wait_enc(self, done, what, i):
        """The current stream waits for an encoder batch's completion event;
        with `wait_log` set (diagnostic), timing events bracket the wait on
        the device so the stall it causes can be read afterwards."""
        st = torch.cuda.current_stream(self.device)
        if self.wait_log is None:
            st.wait_event(done)
            return
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        st.wait_event(done)
        e1.record(st)
        self.wait_log.append((what, i, e0, e1))

    def _take_prefetched(self, i, T_WC):
        if i not in self._queue:
            return None
        frame, done = self._queue.pop(i)
        self._wait_enc(done, "frame", i)
        frame.T_WC = T_WC
        return frame

    def drain(self):
        """Wait until every queued render (and its PNG write / read-back) has
        been issued by the render worker (no-op without one)."""
        for t in self._tickets:
            t.done.wait()
        self._tickets = []
        self._aux_join()
        if self._pending:
            # on the stream the renders were issued on (their buffers belong to it)
            st = self.main_stream if self.main_stream is not None else \
                torch.cuda.current_stream(self.device)
            with torch.cuda.stream(st):
                self._deliver(block=True)
        if self._rworker is not None:
            if self._rworker.timeouts:
                n, self._rworker.timeouts = self._rworker.timeouts, 0
                raise RuntimeError(f"{n} render(s) dropped: no keep/drop decision within "
                                   f"{_RenderWorker.DECISION_TIMEOUT_S} s")
            if self._rworker.error is not None:
                e, self._rworker.error = self._rworker.error, None
                raise e

    def close(self):
        """End the session: wait for queued renders, stop the render worker
        thread and release the decode-ahead slot this session left on the
        shared model (its views keep the pair plan's outputs alive)."""
        try:
            self.drain()
        finally:
            if self._rworker is not None:
                self._rworker.close()
                self._rworker = None
            _clear_ahead_slot(self.model)
        self.check_f16_range()

    def check_f16_range(self) -> int:
        """Warn when an fp16 store guard of the network fired (an activation
        beyond +-65504 was saturated instead of becoming inf: a real
        checkpoint whose GELU / fc2 / LayerNorm outputs overflow fp16 would
        otherwise degrade silently).  Reads the device flags (a sync): called
        at close(), never inside step().  Returns the count since the last
        reset (the flags are per process, shared by every frontend)."""
        from . import ops
        n = ops.f16_saturations()
        self._stats["f16_saturations"] = n
        if n:
            import warnings
            warnings.warn(f"splatt3r-slam_amd: {n} fp16 store guard(s) fired: network "
                          f"activations exceeded the fp16 range and were saturated",
                          RuntimeWarning, stacklevel=2)
        return n

    @property
    def last_render(self):
        self.drain()
        if self._rb_event is not None:
            self._rb_event.synchronize()
        return self._last_render

    def _render_task(self, frame, ref, target):
        """splatt3r_render of `frame` at pose `target` (None: its own pose)
        queued on the render worker; returns the ticket."""
        snap = types.SimpleNamespace(gaussian_pred=frame.gaussian_pred,
                                     gaussian_pred_cross=frame.gaussian_pred_cross,
                                     img=frame.img, T_WC=frame.T_WC)
        rsnap = types.SimpleNamespace(img=ref.img)
        tgt = frame.T_WC if target is None else target
        ts = [snap.img, rsnap.img, snap.T_WC.data, tgt.data]
        for g in (snap.gaussian_pred, snap.gaussian_pred_cross):
            if g is not None:
                ts += [v for v in g.values() if torch.is_tensor(v)]
        model, K = self.model, self.K
        t = self._rworker.submit(lambda: splatt3r_render(model, snap, rsnap, K=K, target_T_WC=tgt),
                                 ts)
        self._tickets = [x for x in self._tickets if not x.done.is_set()] + [t]
        return t

    def _render(self, frame, ref, target, prefix="gs_track"):
        if not self.render:
            return
        if self._rworker is not None:
            idx = frame.frame_id
            self._stats["rendered"] += 1
            self._render_task(frame, ref, target).keep(
                lambda img: self._finish_render(img, idx, prefix, count=False))
            return
        self._finish_render(splatt3r_render(self.model, frame, ref, K=self.K, target_T_WC=target,
                                            sizing=self.sizing),
                            frame.frame_id, prefix)

    def _speculate(self, frame, ref):
        """Hook for FrameTracker.track: with the map off, the tracked frame's
        world records and render depend only on its pose, so they are queued
        from the device-side pose of the first GN chunk, ahead of the
        tracker's decision sync; kept when that pose is final and the frame
        is not lost (the common case), recomputed otherwise."""
        def hook(T_WC):
            saved = frame.T_WC
            frame.T_WC = T_WC
            try:
                # the render first: it is on the main stream, right behind
                # the GN chunk; the aux stream's world records after it
                if not self.render or "render" in _DIAG_SKIP:
                    img = None
                elif self._rworker is not None:
                    img = self._render_task(frame, ref, T_WC)      # a ticket
                elif self.render_on_aux and self.sizing.capacity is not None:
                    img = self._render_aux(frame, ref, T_WC)
                else:
                    img = splatt3r_render(self.model, frame, ref, K=self.K, target_T_WC=T_WC,
                                          sizing=self.sizing)
                recs = None if "world" in _DIAG_SKIP else self._world_records_aux(frame)
            finally:
                frame.T_WC = saved
            # earlier frames' finished renders are handed over here, while
            # the host is about to wait for the GN chunk anyway, instead of
            # at the next step's start, where the read-back issue delays the
            # next frame's first launches
            self._deliver(block=False)
            return recs, img
        return hook

    def _render_aux(self, frame, ref, T_WC):
        """The sync-free splatt3r_render on the aux stream, ordered after the
        calling stream's work so far (the pose of the GN chunk, the
        predictions), its inputs kept alive for the aux stream.  The image
        carries its stream (`_s3_stream`): the flag copy, the read-back and
        the PNG writer's copy are ordered after it there."""
        cur = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        ins = [frame.img, ref.img, frame.T_WC.data, T_WC.data]
        for g in (frame.gaussian_pred, frame.gaussian_pred_cross):
            if g is not None:
                ins += [v for v in g.values() if torch.is_tensor(v)]
        with torch.cuda.stream(self.aux_stream):
            self.aux_stream.wait_event(ready)
            img = splatt3r_render(self.model, frame, ref, K=self.K, target_T_WC=T_WC,
                                  sizing=self.sizing)
        for t in ins:
            if t.is_cuda:
                t.record_stream(self.aux_stream)
        if img is not None:
            img._s3_stream = self.aux_stream
        return img

    def _finish_render(self, img, index=0, prefix="gs_track", count=True):
        if img is not None and count:
            self._stats["rendered"] += 1
        src = getattr(img, "_s3_stream", None)   # the aux stream (_render_aux) or None
        chk = getattr(img, "_gsr_check", None)
        if chk is not None:
            # pinned flag mirrors from a fixed ring (a pinned allocation in
            # the frame loop can stall the host for milliseconds); a slot is
            # reused only after its render has been delivered
            if self._info_ring is None:
                self._info_ring = [torch.empty(3, dtype=torch.int64, pin_memory=True)
                                   for _ in range(self._INFO_RING)]
            while len(self._pending) >= self._INFO_RING:
                self._deliver_one(block=True)
            info = self._info_ring[self._info_i]
            self._info_i = (self._info_i + 1) % self._INFO_RING
            # the copy and the event on the frontend device's stream (the
            # Frontend's device need not be the current device)
            st = src if src is not None else torch.cuda.current_stream(self.device)
            with torch.cuda.stream(st):
                info.copy_(chk.info, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
            self._pending.append((img, chk, info, ev, index, prefix))
            return
        ready = None
        if src is not None:
            ready = torch.cuda.Event()
            ready.record(src)
        self._deliver_image(img, index, prefix, ready)

    def _deliver(self, block: bool):
        """Hand the validated sync-free renders to the writer / read-back in
        frame order: each one once its flag copy has landed (without waiting
        for it unless `block`), re-rendered by the two-call path if it did
        not fit."""
        while self._pending:
            if not self._deliver_one(block):
                return

    def reserve_memory(self, large_mb: int = 2048, small_blocks: int = 64):
        """Grow torch's caching allocator on this frontend's streams (call
        once the plans are captured: a graph capture empties the cache).
        The map and keyframe state grow frame after frame; an allocation the
        cache cannot serve is a device allocation inside the frame loop,
        which can hold the host until the device drains (~6-7 ms,
        profiles/r04p_host_steps.log).  A freed large segment is split for
        later large allocations of its stream, and `small_blocks` freed 1 MiB
        blocks keep the small pool (<= 1 MiB requests) from growing."""
        # the aux stream too: the world records and read-backs allocate there
        # (3 small-pool segments grew inside every timed window without it)
        streams = [s for s in (self.enc_stream, self.main_stream, self.aux_stream)
                   if s is not None]
        streams.append(torch.cuda.current_stream(self.device))
        seen = set()
        for st in streams:
            if st.cuda_stream in seen:
                continue
            seen.add(st.cuda_stream)
            with torch.cuda.stream(st):
                big = torch.empty(large_mb << 20, dtype=torch.uint8, device=self.device)
                small = [torch.empty(1 << 20, dtype=torch.uint8, device=self.device)
                         for _ in range(small_blocks)]
                del big, small

    def _readback_slot_free(self) -> bool:
        """Whether the next read-back buffer's previous copy has landed (a
        non-blocking delivery never waits for it: that copy can sit behind
        a whole pair-plan replay on the stream, ~6-7 ms, profiles/r04s)."""
        if self.render_writer is not None or not self.readback or self._rb_events is None:
            return True
        e = self._rb_events[self._rb_i]
        return e is None or e.query()

    def _deliver_one(self, block: bool) -> bool:
        img, chk, info, ev, index, prefix = self._pending[0]
        if not block and (not ev.query() or not self._readback_slot_free()):
            return False
        ev.synchronize()
        self._pending.pop(0)
        status, total, bits = (int(v) for v in info.tolist())
        chk.sizing.update(total, bits)
        if status != 0:
            chk.sizing.rerenders += 1
            self._stats["rerendered"] += 1
            img = chk.rerender()
            ev = None                    # the re-render is newer than ev
        self._deliver_image(img, index, prefix, ev)
        return True

    def _deliver_image(self, img, index, prefix, ready=None):
        """Hand one render over (PNG writer, device tensor or the pinned
        read-back ring).  `ready`: an event recorded after the render on its
        stream (None: recorded here, on the current stream)."""
        if img is not None:
            if self.render_writer is not None:
                if ready is not None:
                    # the writer copies on the current stream
                    torch.cuda.current_stream(self.device).wait_event(ready)
                self.render_writer.submit(index, img, prefix)
                self._last_render, self._rb_event = None, None
                return
            if not self.readback:
                self._last_render, self._rb_event = img[0, 0].clamp(0, 1).permute(1, 2, 0), None
                return
            shape = (img.shape[-2], img.shape[-1], img.shape[-3])
            if self._rb_bufs is None or tuple(self._rb_bufs[0].shape) != shape:
                self._rb_bufs = [torch.empty(shape, dtype=img.dtype, pin_memory=True)
                                 for _ in range(self._RB_RING)]
                self._rb_events = [None] * self._RB_RING
            k = self._rb_i
            self._rb_i = (k + 1) % self._RB_RING
            if self._rb_events[k] is not None:      # copy of _RB_RING renders ago
                self._rb_events[k].synchronize()
            host = self._rb_bufs[k]
            # The read-back runs on the aux stream behind the render only.
            # At step start the main stream holds the next frames' queued
            # work (a decode-ahead pair replay, ~6 ms), and a device-to-host
            # copy issued there was caught holding the host until the stream
            # reached it (one step in 6 runs: the 6 ms idle gap of
            # profiles/r05h_stall_trace.log, stack in _deliver_image).
            st = self.aux_stream if self.aux_stream is not None else torch.cuda.current_stream(
                self.device)
            if ready is None:
                ready = torch.cuda.Event()
                ready.record(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(st):
                st.wait_event(ready)
                # made contiguous on the device first: a device-to-host
                # copy_ from a non-contiguous source goes through a
                # synchronous .to(cpu) inside torch, which held the host until
                # the stream drained (every frame on the aux stream, ~0.25 ms;
                # on the main stream the 6 ms stall of profiles/r05h)
                hwc = img[0, 0].clamp(0, 1).permute(1, 2, 0).contiguous()
                host.copy_(hwc, non_blocking=True)
                img.record_stream(st)
                ev = torch.cuda.Event()
                ev.record(st)
            self._rb_events[k] = ev
            self._last_render, self._rb_event = host, ev

    def _to_world(self, frame, kf_idx):
        if self.gmap is not None:
            # viz on: the world records of gaussians_to_world go straight
            # into the device map (stream-ordered, no host sync)
            a = self.gs_args
            T = _sim3_to_4x4(frame.T_WC)[0].to(frame.img.device)
            pred = frame.gaussian_pred
            total = None
            for b in range(pred["means"].shape[0]):
                view = {k: v[b] for k, v in pred.items()}
                rec, cnt = world_records(view, frame.img[min(b, frame.img.shape[0] - 1)], T,
                                         max(1, int(a["spatial_stride"])), 0.05,
                                         a["depth_max_percentile"], a["max_scale"],
                                         a["min_confidence"])
                self.gmap.append_records(rec, cnt, kf_idx, self.map_opacity_threshold)
                total = cnt if total is None else total + cnt
            # gaussians_to_world returns None when every view's records were
            # filtered out (splatt3r_utils.py:318-319); the caller then does
            # not record the append (main.py:424-435).  One host read of the
            # device count, in viz mode only.
            return True if total is not None and int(total.item()) > 0 else None
        # viz off: the reference computes gaussians_to_world and drops the
        # result (main.py:467-488); the same records are computed here (on
        # the aux stream) and kept on the device with their device count
        # (frame.gs_world), so the tracked frame pays no host sync for the count
        return self._keep_world_records(frame, self._world_records_aux(frame))

    def _world_records_aux(self, frame):
        """_world_records on the aux stream (no-viz path): ordered after the
        calling stream's work so far (the pose, the predictions), inputs kept
        alive for the aux stream, outputs allocated there."""
        if self.aux_stream is None or self.gmap is not None or frame.gaussian_pred is None:
            return self._world_records(frame)
        cur = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        ins = [t for t in frame.gaussian_pred.values() if torch.is_tensor(t)]
        ins += [frame.img, frame.T_WC.data]
        with torch.cuda.stream(self.aux_stream):
            self.aux_stream.wait_event(ready)
            recs = self._world_records(frame)
        for t in ins:
            if t.is_cuda:
                t.record_stream(self.aux_stream)
        self._aux_used = True
        return recs

    def _aux_join(self):
        """The current stream waits for the aux stream's world records."""
        if self._aux_used and self.aux_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.aux_stream)

    def _world_records(self, frame):
        a = self.gs_args
        if frame.gaussian_pred is None:
            return None
        T = _sim3_to_4x4(frame.T_WC)[0].to(frame.img.device)
        pred = frame.gaussian_pred
        recs = []
        for b in range(pred["means"].shape[0]):
            view = {k: v[b] for k, v in pred.items()}
            recs.append(world_records(view, frame.img[min(b, frame.img.shape[0] - 1)], T,
                                      max(1, int(a["spatial_stride"])), 0.05,
                                      a["depth_max_percentile"], a["max_scale"],
                                      a["min_confidence"]))
        return recs

    def _keep_world_records(self, frame, recs):
        if recs is None:
            return None
        # the running count on the stream that produced the records
        on_aux = self._aux_used and self.gmap is None and self.aux_stream is not None
        ctx = torch.cuda.stream(self.aux_stream) if on_aux else contextlib.nullcontext()
        ready = None
        with ctx:
            for _, cnt in recs:
                self._gw_count = cnt.clone() if self._gw_count is None else self._gw_count + cnt
            if on_aux:
                # readers of frame.gs_world wait on this (Frame.gs_world)
                ready = torch.cuda.Event()
                ready.record(self.aux_stream)
        frame.set_gs_world(recs, ready)
        return recs

    @property
    def stats(self) -> dict:
        """Frame counters; `gaussians_world` is read from its device counter
        here (a host sync), never inside step()."""
        if self._gw_count is not None:
            self._aux_join()
            self._stats["gaussians_world"] = int(self._gw_count.item())
        return self._stats

    def _kf_added(self, frame):
        """states.queue_global_optimization (main.py:409, 525-526)."""
        if self.backend is not None:
            idx = len(self.keyframes) - 1
            self.backend.on_keyframe(idx, frame)
            self.backend.queue_global_optimization(idx)

    def _event(self):
        if self.spans is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def step(self, i: int, img, next_img=None) -> Frame:
        if self.main_stream is not None:
            caller = torch.cuda.current_stream(self.device)
            self.main_stream.wait_stream(caller)
            with torch.cuda.stream(self.main_stream):
                frame = self._step_timed(i, img, next_img)
            caller.wait_stream(self.main_stream)
            return frame
        return self._step_timed(i, img, next_img)

    def _step_timed(self, i, img, next_img):
        if self.spans is None:
            return self._step(i, img, next_img)
        e0 = [None]
        frame = self._step(i, img, next_img, e0)
        self.spans.append(("main", i, e0[0], self._event()))
        return frame

    def _step(self, i: int, img, next_img=None, e0=None) -> Frame:
        mark = getattr(self.tracker, "mark", None)     # host-phase recorder (diagnostic)
        if mark:
            mark("step_begin")
        if self.fps_timer is None:
            self.fps_timer = time.time()
        # renders of earlier frames whose validity flags have landed
        self._deliver(block=False)
        if mark:
            mark("delivered")
        # keyframe poses the backend worker has finished optimising
        # (SharedKeyframes' in-place writes, frame.py:269-330)
        self.keyframes.apply_pending()
        T_WC = (lietorch.Sim3.Identity(1, device=self.device) if self.last_T_WC is None
                else self.last_T_WC)
        frame = self._take_prefetched(i, T_WC)
        if frame is None and self.enc_stream is not None:
            # every encode goes through the side stream (one encoder plan,
            # one stream: no two replays of its buffers can overlap)
            self._prefetch(i, [img])
            frame = self._take_prefetched(i, T_WC)
        if frame is None:
            frame = create_frame(i, img, T_WC, device=self.device)
        self._next_enc = max(self._next_enc, i + 1)
        pending = []
        if next_img is not None and self.enc_stream is not None:
            # next_img: the next frame's image, or a list of the next frames'
            # images (lookahead); up to enc_batch of them are encoded together,
            # until frames up to i + enc_ahead are queued
            nxt = list(next_img) if isinstance(next_img, (list, tuple)) else [next_img]
            for s, c in lookahead_batches(i, self._next_enc, len(nxt), self.enc_batch,
                                          self.enc_ahead):
                pending.append((s, nxt[s - (i + 1):s - (i + 1) + c]))
                self._next_enc = s + c
            # late prefetch: a tracked frame queues the next encoder after
            # its GN sync, so the encoder fills the device while the host
            # issues the post-GN launches (pose update, map, render)
            if not (self.late_prefetch and self.mode == Mode.TRACKING):
                for b in pending:
                    self._prefetch(*b)
                pending = []
        if e0 is not None:
            e0[0] = self._event()
        if mark:
            mark("prefetched")
        self._stats["frames"] += 1
        add_new_kf = False
        T_state = frame.T_WC
        if self.mode == Mode.INIT:
            X, C = splatt3r_inference_mono(self.model, frame)
            frame.update_pointmap(X, C)
            self.keyframes.append(frame)
            self.new_kf_frames.append(i)
            self._last_kf_i, self._kf_fracs = i, []
            self._stats["keyframes"] += 1
            self._kf_added(frame)
            self.mode = Mode.TRACKING
            if self._to_world(frame, len(self.keyframes) - 1) is not None and self.viz:
                self.last_append_T_WC, self.last_append_idx = frame.T_WC, i
            self._render(frame, frame, None, prefix="gs_init")
            self.last_T_WC = frame.T_WC
            return frame
        if self.mode == Mode.TRACKING:
            hook = self._speculate(frame, self.keyframes.last_keyframe()) if self.gmap is None \
                else None
            add_new_kf, _, try_reloc = self.tracker.track(
                frame, before_sync=hook,
                ahead=self._ahead_source(i, frame) if self.decode_ahead else None,
                keep_info=False)
            # states.set_frame(frame) (main.py:455): the next frame starts from
            # the tracked pose, not from what the backend later writes into
            # the keyframe (the same object here, a shared-memory copy there)
            T_state = frame.T_WC
            if mark:
                mark("tracked")
            spec = self.tracker.spec if (self.tracker.spec_valid and not try_reloc) else None
            if (spec is None and self.tracker.spec is not None
                    and isinstance(self.tracker.spec[1], _RenderTicket)):
                self.tracker.spec[1].drop()         # speculative render not kept
            for b in pending:
                self._prefetch(*b)
            self._stats["gn_iters"] += self.tracker.last_iters
            self._stats["tracked"] += 1
            if not try_reloc:
                st = self._kf_at_dist.setdefault(i - self._last_kf_i, [0, 0])
                st[0] += int(add_new_kf)
                st[1] += 1
            if try_reloc or add_new_kf:
                self._kf_fracs = []
            else:
                self._kf_fracs.append(min(self.tracker.last_fracs[1:]))
            if try_reloc:
                self.mode = Mode.RELOC
            if not try_reloc and should_append_gaussians(
                    add_new_kf, i, frame.T_WC, self.last_append_T_WC, self.last_append_idx,
                    self.min_translation, self.min_frame_gap):
                if spec is not None:
                    self._keep_world_records(frame, spec[0])
                elif self._to_world(frame, len(self.keyframes)) is not None and self.viz:
                    self.last_append_T_WC, self.last_append_idx = frame.T_WC, i
            if not try_reloc:
                if spec is not None and isinstance(spec[1], _RenderTicket):
                    self._stats["rendered"] += 1
                    spec[1].keep(lambda img, i=i: self._finish_render(img, i, "gs_track",
                                                                      count=False))
                elif spec is not None:
                    self._finish_render(spec[1], i, "gs_track")
                else:
                    self._render(frame, self.keyframes.last_keyframe(), frame.T_WC)
        elif self.mode == Mode.RELOC:
            # main.py:508-517 + relocalization (main.py:76-119): with a
            # backend the frame is matched against the retrieval database and
            # becomes a keyframe only if strict add_factors accepts it;
            # without one the frontend stays in RELOC (no keyframe is made
            # from an unverified pose)
            X, C = splatt3r_inference_mono(self.model, frame)
            frame.update_pointmap(X, C)
            T_state = frame.T_WC                  # states.set_frame (main.py:511)
            self._stats["reloc"] += 1
            if self.backend is not None:
                self.backend.wait()
                if self.backend.relocalization(frame):
                    self._stats["keyframes"] += 1
                    self.new_kf_frames.append(i)
                    self._last_kf_i, self._kf_fracs = i, []
                    self.tracker.reset_idx_f2k()
                    self.mode = Mode.TRACKING
        if add_new_kf:
            self._last_kf_i = i
            self.keyframes.append(frame)
            self.new_kf_frames.append(i)
            self._stats["keyframes"] += 1
            self.tracker.reset_idx_f2k()
            self._kf_added(frame)
        self.last_T_WC = T_state
        if mark:
            mark("step_end")
        return frame
