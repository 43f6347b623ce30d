"""The frontend of the SLAM loop: main.py:395-535 (one call of `step` = one
frame of the reference's `while True` body) without the viz/backend
processes, which are out of scope (the tracker path is a
replica per GPU; the pair batches of the backend shard across GPUs in
splatt3r_amd/pairs.py).

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
tracker.  Every frame is still encoded exactly once, from its own image;
the outputs are identical.
"""
from __future__ import annotations

import time

import torch

import lietorch
from splatt3r_amd.frame import Frame, Keyframes, Mode, create_frame
from splatt3r_amd.splatt3r_utils import (gaussians_to_world, splatt3r_inference_mono,
                                         splatt3r_render)
from splatt3r_amd.tracker import FrameTracker


def should_append_gaussians(add_new_kf, frame_idx, current_T_WC, last_append_T_WC,
                            last_append_frame_idx, min_translation, min_frame_gap) -> bool:
    """main.py:54-73."""
    if add_new_kf or last_append_T_WC is None:
        return True
    if frame_idx - last_append_frame_idx < min_frame_gap:
        return False
    t_cur = current_T_WC.matrix()[0, :3, 3]
    t_last = last_append_T_WC.matrix()[0, :3, 3]
    return float(torch.linalg.norm(t_cur - t_last)) >= min_translation


class Frontend:
    def __init__(self, model, device="cuda", K=None, spatial_stride=4, render=True,
                 depth_max_percentile=0.98, max_scale=1.0, min_confidence=1.5,
                 readback=True):
        self.model = model
        self.device = device
        self.K = K
        self.keyframes = Keyframes()
        self.tracker = FrameTracker(model, self.keyframes, device)
        self.mode = Mode.INIT
        self.render = render
        self.readback = readback
        self.gs_args = dict(include_cross=False, spatial_stride=spatial_stride,
                            depth_max_percentile=depth_max_percentile, max_scale=max_scale,
                            min_confidence=min_confidence)
        self.last_T_WC = None
        self.last_append_T_WC = None
        self.last_append_idx = 0
        self.min_translation, self.min_frame_gap = 0.12, 3   # main.py:339-340
        self.new_kf_frames: list[int] = []
        self.stats = dict(frames=0, tracked=0, reloc=0, keyframes=0, gn_iters=0,
                          gaussians_world=0, rendered=0)
        self.last_render = None
        self.fps_timer = None
        self.enc_stream = torch.cuda.Stream(device=device) if torch.cuda.is_available() else None
        self._next = None          # (frame index, Frame whose encoder is queued, done event)

    def _prefetch(self, i, img):
        """Create frame i and queue its encoder on the side stream."""
        main = torch.cuda.current_stream(self.device)
        frame = create_frame(i, img, None, device=self.device)
        ready = torch.cuda.Event()
        ready.record(main)                       # the image upload / producer
        with torch.cuda.stream(self.enc_stream):
            self.enc_stream.wait_event(ready)
            frame.feat, frame.pos, _ = self.model.encoder._encode_image(frame.img,
                                                                         frame.img_true_shape)
            done = torch.cuda.Event()
            done.record(self.enc_stream)
        # allocated on the side stream, read on the main one
        frame.feat.record_stream(main)
        frame.pos.record_stream(main)
        frame.img.record_stream(self.enc_stream)
        self._next = (i, frame, done)

    def _take_prefetched(self, i, T_WC):
        if self._next is None or self._next[0] != i:
            return None
        _, frame, done = self._next
        self._next = None
        torch.cuda.current_stream(self.device).wait_event(done)
        frame.T_WC = T_WC
        return frame

    def _render(self, frame, ref, target):
        if not self.render:
            return
        img = splatt3r_render(self.model, frame, ref, K=self.K, target_T_WC=target)
        if img is not None:
            self.stats["rendered"] += 1
            self.last_render = img[0, 0].clamp(0, 1).permute(1, 2, 0)
            if self.readback:
                self.last_render = self.last_render.cpu()

    def _to_world(self, frame):
        gs = gaussians_to_world(frame, **self.gs_args)
        if gs is not None:
            self.stats["gaussians_world"] += int(gs[0].shape[0])
        return gs

    def step(self, i: int, img, next_img=None) -> Frame:
        if self.fps_timer is None:
            self.fps_timer = time.time()
        T_WC = (lietorch.Sim3.Identity(1, device=self.device) if self.last_T_WC is None
                else self.last_T_WC)
        frame = self._take_prefetched(i, T_WC)
        if frame is None and self.enc_stream is not None:
            # every encode goes through the side stream (one encoder plan,
            # one stream: no two replays of its buffers can overlap)
            self._prefetch(i, img)
            frame = self._take_prefetched(i, T_WC)
        if frame is None:
            frame = create_frame(i, img, T_WC, device=self.device)
        if next_img is not None and self.enc_stream is not None:
            self._prefetch(i + 1, next_img)
        self.stats["frames"] += 1
        add_new_kf = False
        if self.mode == Mode.INIT:
            X, C = splatt3r_inference_mono(self.model, frame)
            frame.update_pointmap(X, C)
            self.keyframes.append(frame)
            self.new_kf_frames.append(i)
            self.stats["keyframes"] += 1
            self.mode = Mode.TRACKING
            self._to_world(frame)
            self.last_append_T_WC, self.last_append_idx = frame.T_WC, i
            self._render(frame, frame, None)
            self.last_T_WC = frame.T_WC
            return frame
        if self.mode == Mode.TRACKING:
            add_new_kf, _, try_reloc = self.tracker.track(frame)
            self.stats["gn_iters"] += self.tracker.last_iters
            self.stats["tracked"] += 1
            if try_reloc:
                self.mode = Mode.RELOC
            if not try_reloc and should_append_gaussians(
                    add_new_kf, i, frame.T_WC, self.last_append_T_WC, self.last_append_idx,
                    self.min_translation, self.min_frame_gap):
                self._to_world(frame)
            if not try_reloc:
                self._render(frame, self.keyframes.last_keyframe(), frame.T_WC)
        elif self.mode == Mode.RELOC:
            # Relocalisation against the retrieval database runs in the
            # backend (main.py:76-127), which is out of scope; the frame is
            # re-initialised as a keyframe at the last pose instead.
            X, C = splatt3r_inference_mono(self.model, frame)
            frame.update_pointmap(X, C)
            self.stats["reloc"] += 1
            add_new_kf = True
            self.mode = Mode.TRACKING
        if add_new_kf:
            self.keyframes.append(frame)
            self.new_kf_frames.append(i)
            self.stats["keyframes"] += 1
            self.tracker.reset_idx_f2k()
        self.last_T_WC = frame.T_WC
        return frame
