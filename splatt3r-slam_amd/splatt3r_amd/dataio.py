"""Harness input/output around the per-frame path, inside
the reference's FPS window (main.py:363-535):

  TUMDataset      splatt3r_slam/dataloader.py:18-60 (+ TUM rgb.txt parsing,
                  :63-78): dataset[i] -> (timestamp, HxWx3 float32 in [0, 1])
  FrameLoader     dataset[i] -> create_frame's host work (resize_img: PIL
                  LANCZOS 640x480 -> 512x384 + centre crop + ImgNorm,
                  splatt3r_utils.py:658-693, frame.py:122-133) -> pinned
                  buffer -> H2D on a copy stream, on worker threads a few
                  frames ahead of the tracker
  RenderWriter    the per-frame render export (main.py:436-446 `gs_init_*`,
                  :490-506 `gs_track_*`): D2H of the rendered [1,1,3,H,W]
                  image into a pinned ring, then uint8 conversion and the
                  PNG write on writer threads
  write_synthetic_tum  a TUM-layout sequence (rgb/*.png + rgb.txt) of 640x480
                  frames for the benchmark when fr1_desk itself is absent

The reference does all of this synchronously in the tracking loop (its
dataset read, its resize and its cv2.imwrite sit between the GPU calls);
here the host work runs on threads that overlap the GPU, with the same
bytes in and out: the frames the tracker sees are resize_img's output, and
each PNG holds `uint8(clamp(render, 0, 1) * 255)` (truncation, as the
reference's `.astype("uint8")`), in RGB order (cv2 writes the BGR array it
was given, i.e. RGB on disk; PIL writes RGB).  cv2 is not installed here:
PIL does the PNG codec work, at cv2's default compression level 1.
"""
from __future__ import annotations

import concurrent.futures as cf
import pathlib
import queue
import threading
from typing import Optional

import numpy as np
import torch


# ------------------------------------------------------------------ input --
class TUMDataset:
    """TUM RGB-D layout (rgb.txt: "timestamp rgb/<file>.png", '#' comments),
    dataloader.py:18-78: __getitem__ -> (timestamp, img float32 [H,W,3] in
    [0, 1], RGB).  cv2.imread + BGR2RGB in the reference; PIL reads RGB."""

    def __init__(self, root, subsample: int = 1):
        self.root = pathlib.Path(root)
        rows = []
        with open(self.root / "rgb.txt") as f:
            for line in f:
                if line.startswith("#") or not line.strip():
                    continue
                t, path = line.split()[:2]
                rows.append((float(t), self.root / path))
        rows = rows[::subsample]
        self.timestamps = np.array([t for t, _ in rows], dtype=np.float64)
        self.rgb_files = [p for _, p in rows]
        self.img_size = 512
        self.dtype = np.float32

    def __len__(self):
        return len(self.rgb_files)

    def read_img(self, idx) -> np.ndarray:
        from PIL import Image
        with Image.open(self.rgb_files[idx]) as im:
            return np.asarray(im.convert("RGB"))

    def __getitem__(self, idx):
        img = self.read_img(idx)
        return self.timestamps[idx], img.astype(self.dtype) / 255.0


def write_synthetic_tum(root, n: int, H: int = 480, W: int = 640, seed: int = 0,
                        step_px: float = 2.5) -> pathlib.Path:
    """A TUM-layout sequence of n H x W PNG frames panning over a smooth
    multi-scale texture (synthetic.tum_like_sequence's generator at the
    camera's native 640x480, before resize_img)."""
    from PIL import Image
    from splatt3r_amd.synthetic import smooth_texture
    root = pathlib.Path(root)
    (root / "rgb").mkdir(parents=True, exist_ok=True)
    pad = int(np.ceil(step_px * n)) + 8
    tex = smooth_texture(H + pad, W + pad, seed)           # [3, H', W'] in [0, 1]
    lines = ["# color images", "# synthetic TUM-layout sequence", "# timestamp filename"]
    for i in range(n):
        oy = int(round(0.5 * step_px * i)) + 4
        ox = int(round(step_px * i)) + 4
        frame = tex[:, oy:oy + H, ox:ox + W].transpose(1, 2, 0)
        t = 1305031102.175304 + i / 30.0
        name = f"rgb/{t:.6f}.png"
        Image.fromarray(np.round(frame * 255).astype(np.uint8)).save(root / name,
                                                                      compress_level=1)
        lines.append(f"{t:.6f} {name}")
    (root / "rgb.txt").write_text("\n".join(lines) + "\n")
    return root


class LoadedFrame:
    """One frame as create_frame needs it: img [1,3,H,W] on the device
    (ImgNorm), true_shape [[H, W]], the unnormalised uint8 image and the
    copy-stream event after which `img` is valid."""

    __slots__ = ("index", "timestamp", "img", "true_shape", "uimg", "ready")

    def __init__(self, index, timestamp, img, true_shape, uimg, ready):
        self.index, self.timestamp, self.img = index, timestamp, img
        self.true_shape, self.uimg, self.ready = true_shape, uimg, ready

    def consume(self, stream=None):
        """Order `stream` (default: the current one) after the upload and
        tell the allocator the image is used there."""
        s = stream or torch.cuda.current_stream(self.img.device)
        s.wait_event(self.ready)
        self.img.record_stream(s)
        return self.img


class FrameLoader:
    """dataset[i] + create_frame's host work + H2D, `depth` frames ahead of
    the consumer on `workers` threads (PIL releases the GIL in its decode and
    resample loops).  Frames come out in index order: `next()` or
    iteration.  `close()` stops the workers."""

    def __init__(self, dataset, device, img_size: int = 512, workers: int = 3, depth: int = 6,
                 start: int = 0, stop: Optional[int] = None):
        self.ds = dataset
        self.device = torch.device(device)
        self.img_size = img_size
        self.stream = torch.cuda.Stream(device=self.device)
        self._pool = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="s3-load")
        self._next = start
        self._stop = len(dataset) if stop is None else min(stop, len(dataset))
        self._futs: dict = {}
        self._depth = depth
        self._lock = threading.Lock()
        self._fill()

    def _fill(self):
        while len(self._futs) < self._depth:
            i = self._next + len(self._futs)
            if i >= self._stop:
                break
            self._futs[i] = self._pool.submit(self._load, i)

    def _load(self, i) -> LoadedFrame:
        from splatt3r_amd.splatt3r_utils import resize_img
        t, img = self.ds[i]
        r = resize_img(img, self.img_size)
        host = r["img"].pin_memory()
        # one upload stream shared by the workers: the lock keeps each
        # copy + its event together
        with self._lock, torch.cuda.stream(self.stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        # (torch's caching host allocator keeps the pinned block until the
        # non_blocking copy that read it has completed)
        return LoadedFrame(i, t, dev, torch.tensor(r["true_shape"]), r["unnormalized_img"], ev)

    def __len__(self):
        return self._stop

    def __iter__(self):
        return self

    def __next__(self) -> LoadedFrame:
        if self._next >= self._stop:
            raise StopIteration
        f = self._futs.pop(self._next).result()
        self._next += 1
        self._fill()
        return f

    def close(self):
        for f in self._futs.values():
            f.cancel()
        self._pool.shutdown(wait=True)


# ----------------------------------------------------------------- output --
def render_to_uint8(img_hwc: np.ndarray) -> np.ndarray:
    """main.py:441-444 / 501-504: clamp(0, 1) -> * 255 -> astype(uint8)
    (truncating, as numpy's cast)."""
    return (np.clip(img_hwc, 0.0, 1.0) * 255).astype(np.uint8)


class RenderWriter:
    """Per-frame render PNGs (main.py:436-446, 490-506) off the tracking
    thread.  submit() queues an async D2H copy of the [3,H,W] (or
    [1,1,3,H,W]) render into a pinned buffer of a ring of `ring` buffers on
    the current stream; writer threads wait for the copy, convert and write
    `{render_dir}/{prefix}_{i:06d}.png`.  When every buffer is in flight
    submit() waits for the oldest write (back-pressure: the reference writes
    synchronously, this never drops a frame)."""

    def __init__(self, render_dir, workers: int = 3, ring: int = 8, compress_level: int = 1):
        self.dir = pathlib.Path(render_dir)
        self.dir.mkdir(parents=True, exist_ok=True)
        self.compress_level = compress_level
        self._free: "queue.Queue" = queue.Queue()
        self._ring = ring
        self._bufs: list = []
        self._pool = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="s3-png")
        self._pending: list = []
        self._count_lock = threading.Lock()
        self.written = 0

    def _buffer(self, shape):
        if self._bufs and tuple(self._bufs[0].shape) != tuple(shape):
            self.flush()
            self._bufs, self._free = [], queue.Queue()
        if len(self._bufs) < self._ring and self._free.empty():
            b = torch.empty(shape, dtype=torch.float32, pin_memory=True)
            self._bufs.append(b)
            return b
        return self._free.get()

    def submit(self, index: int, img: torch.Tensor, prefix: str = "gs_track"):
        x = img.detach()
        while x.dim() > 3:
            x = x[0]
        x = x.permute(1, 2, 0)                            # [H, W, 3]
        buf = self._buffer(tuple(x.shape))
        buf.copy_(x, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        path = self.dir / f"{prefix}_{index:06d}.png"
        self._pending.append(self._pool.submit(self._write, buf, ev, path))
        self._pending = [f for f in self._pending if not f.done() or f.exception()]

    def _write(self, buf, ev, path):
        from PIL import Image
        try:
            ev.synchronize()
            Image.fromarray(render_to_uint8(buf.numpy())).save(path, compress_level=self.compress_level)
            with self._count_lock:
                self.written += 1
        finally:
            self._free.put(buf)

    def flush(self):
        for f in self._pending:
            f.result()
        self._pending = []

    def close(self):
        self.flush()
        self._pool.shutdown(wait=True)
