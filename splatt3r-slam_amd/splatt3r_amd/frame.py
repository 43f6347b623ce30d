"""Frame / keyframe containers of the tracking loop (splatt3r_slam/frame.py).

`Frame` keeps the reference's field names and `update_pointmap` filtering
modes (frame.py:45-114) so tracker code reads the same.  The reference's
`SharedKeyframes` (multiprocess shared-memory buffers, frame.py:240-330) is
replaced by `Keyframes`, a single-process list with the same accessors: the
frontend and the pair-batch workers run in one process per GPU here, and the
cross-GPU exchange is an explicit RCCL collective (splatt3r_amd/pairs.py).
"""
from __future__ import annotations

import copy
import dataclasses
import threading
from enum import Enum
from typing import Optional

import torch

import lietorch
from splatt3r_amd.config import config


class Mode(Enum):
    INIT = 0
    TRACKING = 1
    RELOC = 2
    TERMINATED = 3


@dataclasses.dataclass
class Frame:
    frame_id: int
    img: torch.Tensor                 # [1,3,H,W] normalised to [-1,1]
    img_shape: torch.Tensor
    img_true_shape: torch.Tensor      # [[H, W]] int32
    uimg: Optional[torch.Tensor] = None
    T_WC: lietorch.Sim3 = None
    X_canon: Optional[torch.Tensor] = None   # [hw,3]
    C: Optional[torch.Tensor] = None         # [hw,1]
    feat: Optional[torch.Tensor] = None      # [1,N,1024]
    pos: Optional[torch.Tensor] = None       # [1,N,2] int64
    N: int = 0
    N_updates: int = 0
    K: Optional[torch.Tensor] = None
    gaussian_pred: Optional[dict] = None
    gaussian_pred_cross: Optional[dict] = None
    # [(records [n,13], device count)] (slam.py _to_world); read through the
    # `gs_world` property, which orders the reader after the producing stream
    _gs_world: Optional[list] = dataclasses.field(default=None, repr=False)
    _gs_world_ready: Optional[object] = dataclasses.field(default=None, repr=False)

    def __post_init__(self):
        if self.T_WC is None:
            self.T_WC = lietorch.Sim3.Identity(1, device=self.img.device)

    @property
    def gs_world(self) -> Optional[list]:
        """The no-viz world records.  They may be produced on the frontend's
        aux stream after step() returns; reading them here makes the caller's
        current stream wait for that producer first (stream-ordered, no host
        sync)."""
        ev = self._gs_world_ready
        if ev is not None and self._gs_world is not None:
            torch.cuda.current_stream(self.img.device).wait_event(ev)
        return self._gs_world

    def set_gs_world(self, recs: Optional[list], ready=None) -> None:
        """Store the records; `ready` is the event recorded on the stream that
        wrote them (None: written on the caller's stream)."""
        self._gs_world = recs
        self._gs_world_ready = ready

    def get_score(self, C):
        mode = config["tracking"]["filtering_score"]
        if mode == "median":
            return torch.median(C)
        if mode == "mean":
            return torch.mean(C)
        raise ValueError(f"unknown filtering_score {mode!r}")

    def update_pointmap(self, X: torch.Tensor, C: torch.Tensor):
        """Fuse a new canonical pointmap estimate (frame.py:53-114)."""
        mode = config["tracking"]["filtering_mode"]
        if self.N == 0:
            self.X_canon, self.C = X.clone(), C.clone()
            self.N = self.N_updates = 1
            if mode == "best_score":
                self.score = self.get_score(C)
            return
        if mode == "first":
            if self.N_updates == 1:
                self.X_canon, self.C, self.N = X.clone(), C.clone(), 1
        elif mode == "recent":
            self.X_canon, self.C, self.N = X.clone(), C.clone(), 1
        elif mode == "best_score":
            s = self.get_score(C)
            if s > self.score:
                self.X_canon, self.C, self.N, self.score = X.clone(), C.clone(), 1, s
        elif mode == "indep_conf":
            # the reference's masked in-place writes (frame.py:80-83) as new
            # tensors: a backend snapshot (Keyframes._snapshot) taken before
            # this update keeps reading the old storage on its own stream
            m = C > self.C
            self.X_canon = torch.where(m, X, self.X_canon)
            self.C = torch.where(m, C, self.C)
            self.N = 1
        elif mode == "weighted_pointmap":
            self.X_canon = (self.C * self.X_canon + C * X) / (self.C + C)
            self.C = self.C + C
            self.N += 1
        elif mode == "weighted_spherical":
            def to_sph(P):
                r = torch.linalg.norm(P, dim=-1, keepdim=True)
                x, y, z = torch.tensor_split(P, 3, dim=-1)
                return torch.cat((r, torch.atan2(y, x), torch.acos(z / r)), -1)

            def to_cart(S):
                r, phi, th = torch.tensor_split(S, 3, dim=-1)
                return torch.cat((r * th.sin() * phi.cos(), r * th.sin() * phi.sin(),
                                  r * th.cos()), -1)

            S = (self.C * to_sph(self.X_canon) + C * to_sph(X)) / (self.C + C)
            self.X_canon = to_cart(S)
            self.C = self.C + C
            self.N += 1
        else:
            raise ValueError(f"unknown filtering_mode {mode!r}")
        self.N_updates += 1

    def get_average_conf(self):
        return self.C / self.N if self.C is not None else None


def create_frame(i, img, T_WC=None, img_size=512, device="cuda:0"):
    """frame.py:122-133.  `img` is either an HxWx3 float array in [0,1]
    (resized by the reference rule, splatt3r_utils.resize_img) or an already
    normalised [1,3,H,W] tensor (the synthetic bench frames)."""
    from splatt3r_amd.splatt3r_utils import resize_img
    if torch.is_tensor(img) and img.dim() == 4:
        rgb = img.to(device)
        H, W = rgb.shape[-2:]
        true_shape = torch.tensor([[H, W]], dtype=torch.int32)
        uimg = None
    else:
        r = resize_img(img, img_size)
        rgb = r["img"].to(device)
        # kept on the host (the reference puts it on the device): it is
        # shape metadata, read by the host glue every frame
        true_shape = torch.tensor(r["true_shape"])
        uimg = torch.from_numpy(r["unnormalized_img"].copy()) / 255.0
    img_shape = true_shape.clone()
    ds = config["dataset"]["img_downsample"]
    if ds > 1:
        if uimg is not None:
            uimg = uimg[::ds, ::ds]
        img_shape = img_shape // ds
    if T_WC is None:
        T_WC = lietorch.Sim3.Identity(1, device=device)
    return Frame(i, rgb, img_shape, true_shape, uimg, T_WC)


class Keyframes:
    """List-backed stand-in for SharedKeyframes (frame.py:240-330).

    The reference shares keyframes between the frontend and the backend
    process through shared-memory buffers guarded by a lock
    (frame.py:269-330): a reader copies out a consistent keyframe, the
    backend writes optimised poses back in place.  Here both sides are
    threads of one process issuing HIP work on different streams, so the
    same contract is kept with stream-ordered handoffs:

      * the owner (frontend) mutates a keyframe under `lock` and publishes
        it (`append` / `__setitem__`), which records a ready event on its
        stream after the producing kernels;
      * a registered reader thread (the backend worker, `register_reader`)
        gets a shallow snapshot from `__getitem__`, taken under the lock: its
        stream waits on the keyframe's ready event, and every tensor it can
        read is `record_stream`-ed onto the reader's stream, so the caching
        allocator cannot hand a block the frontend has since replaced to new
        work while the reader's kernels still read it;
      * poses written by the reader (`set_poses`) are queued with an event on
        the reader's stream and applied by the owner in `apply_pending`
        (start of each frontend step, and `Backend.wait`): the owner's
        stream waits on that event and the new pose tensors are
        `record_stream`-ed onto the owner's stream.
    Single-thread use (no reader registered) is a plain list.
    """

    _SNAP_FIELDS = ("img", "X_canon", "C", "feat", "pos")

    def __init__(self):
        self._kf: list = []
        self.K: Optional[torch.Tensor] = None
        self.lock = threading.RLock()
        self._readers: dict = {}       # thread id -> reader stream
        self._pending: list = []       # [(indices, pose rows [n,8], event)]

    def __len__(self):
        return len(self._kf)

    # ------------------------------------------------ stream handoffs ----
    def register_reader(self, stream):
        """Called on the reader (backend worker) thread with its stream."""
        self._readers[threading.get_ident()] = stream

    def _reader_stream(self):
        return self._readers.get(threading.get_ident()) if self._readers else None

    @staticmethod
    def _ready_event(frame):
        if frame.img is not None and frame.img.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(frame.img.device))
            frame._kf_ready = ev

    def _snapshot(self, kf, stream):
        with self.lock:
            snap = copy.copy(kf)
            ev = getattr(kf, "_kf_ready", None)
        if ev is not None:
            stream.wait_event(ev)
        for name in self._SNAP_FIELDS:
            t = getattr(snap, name)
            if torch.is_tensor(t) and t.is_cuda:
                t.record_stream(stream)
        if snap.T_WC is not None and snap.T_WC.data.is_cuda:
            snap.T_WC.data.record_stream(stream)
        return snap

    def set_poses(self, indices, poses: torch.Tensor):
        """Write keyframe poses [n, 8] (lietorch layout).  From a reader
        thread the write is deferred to the owner's `apply_pending`."""
        stream = self._reader_stream()
        if stream is None:
            with self.lock:
                for r, i in enumerate(indices):
                    self._kf[int(i)].T_WC = lietorch.Sim3(poses[r:r + 1].clone())
            return
        rows = poses.clone()
        ev = torch.cuda.Event()
        ev.record(stream)
        with self.lock:
            self._pending.append(([int(i) for i in indices], rows, ev))

    def apply_pending(self, wait: bool = False) -> int:
        """Owner side: install the reader's finished pose writes (all of them
        when `wait`, else those whose event has completed, in order)."""
        if not self._pending:
            return 0
        done = 0
        with self.lock:
            while self._pending:
                idx, rows, ev = self._pending[0]
                if not wait and not ev.query():
                    break
                self._pending.pop(0)
                cur = torch.cuda.current_stream(rows.device)
                cur.wait_event(ev)
                rows.record_stream(cur)
                for r, i in enumerate(idx):
                    if i < len(self._kf):
                        self._kf[i].T_WC = lietorch.Sim3(rows[r:r + 1])
                        self._ready_event(self._kf[i])
                done += 1
        return done

    # ------------------------------------------------------- accessors ----
    def __getitem__(self, i) -> Frame:
        kf = self._kf[i]
        if self.K is not None:
            kf.K = self.K      # frame.py:295 (SharedKeyframes.__getitem__)
        stream = self._reader_stream()
        if stream is None:
            return kf
        snap = self._snapshot(kf, stream)
        # the reader's own pose writes not yet installed by the owner are
        # what it sees (the reference backend reads back what it wrote)
        i = i % len(self._kf) if isinstance(i, int) else int(i)
        with self.lock:
            for idx, rows, _ in reversed(self._pending):
                if i in idx:
                    snap.T_WC = lietorch.Sim3(rows[idx.index(i):idx.index(i) + 1])
                    break
        return snap

    def set_intrinsics(self, K: torch.Tensor):
        """frame.py:346-349 (use_calib only)."""
        self.K = K

    def get_intrinsics(self) -> Optional[torch.Tensor]:
        return self.K

    def __setitem__(self, i, frame: Frame):
        with self.lock:
            self._kf[i] = frame
            self._ready_event(frame)

    def append(self, frame: Frame):
        with self.lock:
            self._kf.append(frame)
            self._ready_event(frame)

    def pop_last(self):
        with self.lock:
            self._kf.pop()

    def last_keyframe(self) -> Optional[Frame]:
        return self[len(self._kf) - 1] if self._kf else None

    def get_poses(self) -> lietorch.Sim3:
        return lietorch.Sim3(torch.cat([self[i].T_WC.data.reshape(1, 8)
                                        for i in range(len(self._kf))]))
