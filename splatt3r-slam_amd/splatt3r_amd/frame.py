"""Frame / keyframe containers of the tracking loop (splatt3r_slam/frame.py).

`Frame` keeps the reference's field names and `update_pointmap` filtering
modes (frame.py:45-114) so tracker code reads the same.  The reference's
`SharedKeyframes` (multiprocess shared-memory buffers, frame.py:240-330) is
replaced by `Keyframes`, a single-process list with the same accessors: the
frontend and the pair-batch workers run in one process per GPU here, and the
cross-GPU exchange is an explicit RCCL collective (splatt3r_amd/pairs.py).
"""
from __future__ import annotations

import dataclasses
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
    gs_world: Optional[list] = None   # [(records [n,13], device count)] (slam.py _to_world)

    def __post_init__(self):
        if self.T_WC is None:
            self.T_WC = lietorch.Sim3.Identity(1, device=self.img.device)

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
            m = C > self.C
            self.X_canon[m.repeat(1, 3)] = X[m.repeat(1, 3)]
            self.C[m] = C[m]
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
    """List-backed stand-in for SharedKeyframes (frame.py:240-330)."""

    def __init__(self):
        self._kf: list = []
        self.K: Optional[torch.Tensor] = None

    def __len__(self):
        return len(self._kf)

    def __getitem__(self, i) -> Frame:
        kf = self._kf[i]
        if self.K is not None:
            kf.K = self.K      # frame.py:295 (SharedKeyframes.__getitem__)
        return kf

    def set_intrinsics(self, K: torch.Tensor):
        """frame.py:346-349 (use_calib only)."""
        self.K = K

    def get_intrinsics(self) -> Optional[torch.Tensor]:
        return self.K

    def __setitem__(self, i, frame: Frame):
        self._kf[i] = frame

    def append(self, frame: Frame):
        self._kf.append(frame)

    def pop_last(self):
        self._kf.pop()

    def last_keyframe(self) -> Optional[Frame]:
        return self[len(self._kf) - 1] if self._kf else None

    def get_poses(self) -> lietorch.Sim3:
        return lietorch.Sim3(torch.cat([k.T_WC.data.reshape(1, 8) for k in self._kf]))
