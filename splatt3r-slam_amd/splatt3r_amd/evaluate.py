"""Harness output formats: TUM trajectory, PLY point
cloud, keyframe PNGs — splatt3r_slam/evaluate.py.

Same function names, argument meaning and file bytes as the reference:

* `save_traj` (evaluate.py:23-44): one line per keyframe,
  `"{t} {x} {y} {z} {qx} {qy} {qz} {qw}"` with the Sim3 scale dropped
  (`as_SE3`, lietorch_utils.py:6-13) and each value formatted from its
  float32 the way the reference's f-string formats numpy float32 scalars.
* `save_ply` (evaluate.py:88-106): binary little-endian PLY, vertex element
  `x y z` float + `red green blue` uchar — the header plyfile writes for
  that structured dtype (plyfile is not installed here; the bytes are
  written directly).
* `save_reconstruction` (evaluate.py:47-71): world points `T_WC.act(X_canon)`
  of every keyframe, colours `uint8(uimg * 255)`, kept where the average
  confidence exceeds `c_conf_threshold`.
* `save_keyframes` (evaluate.py:74-85): `{t}.png` per keyframe (PIL instead
  of cv2; cv2's BGR swap followed by its BGR->RGB write is the identity).

save_reconstruction's use_calib branch constrains points to their pixel
rays first (evaluate.py:55-59).  save_traj's `intrinsics` branch calls
`intrinsics.refine_pose_with_calibration(keyframe)` (evaluate.py:42), a
method the reference's Intrinsics class does not define
(dataloader.py:277-317): the reference raises AttributeError there, and so
does this one, with the same exception type.
"""
from __future__ import annotations

import pathlib
from typing import Optional

import numpy as np
import torch

from splatt3r_amd.config import config


def prepare_savedir(args, dataset):
    """evaluate.py:14-20: logs/[save_as]/ and the sequence name."""
    save_dir = pathlib.Path("logs")
    if args.save_as != "default":
        save_dir = save_dir / args.save_as
    save_dir.mkdir(exist_ok=True, parents=True)
    return save_dir, pathlib.Path(dataset.dataset_path).stem


def as_SE3_data(T_WC) -> np.ndarray:
    """lietorch_utils.py:6-13: Sim3 [t, q, s] -> SE3 [t, q] as float32 rows."""
    d = T_WC.data.detach().cpu() if hasattr(T_WC, "data") else torch.as_tensor(T_WC)
    if d.shape[-1] == 7:          # already an SE3 [t, q]
        return d.reshape(-1, 7).numpy().astype(np.float32)
    d = d.reshape(-1, 8)
    return torch.cat([d[:, :3], d[:, 3:7]], -1).numpy().astype(np.float32)


def traj_line(t, pose7: np.ndarray) -> str:
    x, y, z, qx, qy, qz, qw = np.asarray(pose7, np.float32).reshape(-1)
    return f"{t} {x} {y} {z} {qx} {qy} {qz} {qw}\n"


def save_traj(logdir, logfile, timestamps, frames, intrinsics: Optional[object] = None):
    if intrinsics is not None and not hasattr(intrinsics, "refine_pose_with_calibration"):
        raise AttributeError(
            "'Intrinsics' object has no attribute 'refine_pose_with_calibration' "
            "(the reference's save_traj calls a method its Intrinsics does not define, "
            "dataloader.py:277-317)")
    logdir = pathlib.Path(logdir)
    logdir.mkdir(exist_ok=True, parents=True)
    with open(logdir / logfile, "w") as f:
        for i in range(len(frames)):
            kf = frames[i]
            T = kf.T_WC if intrinsics is None else intrinsics.refine_pose_with_calibration(kf)
            f.write(traj_line(timestamps[kf.frame_id], as_SE3_data(T)[0]))


_PLY_HEADER = ("ply\nformat binary_little_endian 1.0\nelement vertex {n}\n"
               "property float x\nproperty float y\nproperty float z\n"
               "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")


def save_ply(filename, points, colors):
    points = np.asarray(points)
    colors = np.asarray(colors).astype(np.uint8)
    pcd = np.empty(len(points), dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                                       ("red", "u1"), ("green", "u1"), ("blue", "u1")])
    pcd["x"], pcd["y"], pcd["z"] = points.T
    pcd["red"], pcd["green"], pcd["blue"] = colors.T
    with open(filename, "wb") as f:
        f.write(_PLY_HEADER.format(n=len(points)).encode("ascii"))
        f.write(pcd.tobytes())


def load_ply(filename):
    """Reader for the files save_ply writes (tests, tooling)."""
    with open(filename, "rb") as f:
        raw = f.read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    n = int(raw[:end].decode().split("element vertex ")[1].split("\n")[0])
    pcd = np.frombuffer(raw[end:], dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                                          ("red", "u1"), ("green", "u1"), ("blue", "u1")], count=n)
    pts = np.stack([pcd["x"], pcd["y"], pcd["z"]], -1)
    col = np.stack([pcd["red"], pcd["green"], pcd["blue"]], -1)
    return pts, col


def save_reconstruction(savedir, filename, keyframes, c_conf_threshold):
    savedir = pathlib.Path(savedir)
    savedir.mkdir(exist_ok=True, parents=True)
    pts, cols = [], []
    for i in range(len(keyframes)):
        kf = keyframes[i]
        if config.get("use_calib", False):
            from splatt3r_amd.geometry import constrain_points_to_ray
            kf.X_canon = constrain_points_to_ray(kf.img_shape.flatten()[:2], kf.X_canon[None],
                                                 kf.K).squeeze(0)
        pW = kf.T_WC.act(kf.X_canon).cpu().numpy().reshape(-1, 3)
        color = (kf.uimg.cpu().numpy() * 255).astype(np.uint8).reshape(-1, 3)
        valid = kf.get_average_conf().cpu().numpy().astype(np.float32).reshape(-1) > c_conf_threshold
        pts.append(pW[valid])
        cols.append(color[valid])
    save_ply(savedir / filename, np.concatenate(pts, 0), np.concatenate(cols, 0))


def save_keyframes(savedir, timestamps, keyframes):
    from PIL import Image
    savedir = pathlib.Path(savedir)
    savedir.mkdir(exist_ok=True, parents=True)
    for i in range(len(keyframes)):
        kf = keyframes[i]
        t = timestamps[kf.frame_id]
        Image.fromarray((kf.uimg.cpu().numpy() * 255).astype(np.uint8)).save(savedir / f"{t}.png")
