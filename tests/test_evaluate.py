"""Harness output formats (splatt3r_slam/evaluate.py) — CPU only."""
import types

import numpy as np
import torch

from splatt3r_amd import evaluate as E


def test_ply_header_and_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(37, 3)).astype(np.float32)
    col = rng.integers(0, 256, size=(37, 3)).astype(np.uint8)
    p = tmp_path / "a.ply"
    E.save_ply(p, pts, col)
    raw = p.read_bytes()
    head = raw[: raw.index(b"end_header\n") + 11].decode()
    # the header plyfile writes for evaluate.py:91-105's structured dtype
    assert head == ("ply\nformat binary_little_endian 1.0\nelement vertex 37\n"
                    "property float x\nproperty float y\nproperty float z\n"
                    "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
    assert len(raw) == len(head) + 37 * 15
    P, C = E.load_ply(p)
    np.testing.assert_array_equal(P, pts)
    np.testing.assert_array_equal(C, col)


def test_ply_empty(tmp_path):
    E.save_ply(tmp_path / "e.ply", np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint8))
    P, C = E.load_ply(tmp_path / "e.ply")
    assert P.shape == (0, 3) and C.shape == (0, 3)


def test_traj_lines(tmp_path):
    # Sim3 data [t(3), q(xyzw), s]: scale dropped (lietorch_utils.py:6-13)
    poses = [torch.tensor([[0.1, -2.5, 3.0, 0.0, 0.0, 0.0, 1.0, 1.7]]),
             torch.tensor([[1e-8, 2.0, -0.3333333, 0.5, 0.5, 0.5, 0.5, 0.9]])]
    frames = [types.SimpleNamespace(frame_id=i * 2, T_WC=types.SimpleNamespace(data=poses[i]))
              for i in range(2)]
    ts = [1305031102.175304, 0.5, 1305031102.211214, 7.0]
    E.save_traj(tmp_path, "traj.txt", ts, frames)
    lines = (tmp_path / "traj.txt").read_text().splitlines()
    assert len(lines) == 2
    for ln, fr in zip(lines, frames):
        # evaluate.py:43-44 restated: numpy float32 scalars through an f-string
        x, y, z, qx, qy, qz, qw = fr.T_WC.data[0, :7].numpy().reshape(-1)
        assert ln == f"{ts[fr.frame_id]} {x} {y} {z} {qx} {qy} {qz} {qw}"
    vals = np.array([float(v) for v in lines[0].split()[1:]], np.float32)
    np.testing.assert_array_equal(vals, poses[0][0, :7].numpy())


def test_traj_with_intrinsics_matches_reference_error(tmp_path):
    """evaluate.py:42 calls Intrinsics.refine_pose_with_calibration, which the
    reference's Intrinsics (dataloader.py:277-317) does not define: the
    reference raises AttributeError for any intrinsics object; so do we, and
    an object that does provide the method gets its pose written."""
    import pytest
    poses = torch.tensor([[0.1, -2.5, 3.0, 0.0, 0.0, 0.0, 1.0, 1.7]])
    frames = [types.SimpleNamespace(frame_id=0, T_WC=types.SimpleNamespace(data=poses))]
    with pytest.raises(AttributeError):
        E.save_traj(tmp_path, "t.txt", [0.0], frames, intrinsics=types.SimpleNamespace(K=None))
    refined = types.SimpleNamespace(data=torch.tensor([[1.0, 2.0, 3.0, 0.0, 0.0, 0.0, 1.0]]))
    intr = types.SimpleNamespace(refine_pose_with_calibration=lambda kf: refined)
    E.save_traj(tmp_path, "t.txt", [0.0], frames, intrinsics=intr)
    vals = [float(v) for v in (tmp_path / "t.txt").read_text().split()[1:]]
    assert vals == [1.0, 2.0, 3.0, 0.0, 0.0, 0.0, 1.0]
