"""Harness I/O in the FPS window (splatt3r_amd/dataio.py): TUM-layout
dataset reading (dataloader.py:18-78), the frame loader (create_frame's
resize_img + ImgNorm + H2D on worker threads, frame.py:122-133) and the
per-frame render PNG writer (main.py:436-446, 490-506)."""
import os

import numpy as np
import pytest
import torch


def test_tum_dataset_reads_synthetic_layout(tmp_path):
    from splatt3r_amd.dataio import TUMDataset, write_synthetic_tum
    root = write_synthetic_tum(tmp_path / "seq", 4, seed=1)
    ds = TUMDataset(root)
    assert len(ds) == 4
    t, img = ds[2]
    assert img.shape == (480, 640, 3) and img.dtype == np.float32
    assert 0.0 <= img.min() and img.max() <= 1.0
    assert np.all(np.diff(ds.timestamps) > 0)
    # dataloader.py:50: uint8 / 255.0
    assert np.array_equal(np.round(img * 255).astype(np.uint8), (img * 255).round().astype(np.uint8))
    assert TUMDataset(root, subsample=2).rgb_files == ds.rgb_files[::2]


def test_render_to_uint8_truncates_like_the_reference():
    from splatt3r_amd.dataio import render_to_uint8
    x = np.array([[[-0.5, 0.0, 0.999], [0.5, 1.0, 2.0]]], np.float32)
    # main.py:441-444: (clamp(0, 1) * 255).astype("uint8")
    np.testing.assert_array_equal(render_to_uint8(x),
                                  (np.clip(x, 0, 1) * 255).astype(np.uint8))
    assert render_to_uint8(x)[0, 0, 2] == 254      # truncation, not rounding


@pytest.mark.gpu
def test_frame_loader_matches_create_frame(tmp_path):
    from splatt3r_amd.dataio import FrameLoader, TUMDataset, write_synthetic_tum
    from splatt3r_amd.frame import create_frame
    root = write_synthetic_tum(tmp_path / "seq", 6, seed=2)
    ds = TUMDataset(root)
    loader = FrameLoader(ds, "cuda", workers=3, depth=4)
    for i, lf in enumerate(loader):
        assert lf.index == i
        img = lf.consume()
        ref = create_frame(i, ds[i][1], device="cuda")
        assert torch.equal(img, ref.img)
        assert lf.true_shape.tolist() == [[384, 512]]
    loader.close()


@pytest.mark.gpu
def test_render_writer_png_bytes(tmp_path):
    from PIL import Image
    from splatt3r_amd.dataio import RenderWriter, render_to_uint8
    g = torch.Generator(device="cuda").manual_seed(0)
    w = RenderWriter(tmp_path / "r", workers=2, ring=3)
    imgs = [torch.rand(1, 1, 3, 40, 56, device="cuda", generator=g) * 1.2 - 0.1 for _ in range(7)]
    for i, im in enumerate(imgs):
        w.submit(i, im, "gs_track" if i else "gs_init")
    w.close()
    assert w.written == 7
    for i, im in enumerate(imgs):
        name = f"{'gs_track' if i else 'gs_init'}_{i:06d}.png"
        got = np.asarray(Image.open(tmp_path / "r" / name))
        want = render_to_uint8(im[0, 0].permute(1, 2, 0).cpu().numpy())
        np.testing.assert_array_equal(got, want)
