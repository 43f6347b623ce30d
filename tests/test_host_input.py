"""Host-side input path: resize_img (A1) and checkpoint loading (B4).

resize_img fixture: tests/golden/resize_img.npz, produced by the reference's
own `_resize_pil_image` / `resize_img` function text
(splatt3r_slam/splatt3r_utils.py:646-693, compiled from the file by
oracle/gen_golden.py `resize`; torchvision's ImgNorm restated as
ToTensor + Normalize(0.5, 0.5)).  Bar: bit-exact (uint8 image, true_shape,
transformation tuple); the normalised tensor is ImgNorm of the uint8 image.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

CASES = ((480, 640, 512), (480, 752, 512), (512, 512, 512), (640, 480, 512),
         (540, 960, 512), (300, 400, 512), (480, 640, 224))


def resize_input(h, w, seed):
    """Same recipe as oracle/gen_golden.py resize_input."""
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    img = np.stack([0.45 + 0.45 * np.sin(6 * xx + 4 * yy + k + seed) for k in range(3)], -1)
    iy, ix = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    img += 0.1 * (((ix // 3) + (iy // 3)) % 2)[..., None]
    return np.clip(img, 0, 1).astype(np.float32)


@pytest.mark.parametrize("i", range(len(CASES)))
def test_resize_img_matches_reference_fixture(i):
    from splatt3r_amd.splatt3r_utils import resize_img
    g = np.load(os.path.join(GOLDEN, "resize_img.npz"))
    h, w, size = CASES[i]
    res, tr = resize_img(resize_input(h, w, i), size, return_transformation=True)
    np.testing.assert_array_equal(res["unnormalized_img"], g[f"case{i}_uimg"])
    np.testing.assert_array_equal(res["true_shape"], g[f"case{i}_true_shape"])
    np.testing.assert_array_equal(np.float64(tr), g[f"case{i}_transform"])
    ref_img = (g[f"case{i}_uimg"].astype(np.float32) / 255.0 - 0.5) / 0.5
    np.testing.assert_array_equal(res["img"][0].permute(1, 2, 0).numpy(), ref_img)
    assert res["img"].shape == (1, 3, *g[f"case{i}_true_shape"][0])


def test_create_frame_resizes_by_the_reference_rule():
    from splatt3r_amd.frame import create_frame
    g = np.load(os.path.join(GOLDEN, "resize_img.npz"))
    f = create_frame(3, resize_input(480, 752, 1), device="cpu")
    assert f.img.shape == (1, 3, 320, 512)                       # C4: EuRoC -> 512x320
    assert f.img_true_shape.tolist() == [[320, 512]]
    np.testing.assert_array_equal((f.uimg.numpy() * 255).round().astype(np.uint8),
                                  g["case1_uimg"])


def _small_state_dict():
    from splatt3r_amd import weights as W
    return {n: torch.from_numpy(W.prng_tensor_numpy(1234, n, s))
            for n, s in W.manifest(W.SMALL)}


@pytest.mark.parametrize("fmt", ["lightning", "safetensors"])
def test_load_state_dict_file_weights_only(tmp_path, fmt):
    """The local-checkpoint path (splatt3r_utils.py:43-64): a Lightning ckpt
    (keys under state_dict, prefixed 'encoder.') loaded with
    weights_only=True, or safetensors; tensors come back bit-identical."""
    from splatt3r_amd import weights as W
    sd = _small_state_dict()
    if fmt == "lightning":
        p = tmp_path / "epoch=19-step=1200.ckpt"
        torch.save({"state_dict": {"encoder." + k: v for k, v in sd.items()},
                    "epoch": 19}, p)
    else:
        from safetensors.torch import save_file
        p = tmp_path / "w.safetensors"
        # safetensors refuses shared storage: aliases (layer_rn.N) are copies
        save_file({k: v.clone().contiguous() for k, v in sd.items()}, str(p))
    got = W.load_state_dict_file(str(p), "cpu")
    assert set(got) == set(sd)
    for k, v in sd.items():
        assert torch.equal(got[k], v), k
    W.check_state_dict(W.SMALL, got)


@pytest.mark.gpu
def test_load_splatt3r_from_file_matches_prng_model(tmp_path):
    """load_splatt3r(path) builds the same network as the portable-PRNG
    weights it was saved from: identical encoder features and head outputs."""
    from splatt3r_amd import weights as W
    from splatt3r_amd.net import Splatt3RNet
    from splatt3r_amd.splatt3r_utils import load_splatt3r
    sd = _small_state_dict()
    p = tmp_path / "epoch=19-step=1200.ckpt"
    torch.save({"state_dict": {"encoder." + k: v for k, v in sd.items()}}, p)
    m = load_splatt3r(str(p), cfg=W.SMALL, graphs=False)
    ref = Splatt3RNet(W.SMALL, seed=1234, graphs=False)
    img = torch.rand(1, 3, 48, 64, generator=torch.Generator().manual_seed(0)) * 2 - 1
    fa, pa, _ = m.encoder._encode_image(img.cuda(), None)
    fb, pb, _ = ref._encode_image(img.cuda(), None)
    assert torch.equal(fa, fb) and torch.equal(pa, pb)
    ra, _, _ = m.encoder.infer_pair(fa, pa, fa, pa, (48, 64))
    ra = {k: v.clone() for k, v in ra.items()}
    rb, _, _ = ref.infer_pair(fb, pb, fb, pb, (48, 64))
    for k in ("pts3d", "conf", "desc", "means", "opacities"):
        assert torch.equal(ra[k], rb[k]), k


def test_block_copies_equal_per_tensor_clones():
    """splatt3r_utils._clone_together / _pair_view (the pair plan keeps its
    outputs in blocks so the reference's clones and head stack are one copy
    each): same values as per-tensor clones / torch.stack, fresh storage, and
    the per-tensor fallback when the tensors do not tile one range."""
    import torch
    from splatt3r_amd.splatt3r_utils import _adjacent, _clone_together, _pair_view
    n, widths = 6, {"pts3d": 3, "conf": 1, "desc": 24, "desc_conf": 1}
    blk = torch.randn(2 * n * sum(widths.values()))
    heads, off = [{}, {}], 0
    for k, c in widths.items():
        v = blk[off:off + 2 * n * c].view(2, n * c)
        off += 2 * n * c
        for h in range(2):
            heads[h][k] = v[h].view(1, 2, 3, c) if c > 1 else v[h].view(1, 2, 3)
    assert all(_adjacent(heads[0][k], heads[1][k]) for k in widths)
    out = _clone_together(_pair_view(heads[0][k], heads[1][k]) for k in widths)
    for t, k in zip(out, widths):
        assert torch.equal(t, torch.stack((heads[0][k], heads[1][k])))
        assert t.untyped_storage().data_ptr() != blk.untyped_storage().data_ptr()
    assert len({t.untyped_storage().data_ptr() for t in out}) == 1   # one copy
    g = torch.randn(40)
    gap = [g[0:10], g[20:40]]                                        # not one range
    c = _clone_together(gap)
    assert all(torch.equal(a, b) for a, b in zip(c, gap))
    assert len({t.untyped_storage().data_ptr() for t in c}) == 2
