"""Generate the golden fixtures under tests/golden/ by importing the Python
reference from /root/reference (this container only; the GPU box never reads
/root/reference).  Committed outputs are data only (inputs + expected
outputs), never reference source.

  python oracle/gen_golden.py [section ...]     sections: matching, net, render

matching : splatt3r_slam/image.py img_gradient (imported) driven exactly as
           splatt3r_slam/matching.py:25-49 prep_for_iter_proj does.
net      : see gen_net() — reduced-size MASt3RGaussians forward with
           portable-PRNG weights (oracle/prng.py).
render   : see gen_render() — rasterizer boundary inputs captured through a
           stub diff_gaussian_rasterization module.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _load_file(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def gen_matching():
    img = _load_file("ref_image", os.path.join(REF, "splatt3r_slam", "image.py"))
    g = torch.Generator().manual_seed(0)
    b, h, w = 2, 12, 16
    X11 = torch.randn(b, h, w, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0])
    X21 = torch.randn(b, h, w, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0])
    # matching.py:25-49
    rays_img = F.normalize(X11, dim=-1).permute(0, 3, 1, 2)
    gx, gy = img.img_gradient(rays_img)
    rays_with_grad = torch.cat((rays_img, gx, gy), dim=1).permute(0, 2, 3, 1).contiguous()
    pts = F.normalize(X21.view(b, -1, 3), dim=-1)
    np.savez_compressed(os.path.join(GOLDEN, "matching_prep.npz"),
                        X11=X11.numpy(), X21=X21.numpy(),
                        rays_with_grad=rays_with_grad.numpy(), pts3d_norm=pts.numpy())
    print("wrote matching_prep.npz")


SECTIONS = {"matching": gen_matching}


def main(argv):
    if not os.path.isdir(REF):
        raise SystemExit("/root/reference not present: fixtures are generated in the build container")
    os.makedirs(GOLDEN, exist_ok=True)
    torch.set_grad_enabled(False)
    for s in (argv or list(SECTIONS)):
        SECTIONS[s]()


if __name__ == "__main__":
    main(sys.argv[1:])
