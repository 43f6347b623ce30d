"""Shape of the refine's query points on the tracking loop (diagnostic for
the refine kernel design): for every 64-query wave of the tracked frames'
refine_matches calls, the spread of the window-centre rows (v) and columns
(u) before the first dilation level.  python -m tools.refine_stats"""
from __future__ import annotations

import torch

from splatt3r_amd import matching
from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def main():
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    frames = tum_like_sequence(24, 384, 512, seed=0, step_px=2.0, device=dev)
    seen = []
    orig = matching.refine_matches

    def spy(D11, D21, p1, radius, dilation_max):
        seen.append(p1.detach().clone())
        return orig(D11, D21, p1, radius, dilation_max)

    matching.refine_matches = spy
    fe = Frontend(model, device=dev, spatial_stride=4, render=False)
    for i in range(20):
        fe.step(i, frames[i])
    torch.cuda.synchronize()
    matching.refine_matches = orig
    for k, p1 in enumerate(seen[:12]):
        b, n, _ = p1.shape
        g = p1.reshape(b, n // 64, 64, 2)
        vs = (g[..., 1].amax(-1) - g[..., 1].amin(-1)).flatten()
        us = (g[..., 0].amax(-1) - g[..., 0].amin(-1)).flatten()
        q = torch.tensor([0.5, 0.9, 0.99], device=dev)
        print(f"call {k}: b={b} waves={vs.numel()} v-spread==0 {float((vs == 0).float().mean()):.3f}"
              f" <=1 {float((vs <= 1).float().mean()):.3f} <=2 {float((vs <= 2).float().mean()):.3f}"
              f" | v-spread q50/90/99 {torch.quantile(vs.float(), q).tolist()}"
              f" | u-span q50/90/99 {torch.quantile(us.float(), q).tolist()}"
              f" u-span<=97 {float((us <= 97).float().mean()):.3f}", flush=True)


if __name__ == "__main__":
    main()
