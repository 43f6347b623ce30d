"""Counter runs of the refine on one captured tracker call (diagnostic):
the default 16-lane kernel in pixel order, then the per-lane kernel in
window-centre tile order, 5 launches each.  Run under rocprofv3 --pmc.
python -m tools.refine_pmc"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, matching
from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def capture(n_frames=8):
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    frames = tum_like_sequence(n_frames + 2, 384, 512, seed=0, step_px=2.0, device=dev)
    seen = []
    orig = matching.refine_matches

    def spy(D11, D21, p1, radius, dilation_max):
        seen.append((D11.clone(), D21.clone(), p1.clone(), radius, dilation_max))
        return orig(D11, D21, p1, radius, dilation_max)

    matching.refine_matches = spy
    fe = Frontend(model, device=dev, spatial_stride=4, render=False)
    for i in range(n_frames):
        fe.step(i, frames[i])
    torch.cuda.synchronize()
    matching.refine_matches = orig
    return seen


def main():
    D11, D21, p1, r, dil = capture()[5]
    b, h, w, f = D11.shape
    n = D21.shape[1]
    out = torch.empty_like(p1)
    L = _lib.lib()
    for lanes, mode in ((16, 0), (1, 0x33), (1, 0)):
        L.s3m_refine_set_lanes(lanes)
        L.s3m_refine_set_sort(mode)
        for _ in range(5):
            _lib.call("s3m_refine_matches", D11.data_ptr(), D21.data_ptr(), p1.data_ptr(),
                      out.data_ptr(), b, h, w, n, f, r, dil, _lib.stream())
        torch.cuda.synchronize()
    L.s3m_refine_set_lanes(-1)
    L.s3m_refine_set_sort(-1)
    print("done", flush=True)


if __name__ == "__main__":
    main()
