"""Where does splatt3r_render's time go? (tuning harness)  Runs a few
frontend frames, then times the render glue stage by stage (host wall with a
device sync after each stage) and the whole call unsynced.

  python -m tools.profile_render
"""
from __future__ import annotations

import time

import torch

import diff_gaussian_rasterization as dgr
from splatt3r_amd import render as R
from splatt3r_amd import splatt3r_utils as su
from splatt3r_amd.slam import Frontend
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def main():
    dev = torch.device("cuda", 0)
    model = su.load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    frames = tum_like_sequence(6, 384, 512, seed=0, step_px=2.0, device=dev)
    fe = Frontend(model, device=dev, spatial_stride=4, render=True)
    for i in range(5):
        fe.step(i, frames[i])
    frame, ref = fe.keyframes[len(fe.keyframes) - 1], fe.keyframes[0]
    torch.cuda.synchronize()
    acc = {}

    def wrap(mod, name):
        fn = getattr(mod, name)

        def w(*a, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
            return r
        setattr(mod, name, w)
        return fn

    n = 20
    for _ in range(3):
        su.splatt3r_render(model, frame, ref, target_T_WC=frame.T_WC)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        img = su.splatt3r_render(model, frame, ref, target_T_WC=frame.T_WC)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(n):
        img = su.splatt3r_render(model, frame, ref, target_T_WC=frame.T_WC)
        img[0, 0].clamp(0, 1).permute(1, 2, 0).cpu()
    t2 = time.perf_counter()
    print(f"render unsynced {(t1 - t0) / n * 1e3:.3f} ms/call, with readback "
          f"{(t2 - t1) / n * 1e3:.3f} ms/call")
    orig = [wrap(su, "_sim3_to_4x4"), wrap(su, "camera_settings"), wrap(su, "pack_splats"),
            wrap(dgr._RasterizeGaussians, "apply")]
    t0 = time.perf_counter()
    for _ in range(n):
        su.splatt3r_render(model, frame, ref, target_T_WC=frame.T_WC)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / n * 1e3
    print(f"stage-synced {tot:.3f} ms/call")
    for k, v in acc.items():
        print(f"  {k:24s} {v / n * 1e3:.3f} ms")
    del orig


if __name__ == "__main__":
    main()
