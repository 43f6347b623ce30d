"""Host-side profile of the per-frame SLAM step (cProfile over bench.py's
frame loop) — where the frame's wall time goes outside GPU kernels.

  python -m tools.profile_frame [--steps 10]
"""
from __future__ import annotations

import argparse
import cProfile
import pstats
import time

import torch

from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    frames = tum_like_sequence(2 * a.steps + 5, 384, 512, seed=0, step_px=2.0, device=dev)
    fe = Frontend(model, device=dev, spatial_stride=4, render=True)
    for i in range(4):
        fe.step(i, frames[i])
    torch.cuda.synchronize()
    # stage wall times with a device sync at every boundary (perturbs the
    # overlap, shows where a frame's time goes)
    import splatt3r_amd.tracker as trk
    import splatt3r_amd.splatt3r_utils as su
    import splatt3r_amd.slam as sl
    acc = {}

    def wrap(mod, name):
        fn = getattr(mod, name)

        def w(*x, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = fn(*x, **k)
            torch.cuda.synchronize()
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
            return r
        setattr(mod, name, w)
        return fn

    orig = {}
    for mod, names in ((su, ["splatt3r_asymmetric_inference", "gaussians_to_world",
                             "splatt3r_render", "_extract_gaussian_params"]),
                       (su.matching, ["match"]),
                       (trk.FrameTracker, ["opt_pose_ray_dist_sim3"]),
                       (sl, ["gaussians_to_world", "splatt3r_render"])):
        for n in names:
            orig[(mod, n)] = wrap(mod, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(4, 4 + a.steps):
        fe.step(i, frames[i])
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"stage-synced frame: {tot:.2f} ms")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"   {k:36s} {v / a.steps * 1e3:8.3f} ms")
    for (mod, n), fn in orig.items():
        setattr(mod, n, fn)

    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(4 + a.steps, 4 + 2 * a.steps):
        fe.step(i, frames[i])
    torch.cuda.synchronize()
    pr.disable()
    print(f"{(time.perf_counter() - t0) / a.steps * 1e3:.2f} ms/frame (under cProfile)")
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
