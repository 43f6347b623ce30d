"""Host-side (Python) profile of the bench's frame loop in its default
configuration (encoder batch 8, 8 frames ahead, decode-ahead, main chain on
a high-priority stream): cProfile over `--steps` tracked frames, top
functions by own time and by cumulative time.

  python -m tools.host_profile [--steps 48]
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
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--kb", type=int, default=8)
    ap.add_argument("--ahead", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    n = 8 + 2 * a.steps
    frames = tum_like_sequence(n + 16, 384, 512, seed=0, step_px=2.0, device=dev)
    fe = Frontend(model, device=dev, spatial_stride=4, render=True, enc_batch=a.kb,
                  enc_ahead=a.ahead, decode_ahead=True, main_priority=-1)
    look = a.kb + a.ahead
    nxt = lambda i: [frames[j] for j in range(i + 1, i + 1 + look)]
    for i in range(8 + a.steps):
        fe.step(i, frames[i], next_img=nxt(i))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(8 + a.steps, n):
        fe.step(i, frames[i], next_img=nxt(i))
    torch.cuda.synchronize()
    pr.disable()
    print(f"{(time.perf_counter() - t0) / a.steps * 1e3:.2f} ms/frame under cProfile")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
