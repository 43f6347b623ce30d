"""s3n_upsample2x on the frame loop's DPT shapes (Bp = 2 pair replay, 4
groups): per-launch device time with HIP events over 50 launches, and a
checksum (S3_UPSAMPLE_PX=1 vs 2 must print the same).
python -m tools.bench_upsample"""
from __future__ import annotations

import json

import torch

from splatt3r_amd import _lib, ops

# (H, W, C, oh, ow): refinenet 4 -> 1 outputs and the head's 128-channel map
SHAPES = [(12, 16, 256, 24, 32), (24, 32, 256, 48, 64), (48, 64, 256, 96, 128),
          (96, 128, 256, 192, 256), (192, 256, 128, 384, 512)]


def main(B=2, groups=4, iters=50):
    out = {}
    g = torch.Generator(device="cuda").manual_seed(0)
    for H, W, C, oh, ow in SHAPES:
        xs = [torch.randn(B, H, W, C, device="cuda", generator=g).half() for _ in range(groups)]
        ys = [torch.empty(B, oh, ow, C, device="cuda", dtype=torch.float16) for _ in range(groups)]
        call = ops.upsample2x(xs, ys, B=B, H=H, W=W, C=C, oh=oh, ow=ow)
        st = _lib.stream()
        for _ in range(3):
            call(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            call(st)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        nbytes = groups * B * (H * W + oh * ow) * C * 2
        out[f"{H}x{W}x{C}->{oh}x{ow}"] = dict(us=round(us, 2), GBps=round(nbytes / us / 1e3, 1),
                                              sum=float(sum(y.double().sum() for y in ys)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
