"""Encoder plan replay time vs image batch (tuning harness).

  python -m tools.bench_encb
"""
from __future__ import annotations

import torch

from splatt3r_amd import weights as W
from splatt3r_amd.net import Splatt3RNet


def main():
    net = Splatt3RNet(W.FULL, seed=1234, graphs=True)
    for B in (1, 2, 3, 4):
        img = torch.rand(B, 3, 384, 512, device="cuda") * 2 - 1
        for _ in range(3):
            net._encode_image(img)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            net._encode_image(img)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f"encoder B={B}: {ms:.3f} ms/call, {ms / B:.3f} ms/image", flush=True)
    img = torch.rand(1, 3, 384, 512, device="cuda") * 2 - 1
    f, p, _ = net._encode_image(img)
    for Bp in (1, 2):
        fb, pb = f.expand(Bp, -1, -1).contiguous(), p.expand(Bp, -1, -1).contiguous()
        for _ in range(3):
            net.infer_pair(fb, pb, fb, pb, (384, 512))
        pp = net.pair_plan(Bp, 384, 512)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            pp.run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        e0.record()
        for _ in range(n):
            net.infer_pair(fb, pb, fb, pb, (384, 512))
        e1.record()
        torch.cuda.synchronize()
        ms2 = e0.elapsed_time(e1) / n
        print(f"pair plan Bp={Bp}: replay {ms:.3f} ms, infer_pair {ms2:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
