"""Per-launch HIP-event profile of the network plans (tuning harness).

  python -m tools.profile_net [--H 384 --W 512 --Bp 1 --reps 5]

Prints one line per distinct launch shape: count, mean us, TFLOP/s, and the
share of the frame's network time."""
from __future__ import annotations

import argparse
from collections import defaultdict

import torch

from splatt3r_amd import weights as W
from splatt3r_amd.net import Splatt3RNet


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=384)
    ap.add_argument("--W", type=int, default=512)
    ap.add_argument("--Bp", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--EB", type=int, default=1, help="encoder batch (frames per encoder replay)")
    a = ap.parse_args()
    net = Splatt3RNet(W.FULL, seed=1234, graphs=False)
    img = torch.rand(a.EB, 3, a.H, a.W, device="cuda") * 2 - 1
    f, p, _ = net._encode_image(img)
    f, p = f[:1], p[:1]
    fb, pb = f.expand(a.Bp, -1, -1).contiguous(), p.expand(a.Bp, -1, -1).contiguous()
    net.infer_pair(fb, pb, fb, pb, (a.H, a.W))
    torch.cuda.synchronize()
    for plan in net.plans():     # warm
        plan.run()
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0, 0])
    for _ in range(a.reps):
        recs = []
        for plan in net.plans():
            recs += plan.run_timed()
        torch.cuda.synchronize()
        for kind, flops, e0, e1, desc in recs:
            d = agg[desc or kind]
            d[0] += 1
            d[1] += e0.elapsed_time(e1) * 1e3
            d[2] += flops
    tot = sum(v[1] for v in agg.values()) / a.reps
    print(f"network total {tot / 1e3:.3f} ms per call set ({a.H}x{a.W}, Bp={a.Bp}, encoder batch {a.EB})")
    print(f"{'launch':48s} {'n':>4s} {'us/launch':>10s} {'TFLOP/s':>8s} {'share':>6s}")
    for desc, (n, us, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        per = us / n
        tf = fl / n / (per * 1e-6) / 1e12 if fl else 0.0
        print(f"{desc:48s} {n // a.reps:4d} {per:10.1f} {tf:8.1f} {us / a.reps / tot:6.1%}")


if __name__ == "__main__":
    main()
