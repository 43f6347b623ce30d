"""gaussians_to_world device time (s3w_gaussians_to_world through
splatt3r_utils.world_records) on a 512x384 view whose depths cluster like a
real scene (z = 2 + 0.3 N(0, 1)): the tracker's stride-4 view (two-launch
path, k_g2w_select) and stride 1 (multi-pass path).  HIP events around 50
calls on torch's current stream.  python -m tools.bench_g2w"""
from __future__ import annotations

import json

import torch

from splatt3r_amd.splatt3r_utils import world_records


def view(H=384, W=512, seed=0, dev="cuda"):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(H, W, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    means = torch.randn(H, W, 3, generator=g) * 0.5
    means[..., 2] = 2.0 + 0.3 * torch.randn(H, W, generator=g)
    p = dict(means=means, scales=torch.exp(torch.randn(H, W, 3, generator=g) - 2.5), rotations=q,
             sh=torch.randn(H, W, 3, 1, generator=g) * 0.3,
             opacities=torch.rand(H, W, 1, generator=g), conf=1 + torch.rand(H, W, generator=g) * 2)
    img = torch.rand(3, H, W, generator=g) * 2.2 - 1.1
    return {k: v.to(dev) for k, v in p.items()}, img.to(dev)


def main(iters=50):
    v, img = view()
    T = torch.eye(4, device="cuda")
    out = {}
    for stride in (4, 1):
        fn = lambda: world_records(v, img, T, stride, 0.05, 0.98, 1.0, 1.5)
        for _ in range(5):
            rec, cnt = fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            rec, cnt = fn()
        e1.record()
        torch.cuda.synchronize()
        out[f"stride{stride}_us"] = e0.elapsed_time(e1) * 1e3 / iters
        out[f"stride{stride}_count"] = int(cnt.item())
        out[f"stride{stride}_checksum"] = float(rec[:int(cnt.item())].double().sum().item())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
