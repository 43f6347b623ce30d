"""Rasterizer microbench (BASELINE config 3): P synthetic Gaussians @ 960x540,
forward + backward through the drop-in GaussianRasterizer.

Algorithmic bytes: forward 56 P + 12 H W, backward
120 P + 12 H W.  Timed with HIP events on torch's current stream (the one the
rasterizer launches on).

  python -m tools.bench_raster --P 4194304 --iters 10
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch

from splatt3r_amd.synthetic import identity_camera_settings, raster_grad, raster_microbench_scene


def fwd_bytes(P, H, W):
    return 56 * P + 12 * H * W


def bwd_bytes(P, H, W):
    return 120 * P + 12 * H * W


def prepare(P, device="cuda", seed=0):
    sc = raster_microbench_scene(P, seed=seed)
    rs, scale = identity_camera_settings(sc["K"], sc["H"], sc["W"], device)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    inputs = dict(means3D=t(sc["means"] * scale), opacities=t(sc["opacities"]), shs=t(sc["shs"]),
                  cov3D_precomp=t(sc["cov6"] * scale * scale))
    grad = t(raster_grad(sc["H"], sc["W"], seed=seed + 1))
    return sc, rs, inputs, grad


def run(P=4_194_304, iters=10, warmup=3, backward=True, device="cuda"):
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import GaussianRasterizer, last_timing, set_timing
    sc, rs, inputs, grad = prepare(P, device)
    H, W = sc["H"], sc["W"]
    rast = GaussianRasterizer(rs)
    leaf = {k: v.clone().requires_grad_(backward) for k, v in inputs.items()}

    def step(with_bwd):
        m2 = torch.zeros_like(leaf["means3D"], requires_grad=with_bwd)
        img, radii = rast(means3D=leaf["means3D"], means2D=m2, opacities=leaf["opacities"],
                          shs=leaf["shs"], cov3D_precomp=leaf["cov3D_precomp"])
        if with_bwd:
            (img * grad).sum().backward()
        return img, radii

    for _ in range(warmup):
        step(backward)
    torch.cuda.synchronize()
    # forward only
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    set_timing(True)
    phases = []
    f_ms = []
    for _ in range(iters):
        ev[0].record()
        with torch.no_grad():
            img, radii = step(False)
        ev[1].record()
        torch.cuda.synchronize()
        f_ms.append(ev[0].elapsed_time(ev[1]))
        phases.append(last_timing())
    set_timing(False)
    # the sync-free forward (gsr_forward_deferred: no host read of the
    # instance count between preprocess and binning; the SLAM frame loop's
    # render path), sized from the two-call forward, image checked equal
    cap = int(dgr.last_num_rendered) + 1024
    col, _, info = dgr.rasterize_deferred(rs, leaf["means3D"].detach(), leaf["opacities"].detach(),
                                          shs=leaf["shs"].detach(),
                                          cov3D_precomp=leaf["cov3D_precomp"].detach(),
                                          capacity=cap, key_bits=32)
    kb = int(info[2])
    d_ms = []
    for _ in range(iters):
        ev[0].record()
        col, _, info = dgr.rasterize_deferred(rs, leaf["means3D"].detach(),
                                              leaf["opacities"].detach(), shs=leaf["shs"].detach(),
                                              cov3D_precomp=leaf["cov3D_precomp"].detach(),
                                              capacity=cap, key_bits=kb)
        ev[1].record()
        torch.cuda.synchronize()
        d_ms.append(ev[0].elapsed_time(ev[1]))
    deferred_ok = int(info[0]) == 0 and bool(torch.equal(col, img.detach().reshape(col.shape)))
    b_ms = []
    if backward:
        for _ in range(iters):
            for v in leaf.values():
                v.grad = None
            m2 = torch.zeros_like(leaf["means3D"], requires_grad=True)
            img, radii = rast(means3D=leaf["means3D"], means2D=m2, opacities=leaf["opacities"],
                              shs=leaf["shs"], cov3D_precomp=leaf["cov3D_precomp"])
            loss = (img * grad).sum()
            torch.cuda.synchronize()
            ev[0].record()
            loss.backward()
            ev[1].record()
            torch.cuda.synchronize()
            b_ms.append(ev[0].elapsed_time(ev[1]))
    ph = np.median(np.array(phases), 0).tolist()
    fwd = float(np.median(f_ms))
    out = dict(P=P, H=H, W=W, fwd_ms=fwd, msplats_per_s=P / (fwd * 1e-3) / 1e6,
               fwd_GBps=fwd_bytes(P, H, W) / (fwd * 1e-3) / 1e9,
               phases_ms=dict(zip(["preprocess", "reduce", "depth_sort", "binning", "blend"], ph)),
               num_rendered=int(dgr.last_num_rendered), visible=int((radii > 0).sum()),
               fwd_deferred_ms=float(np.median(d_ms)), deferred_equal=deferred_ok)
    if backward:
        bwd = float(np.median(b_ms))
        out.update(bwd_ms=bwd, bwd_GBps=bwd_bytes(P, H, W) / (bwd * 1e-3) / 1e9)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=4_194_304)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-backward", action="store_true")
    ap.add_argument("--binning", choices=["tile", "global"], default="global",
                    help="forward binning (gsr_set_binning)")
    a = ap.parse_args()
    from splatt3r_amd import _lib
    _lib.lib().gsr_set_binning(1 if a.binning == "tile" else 0)
    t0 = time.time()
    out = run(a.P, a.iters, backward=not a.no_backward)
    out["binning"] = a.binning
    print(json.dumps(out))
    print(f"# wall {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
