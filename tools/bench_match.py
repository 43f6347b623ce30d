"""Dense matching kernels at C2 size (tuning harness): per-kernel HIP-graph
timing of prep / iter_proj / occlusion / refine_matches on a smooth synthetic
pointmap pair.  python -m tools.bench_match"""
from __future__ import annotations

import torch

from splatt3r_amd import matching
from tools.bench_gemm import timeit


def main():
    h, w = 384, 512
    v, u = torch.meshgrid(torch.arange(h, device="cuda"), torch.arange(w, device="cuda"),
                          indexing="ij")
    X11 = torch.stack([(u - w / 2) / w * 2, (v - h / 2) / w * 2, 2 + 0.1 * torch.sin(u / 30.0)],
                      -1)[None].float()
    X21 = torch.roll(X11, 2, dims=2).contiguous()
    D = torch.nn.functional.normalize(torch.randn(1, h, w, 24, device="cuda"), dim=-1)
    D11, D21 = D.half(), torch.roll(D, 2, dims=2).half().contiguous()
    us = timeit(lambda: matching.match(X11, X21, D11, D21), reps=10)
    print(f"match (all kernels) {us:7.1f} us", flush=True)
    cfg = dict(matching.config["matching"])
    cfg["radius"] = 0
    us0 = timeit(lambda: matching.match_iterative_proj(X11, X21, D11, D21, cfg=cfg), reps=10)
    print(f"match without refine {us0:7.1f} us -> refine ~{us - us0:7.1f} us", flush=True)
    import ctypes
    from splatt3r_amd import _lib
    L = _lib.lib()
    L.s3m_refine_set_lanes.argtypes = [ctypes.c_int]
    ref_idx = matching.match(X11, X21, D11, D21)[0].clone()
    for lanes in (8, 16, 32, 64, 8, 16, 32, 64):
        L.s3m_refine_set_lanes(lanes)
        idx = matching.match(X11, X21, D11, D21)[0]
        same = bool(torch.equal(idx, ref_idx))
        us_l = timeit(lambda: matching.match(X11, X21, D11, D21), reps=10)
        print(f"refine lanes {lanes:2d}: match {us_l:7.1f} us -> refine ~{us_l - us0:7.1f} us "
              f"(idx identical: {same})", flush=True)
    L.s3m_refine_set_lanes(16)


if __name__ == "__main__":
    main()
