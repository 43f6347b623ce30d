"""Dense matching kernels at C2 size (tuning harness): per-kernel HIP-graph
timing of the whole match and of refine_matches alone, per lanes /
load-distance variant, on a smooth synthetic pointmap pair.
python -m tools.bench_match"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, matching
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
    r, dil = int(cfg["radius"]), int(cfg["dilation_max"])
    cfg["radius"] = 0
    us0 = timeit(lambda: matching.match_iterative_proj(X11, X21, D11, D21, cfg=cfg), reps=10)
    print(f"match without refine {us0:7.1f} us -> refine ~{us - us0:7.1f} us", flush=True)
    idx0 = matching.match_iterative_proj(X11, X21, D11, D21, cfg=cfg)[0]
    p1 = torch.stack((idx0 % w, idx0 // w), -1).contiguous()
    D21r = D21.reshape(1, h * w, 24)
    n = h * w
    out = torch.empty_like(p1)

    def plain():
        _lib.call("s3m_refine_matches", D11.data_ptr(), D21r.data_ptr(), p1.data_ptr(),
                  out.data_ptr(), 1, h, w, n, 24, r, dil, _lib.stream())

    L = _lib.lib()
    plain()
    ref = out.clone()
    for lanes, pf in ((1, 3), (16, 3), (1, 2), (1, 4), (1, 6), (2, 2), (2, 3), (2, 4),
                      (4, 2), (4, 3), (1, 3), (16, 3)):
        L.s3m_refine_set_lanes(lanes)
        L.s3m_refine_set_prefetch(pf)
        line = f"refine lanes {lanes:2d} pf {pf}:"
        for name, fn in (("refine", plain),):
            out.fill_(-1)
            fn()
            same = bool(torch.equal(out, ref))
            t = timeit(fn, reps=20)
            line += f"  {name} {t:7.1f} us (same: {same})"
        print(line, flush=True)
    L.s3m_refine_set_lanes(16)
    L.s3m_refine_set_prefetch(4)


if __name__ == "__main__":
    main()
