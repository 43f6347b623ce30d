"""Cold- vs warm-cache timing of the encoder GEMM shapes (tuning harness).

In a frame every layer's weights are read once (1.5 GB of fp16 weights per
frame cycle through the 256 MiB Infinity Cache), so the network's GEMMs run
with their B operand cold.  This times one launch after evicting the caches
(a 512 MiB write), after a streaming read of B only (an L2/MALL prefetch),
and back to back (warm), for each tile/stage choice.

  python -m tools.bench_gemm_cold
"""
from __future__ import annotations

import statistics

import torch

from splatt3r_amd import _lib, ops

SHAPES = [(768, 1024, 1024), (768, 4096, 1024), (768, 1024, 4096), (768, 3072, 1024)]


def main():
    flush = torch.empty(128 * 1024 * 1024, device="cuda")    # 512 MiB
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def one(c, prep):
        ts = []
        for _ in range(12):
            prep()
            ev[0].record()
            c(_lib.stream())
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
        return statistics.median(ts[2:])

    for M, N, K in SHAPES:
        A = torch.randn(M, K, device="cuda").half()
        B = torch.randn(N, K, device="cuda").half() * K ** -0.5
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        cold = lambda: flush.fill_(1.0)
        pref = lambda: (flush.fill_(1.0), B.view(torch.int32).sum(dtype=torch.int64))
        warm = lambda: None
        for tile in (1, 6, 7, 2, 8, 3, 5):
            for sk in (1, 2):
                c = ops.gemm([A], [B], [C], M, N, K, lda=K, split_k=sk, tile=tile)
                r = [one(c, p) for p in (cold, pref, warm)]
                print(f"{M}x{N}x{K} t{tile}s{sk}: cold {r[0]:6.1f}  prefetched {r[1]:6.1f}"
                      f"  warm {r[2]:6.1f} us", flush=True)
        Bt = B.t()
        r = [one(lambda s: A @ Bt, p) for p in (cold, pref, warm)]
        print(f"{M}x{N}x{K} torch : cold {r[0]:6.1f}  prefetched {r[1]:6.1f}  warm {r[2]:6.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
