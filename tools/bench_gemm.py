"""A/B timing of s3n_gemm tile / split-K choices on the network's shapes, in
one process, next to torch.matmul (hipBLASLt) on the same fp16 operands as
a calibration of what the box reaches on that shape.

  python -m tools.bench_gemm
"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, ops

SHAPES = [  # (M, N, K, groups, conv)
    (768, 3072, 1024, 1, None), (768, 4096, 1024, 1, None), (768, 1024, 4096, 1, None),
    (768, 1024, 1024, 1, None), (768, 2304, 768, 2, None), (768, 768, 768, 2, None),
    (768, 3072, 768, 2, None), (768, 768, 3072, 2, None), (768, 6400, 7168, 2, None),
    (196608, 128, 1152, 4, (384, 512, 128)), (12288, 256, 2304, 4, (96, 128, 256)),
    (49152, 128, 2304, 4, (192, 256, 256)),
]


def timeit(fn, reps=20):
    """GPU time per call: `reps` calls captured in one HIP graph and replayed
    (no host enqueue gaps between the kernels)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for M, N, K, g, conv in SHAPES:
        A = [torch.randn(M if conv is None else conv[0] * conv[1], K if conv is None else conv[2],
                         device="cuda").half() for _ in range(g)]
        B = [torch.randn(N, K, device="cuda").half() * K ** -0.5 for _ in range(g)]
        C = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(g)]
        cv = None
        if conv is not None:
            cv = dict(H=conv[0], W=conv[1], C=conv[2], k=3, stride=1, pad=1, oH=conv[0],
                      oW=conv[1])
        fl = 2 * M * N * K * g
        res = []
        for tile in (1, 2, 3, 5, 6, 7, 8, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31):
            for sk in (1, 2, 3, 4):
                if conv is not None and sk > 1:
                    continue
                c = ops.gemm(A, B, C, M, N, K, lda=0 if conv else K, conv=cv, split_k=sk, tile=tile)
                us = timeit(lambda: c(_lib.stream()))
                res.append((us, f"t{tile}s{sk}"))
        auto = ops.gemm(A, B, C, M, N, K, lda=0 if conv else K, conv=cv)
        us_auto = timeit(lambda: auto(_lib.stream()))
        line = f"{M}x{N}x{K} g{g}{' conv' if conv else ''}: auto {us_auto:7.1f}us {fl / us_auto / 1e6:6.0f}TF |"
        best = sorted(res)[:4]
        line += " ".join(f" {n} {u:6.1f}" for u, n in best)
        if conv is None:
            Ab = torch.stack(A)
            Bb = torch.stack(B).transpose(1, 2)
            us_t = timeit(lambda: torch.bmm(Ab, Bb))
            line += f" | torch {us_t:6.1f}us {fl / us_t / 1e6:6.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
