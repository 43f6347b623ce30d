"""Calibration only: the tuned s3n GEMM vs torch fp16 matmul (hipBLASLt)
on the frame loop's batched dense shapes (encoder M = 6144 at encoder batch
8, decoder M = 1536 per branch at Bp = 2), warm back-to-back launches timed
with HIP events.

  python -m tools.gemm_vs_hipblaslt
"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, ops

# (M, N, K, groups): encoder qkv / fc1 / fc2 / proj at 8 images, decoder
# qkv / fc1 / fc2 / proj at 2 pairs per branch, the head MLP at Bp = 2
SHAPES = [(6144, 3072, 1024, 1), (6144, 4096, 1024, 1), (6144, 1024, 4096, 1),
          (6144, 1024, 1024, 1), (1536, 2304, 768, 2), (1536, 3072, 768, 2),
          (1536, 768, 3072, 2), (1536, 768, 768, 2), (1536, 6400, 7168, 2)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for M, N, K, g in SHAPES:
        A = [torch.randn(M, K, device="cuda").half() for _ in range(g)]
        B = [(torch.randn(N, K, device="cuda") * K ** -0.5).half() for _ in range(g)]
        C = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(g)]
        c = ops.gemm(A, B, C, M, N, K, lda=K)
        ours = timeit(lambda: c(_lib.stream()))
        At, Bt = torch.stack(A), torch.stack(B).transpose(1, 2)
        lib = timeit(lambda: torch.bmm(At, Bt))
        fl = 2.0 * M * N * K * g
        print(f"{M}x{N}x{K} g{g}: s3n {ours:8.1f} us ({fl / ours / 1e6:5.0f} TF, "
              f"{c.desc.split()[-1]})  hipBLASLt {lib:8.1f} us ({fl / lib / 1e6:5.0f} TF)",
              flush=True)


if __name__ == "__main__":
    main()
