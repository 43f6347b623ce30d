"""Epilogue cost of the decoder's 768x768x768 grouped GEMMs (tuning only):
the same launch with fp16 output, + bias, fp32 output + in-place residual
(the proj / fc2 form), and the RoPE epilogue (the q form), per tile config.

  python -m tools.bench_gemm_epi
"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit


def main():
    M = N = K = 768
    g = 2
    dev = "cuda"
    A = [torch.randn(M, K, device=dev).half() for _ in range(g)]
    B = [(torch.randn(N, K, device=dev) * K ** -0.5).half() for _ in range(g)]
    b = [torch.randn(N, device=dev) for _ in range(g)]
    C16 = [torch.empty(M, N, device=dev, dtype=torch.float16) for _ in range(g)]
    X = [torch.randn(M, N, device=dev) for _ in range(g)]
    Xo = [torch.randn(M, N, device=dev) for _ in range(g)]
    for tile in (1, 10, 15, 16):
        r = {}
        r["f16"] = timeit(lambda: ops.gemm(A, B, C16, M, N, K, lda=K, tile=tile, split_k=1)(_lib.stream()))
        r["f16+bias"] = timeit(lambda: ops.gemm(A, B, C16, M, N, K, lda=K, bias=b, tile=tile,
                                                split_k=1)(_lib.stream()))
        r["f32+bias"] = timeit(lambda: ops.gemm(A, B, Xo, M, N, K, lda=K, bias=b, tile=tile,
                                                split_k=1)(_lib.stream()))
        r["f32+bias+R1 (other)"] = timeit(lambda: ops.gemm(A, B, Xo, M, N, K, lda=K, bias=b, R1=X,
                                                           ldr1=N, tile=tile, split_k=1)(_lib.stream()))
        r["f32+bias+R1 in place"] = timeit(lambda: ops.gemm(A, B, X, M, N, K, lda=K, bias=b, R1=X,
                                                            ldr1=N, tile=tile, split_k=1)(_lib.stream()))
        print(f"t{tile}: " + "  ".join(f"{k} {v:5.1f}" for k, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
