"""Run one s3n_gemm configuration a few times (for rocprofv3 --pmc passes).

  python -m tools.gemm_one M N K tile [split_k] [debug]
"""
from __future__ import annotations

import sys

import torch

from splatt3r_amd import _lib, ops


def main():
    M, N, K, tile = (int(x) for x in sys.argv[1:5])
    sk = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    dbg = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    A = torch.randn(M, K, device="cuda").half()
    B = torch.randn(N, K, device="cuda").half() * K ** -0.5
    C = torch.empty(M, N, device="cuda", dtype=torch.float16)
    c = ops.gemm([A], [B], [C], M, N, K, lda=K, split_k=sk, tile=tile)
    _lib.lib().s3n_gemm_set_debug(dbg)
    for _ in range(5):
        c(_lib.stream())
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
