"""Where does a GEMM launch's time go?  Each tile config timed in full, with
the MFMAs skipped (operand DMA + barriers + LDS reads) and with the DMA
skipped (LDS reads + MFMAs on stale LDS), HIP-graph replays (tuning only).

  python -m tools.bench_gemm_parts
"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit

import argparse

SHAPES = [(4096, 4096, 4096), (1536, 6400, 7168), (196608, 128, 1152), (12288 * 4, 256, 2304)]
SMALL = [(768, 1024, 1024), (768, 4096, 1024), (768, 1024, 4096), (768, 3072, 1024),
         (1536, 768, 768), (1536, 3072, 768), (1536, 768, 3072)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true", help="the 768-row network shapes")
    ap.add_argument("--tiles", default="3,4,13,14")
    ap.add_argument("--shapes", default="",
                    help="MxNxKxG list (G = groups of one grouped launch), overrides --small")
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    L = _lib.lib()
    shapes = [tuple(int(x) for x in s.split("x")) for s in a.shapes.split(",") if s]
    shapes = shapes or [(M, N, K, 1) for M, N, K in (SMALL if a.small else SHAPES)]
    for M, N, K, G in shapes:
        A = [torch.randn(M, K, device="cuda").half() for _ in range(G)]
        B = [torch.randn(N, K, device="cuda").half() * K ** -0.5 for _ in range(G)]
        C = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(G)]
        fl = 2 * M * N * K * G
        for tile in tiles:
            try:
                c = ops.gemm(A, B, C, M, N, K, lda=K, split_k=1, tile=tile)
            except Exception as e:
                print(f"{M}x{N}x{K}x{G} t{tile}: {type(e).__name__} {str(e)[:60]}", flush=True)
                continue
            r = []
            for dbg in (0, 1, 2, 3, 8, 12):
                L.s3n_gemm_set_debug(dbg)
                r.append(timeit(lambda: c(_lib.stream()), reps=10))
            L.s3n_gemm_set_debug(0)
            print(f"{M}x{N}x{K}x{G} t{tile}: full {r[0]:7.1f} us ({fl / r[0] / 1e6:5.0f} TF)  "
                  f"no-mfma {r[1]:7.1f}  no-dma {r[2]:7.1f}  neither {r[3]:7.1f}  "
                  f"no-loop {r[4]:6.1f}  no-loop-no-epi {r[5]:6.1f}", flush=True)


if __name__ == "__main__":
    main()
