"""Where does an implicit-im2col conv launch's time go?  The network's
large DPT 3x3 convs (4 groups, NHWC fp16), each tile config timed in full,
without the MFMAs, without the operand DMA, without both, and without the
K loop (tuning only).

  python -m tools.bench_conv_parts [--tiles 3,5,28]
"""
from __future__ import annotations

import argparse

import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit

# (B, H, W, Cin, Cout): head conv2 at 384x512, head conv0 at 192x256,
# refinenet stage 0 at 96x128
SHAPES = [(1, 384, 512, 128, 128), (1, 192, 256, 256, 128), (1, 96, 128, 256, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="3,5,28")
    ap.add_argument("--B", type=int, default=1, help="images per group (pairs per replay)")
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    L = _lib.lib()
    G = 4
    for B, H, W, Cin, Cout in SHAPES:
        B *= a.B
        x = [torch.randn(B, H, W, Cin, device="cuda").half() for _ in range(G)]
        w = [(torch.randn(Cout, 9 * Cin, device="cuda") * (9 * Cin) ** -0.5).half()
             for _ in range(G)]
        out = [torch.empty(B, H, W, Cout, device="cuda", dtype=torch.float16) for _ in range(G)]
        conv = dict(H=H, W=W, C=Cin, k=3, stride=1, pad=1, oH=H, oW=W, relu_in=False)
        M, K = B * H * W, 9 * Cin
        fl = 2 * M * Cout * K * G
        for tile in tiles:
            c = ops.gemm(x, w, out, M, Cout, K, lda=0, conv=conv, split_k=1, tile=tile)
            try:
                c(_lib.stream())
            except RuntimeError as e:          # a tile that cannot run this shape
                print(f"{M}x{Cout}x{K} g{G} conv t{tile}: skipped ({e})", flush=True)
                continue
            r = []
            for dbg in (0, 1, 2, 3, 8):
                L.s3n_gemm_set_debug(dbg)
                r.append(timeit(lambda: c(_lib.stream()), reps=10))
            L.s3n_gemm_set_debug(0)
            print(f"{M}x{Cout}x{K} g{G} conv t{tile}: full {r[0]:7.1f} us ({fl / r[0] / 1e6:5.0f} TF)"
                  f"  no-mfma {r[1]:7.1f}  no-dma {r[2]:7.1f}  neither {r[3]:7.1f}  no-loop {r[4]:6.1f}",
                  flush=True)


if __name__ == "__main__":
    main()
