"""B-direct GEMM tiles (csrc/net_gemm_t9.hip, tiles 70-77: the weights read
from a fragment-packed copy straight into registers, A through the LDS
ring) timed on the network's dense shapes next to the LDS-staged tiles of
the same reduction class (16x16x32, no split, vector epilogue) and
hipBLASLt; outputs checked bit-identical to the class's tile 32 ('!' marks
a difference).

  python -m tools.bench_gemm_bd [--tiles 70,71] [--shapes MxNxKxG,...]
"""
from __future__ import annotations

import argparse
import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit

SHAPES = ["1536x768x768x2", "1536x2304x768x2", "1536x1536x768x2", "1536x3072x768x2",
          "1536x768x3072x2", "6144x3072x1024x1", "6144x1024x1024x1", "6144x4096x1024x1",
          "6144x1024x4096x1", "1536x7168x1792x2", "1536x6400x7168x2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="70,71,72,73,74,75,76,77")
    ap.add_argument("--ref-tiles", default="32,26,22,63")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--act", default="gelu")
    a = ap.parse_args()
    st = _lib.stream()
    for sh in a.shapes.split(","):
        M, N, K, G = (int(x) for x in sh.split("x"))
        gen = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
        A = [torch.randn(M, K, device="cuda", generator=gen).half() for _ in range(G)]
        B = [(torch.randn(N, K, device="cuda", generator=gen) * K ** -0.5).half() for _ in range(G)]
        bias = [torch.randn(N, device="cuda", generator=gen) * 0.1 for _ in range(G)]
        C = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(G)]
        fl = 2 * M * N * K * G
        line = [f"{sh:>18}"]
        ref = ops.gemm(A, B, C, M, N, K, lda=K, split_k=1, tile=32, bias=bias, act=a.act)
        ref(st)
        torch.cuda.synchronize()
        want = [c.clone() for c in C]
        for t in (int(x) for x in a.ref_tiles.split(",") if x):
            try:
                c = ops.gemm(A, B, C, M, N, K, lda=K, split_k=1, tile=t, bias=bias, act=a.act)
                us = timeit(lambda: c(_lib.stream()), reps=20)
            except Exception as e:   # tile not valid for this shape
                line.append(f"t{t} --")
                continue
            line.append(f"t{t} {us:6.1f}")
        for t in (int(x) for x in a.tiles.split(",") if x):
            for c in C:
                c.zero_()
            c = ops.gemm(A, B, C, M, N, K, lda=K, split_k=1, tile=t, bias=bias, act=a.act)
            c(_lib.stream())
            torch.cuda.synchronize()
            eq = all(torch.equal(x, w) for x, w in zip(C, want))
            us = timeit(lambda: c(_lib.stream()), reps=20)
            line.append(f"t{t} {us:6.1f}{'' if eq else '!'}")
        # hipBLASLt calibration (no epilogue)
        Bt = [b.t() for b in B]
        us = timeit(lambda: [torch.matmul(x, y) for x, y in zip(A, Bt)], reps=20)
        line.append(f"blt {us:6.1f}")
        print("  ".join(line), f"  ({fl / 1e9:.1f} GF)", flush=True)


if __name__ == "__main__":
    main()
