"""Per-tile s3n_gemm throughput on chosen shapes next to torch.matmul
(hipBLASLt) on the same fp16 operands, warm launches replayed from a HIP
graph (no enqueue gaps), random operands (uniform data would read high,
cdna_hip_programming.md §5.4 rule 25).

  python -m tools.gemm_ceiling --shapes 4096x4096x4096x1,6144x4096x1024x1 --tiles 4,25,32,36
"""
from __future__ import annotations

import argparse

import torch

from splatt3r_amd import _lib, ops


def timeit(fn, reps=20):
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
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e3
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096x4096x1,6144x4096x1024x1,6144x3072x1024x1,"
                                        "6144x1024x4096x1,6144x1024x1024x1,1536x3072x768x2,"
                                        "1536x768x3072x2,1536x2304x768x2,1536x768x768x2,"
                                        "1536x6400x7168x2,1536x7168x1792x2")
    ap.add_argument("--tiles", default="")
    ap.add_argument("--splits", default="1")
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",") if t] or sorted(ops._TILE_SHAPES)
    splits = [int(s) for s in a.splits.split(",")]
    for sh in a.shapes.split(","):
        M, N, K, g = (int(x) for x in sh.split("x"))
        gen = torch.Generator(device="cuda").manual_seed(0)
        A = [torch.rand(M, K, device="cuda", generator=gen).sub_(0.5).half() for _ in range(g)]
        B = [(torch.rand(N, K, device="cuda", generator=gen).sub_(0.5) * 2 * K ** -0.5).half()
             for _ in range(g)]
        C = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(g)]
        fl = 2.0 * M * N * K * g
        ref = [(A[i].float() @ B[i].float().T) for i in range(g)]
        res = []
        for t in tiles:
            if t in ops._HALO:
                continue
            for sk in splits:
                try:
                    c = ops.gemm(A, B, C, M, N, K, lda=K, split_k=sk, tile=t)
                    for x in C:
                        x.fill_(float("nan"))
                    c(_lib.stream())
                    err = max(float(((C[i].float() - ref[i]).abs().max() /
                                     ref[i].abs().max()).item()) for i in range(g))
                    if not err < 2e-3:
                        print(f"  t{t}s{sk}: WRONG rel err {err:.3g}", flush=True)
                        continue
                    us = timeit(lambda: c(_lib.stream()))
                except Exception as e:   # tile not valid for this shape
                    print(f"  t{t}s{sk}: {type(e).__name__}: {str(e)[:80]}", flush=True)
                    continue
                res.append((us, f"t{t}s{sk}"))
        Ab = torch.stack(A)
        Bb = torch.stack(B).transpose(1, 2)
        us_t = timeit(lambda: torch.bmm(Ab, Bb))
        res.sort()
        line = f"{M}x{N}x{K} g{g}: torch {us_t:7.1f}us {fl / us_t / 1e6:5.0f}TF |"
        line += " ".join(f" {n} {u:6.1f}us {fl / u / 1e6:4.0f}TF" for u, n in res[:6])
        print(line, flush=True)


if __name__ == "__main__":
    main()
