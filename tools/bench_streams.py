"""Do two HIP streams share the chip?  Two chains of 768-row GEMMs, run alone,
then on two streams at once, as HIP-graph replays and as eager launches, with
and without a host synchronisation of the first stream in between (tuning).

  python -m tools.bench_streams
"""
from __future__ import annotations

import time

import torch

from splatt3r_amd import _lib, ops


def chain(n):
    A = torch.randn(768, 1024, device="cuda").half()
    B = torch.randn(1024, 1024, device="cuda").half() * 0.03
    C = torch.empty(768, 1024, device="cuda", dtype=torch.float16)
    c = ops.gemm([A], [B], [C], 768, 1024, 1024, lda=1024, split_k=1)
    return lambda: [c(_lib.stream()) for _ in range(n)]


def graph_of(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def wall(fn, reps=5):
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def main():
    n = 200
    f1, f2, f3 = chain(n), chain(n), chain(20)
    g1, g2 = graph_of(f1), graph_of(f2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def on(s, fn):
        with torch.cuda.stream(s):
            fn()

    print(f"graph alone            {wall(lambda: on(s1, g1.replay)):7.2f} ms", flush=True)
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        on(s1, g1.replay)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"  host time of one {n}-node graph replay {(t1 - t0) * 1e3:.3f} ms, "
              f"to completion {(t2 - t0) * 1e3:.3f} ms", flush=True)
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        on(s1, f1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"  host time of {n} eager launches {(t1 - t0) * 1e3:.3f} ms", flush=True)
    print(f"graph x2 same stream   {wall(lambda: (on(s1, g1.replay), on(s1, g2.replay))):7.2f} ms")
    print(f"graph x2 two streams   {wall(lambda: (on(s2, g2.replay), on(s1, g1.replay))):7.2f} ms")

    def with_sync():
        on(s2, g2.replay)
        for _ in range(10):          # main-stream work with host syncs (GN-like)
            on(s1, f3)
            s1.synchronize()
    print(f"graph s2 + 10 synced s1 bursts {wall(with_sync):7.2f} ms "
          f"(s2 alone {wall(lambda: on(s2, g2.replay)):.2f}, bursts alone "
          f"{wall(lambda: [(on(s1, f3), s1.synchronize()) for _ in range(10)]):.2f})")
    d = torch.cuda.default_stream()
    print(f"graph x2 side + default {wall(lambda: (on(s2, g2.replay), on(d, g1.replay))):7.2f} ms")

    def default_sync():
        on(s2, g2.replay)
        for _ in range(10):
            on(d, f3)
            d.synchronize()
    print(f"graph s2 + 10 synced default bursts {wall(default_sync):7.2f} ms")
    x = torch.ones(1024, device="cuda")

    def default_cpu():
        on(s2, g2.replay)
        for _ in range(10):
            on(d, f3)
            x.cpu()
    print(f"graph s2 + 10 default bursts with .cpu() {wall(default_cpu):7.2f} ms")
    hb = torch.empty(1024, pin_memory=True)

    def default_pinned():
        on(s2, g2.replay)
        for _ in range(10):
            on(d, f3)
            hb.copy_(x, non_blocking=True)
            d.synchronize()
    print(f"graph s2 + 10 default bursts with pinned copy {wall(default_pinned):7.2f} ms")
    print(f"eager alone            {wall(lambda: on(s1, f1)):7.2f} ms")
    print(f"eager x2 two streams   {wall(lambda: (on(s2, f2), on(s1, f1))):7.2f} ms")


if __name__ == "__main__":
    main()
