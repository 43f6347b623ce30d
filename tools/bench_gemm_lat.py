"""Per-K-tile latency of one GEMM workgroup in isolation (64 x 64 output,
long K) for each staging depth, plus a 4096^3 throughput point."""
import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit


def main():
    for (M, N, K) in ((64, 64, 65536), (128, 128, 65536), (256, 128, 65536)):
        A = torch.randn(M, K, device="cuda").half()
        B = torch.randn(N, K, device="cuda").half()
        C = torch.empty(M, N, device="cuda")
        for tile in (1, 6, 7, 2, 3, 5, 4):
            try:
                c = ops.gemm([A], [B], [C], M, N, K, lda=K, split_k=1, tile=tile)
            except Exception as e:  # noqa
                continue
            us = timeit(lambda: c(_lib.stream()), reps=5)
            print(f"{M}x{N}x{K} tile{tile}: {us:8.1f} us -> {us / (K / 64) * 1e3:6.0f} ns per K tile",
                  flush=True)
    M = N = K = 4096
    A = torch.randn(M, K, device="cuda").half()
    B = torch.randn(N, K, device="cuda").half()
    C = torch.empty(M, N, device="cuda", dtype=torch.float16)
    for tile in (2, 3, 4, 5):
        c = ops.gemm([A], [B], [C], M, N, K, lda=K, split_k=1, tile=tile)
        us = timeit(lambda: c(_lib.stream()), reps=5)
        print(f"4096^3 tile{tile}: {us:8.1f} us {2 * M * N * K / us / 1e6:6.0f} TF", flush=True)
    us = timeit(lambda: A @ B.T, reps=5)
    print(f"4096^3 torch: {us:8.1f} us {2 * M * N * K / us / 1e6:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
