"""Calibration only: torch fp16 matmul (hipBLASLt) on the network's dense
GEMM shapes, run under rocprofv3 --kernel-trace to read which macro tile /
MFMA / prefetch configuration the library picks per shape (kernel names)."""
import torch

SHAPES = [(768, 3072, 1024, 1), (768, 4096, 1024, 1), (768, 1024, 4096, 1), (768, 1024, 1024, 1),
          (768, 2304, 768, 2), (768, 768, 768, 2), (768, 3072, 768, 2), (768, 768, 3072, 2),
          (768, 6400, 7168, 2)]

for M, N, K, g in SHAPES:
    A = torch.randn(g, M, K, device="cuda").half()
    B = (torch.randn(g, N, K, device="cuda").half() * K ** -0.5).transpose(1, 2)
    for _ in range(5):
        torch.bmm(A, B)
    torch.cuda.synchronize()
    print(M, N, K, g, flush=True)
