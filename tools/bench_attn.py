"""Attention kernel variants on the network's shapes (graph-replay timing;
tuning harness).  python -m tools.bench_attn"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit


def main():
    L = _lib.lib()
    for H, g in ((16, 1), (12, 2)):
        E = H * 64
        qkv = [torch.randn(768, 3 * E, device="cuda").half() for _ in range(g)]
        o = [torch.empty(768, E, device="cuda").half() for _ in range(g)]
        c = ops.attention(qkv, [t[:, E:] for t in qkv], [t[:, 2 * E:] for t in qkv], o, B=1,
                          Nq=768, Nk=768, H=H, q_stride=3 * E, k_stride=3 * E,
                          v_stride=3 * E, o_stride=E, scale=0.125)
        fl = 4 * H * 768 * 768 * 64 * g
        for v in (1, 2, 0, 3):
            L.s3n_attention_set_variant(v)
            us = timeit(lambda: c(_lib.stream()), reps=20)
            print(f"H{H} g{g} variant {v}: {us:6.1f} us  {fl / us / 1e6:6.1f} TF", flush=True)
        L.s3n_attention_set_variant(0)


if __name__ == "__main__":
    main()
