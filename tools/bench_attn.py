"""Attention kernel variants on the network's shapes (graph-replay timing;
tuning harness): the encoder (8 images, 16 heads) and the decoder (1 or 2
pairs, 12 heads, 2 branches), default kernel with and without the XCD-aware
workgroup order, and the other variants.  python -m tools.bench_attn"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, ops
from tools.bench_gemm import timeit


def main():
    L = _lib.lib()
    for B, H, g in ((8, 16, 1), (1, 12, 2), (2, 12, 2)):
        E = H * 64
        N = 768
        qkv = [torch.randn(B * N, 3 * E, device="cuda").half() for _ in range(g)]
        o = [torch.empty(B * N, E, device="cuda").half() for _ in range(g)]
        c = ops.attention(qkv, [t[:, E:] for t in qkv], [t[:, 2 * E:] for t in qkv], o, B=B,
                          Nq=N, Nk=N, H=H, q_stride=3 * E, k_stride=3 * E,
                          v_stride=3 * E, o_stride=E, scale=0.125)
        fl = 4 * B * H * N * N * 64 * g
        ref = None
        for v, name in ((0, "default xcd"), (-1, "default plain"), (-2, "default xcd"),
                        (2, "1 key group"), (3, "4 key groups"), (5, "128-query WG"),
                        (0, "default")):
            L.s3n_attention_set_variant(v)
            if v == -1:
                L.s3n_attention_set_variant(0)
            c(_lib.stream())
            torch.cuda.synchronize()
            if ref is None:
                ref = [x.clone() for x in o]
            same = all(torch.equal(x, y) for x, y in zip(o, ref))
            us = timeit(lambda: c(_lib.stream()), reps=20)
            print(f"B{B} H{H} g{g} {name:14s}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF  same {same}",
                  flush=True)
        L.s3n_attention_set_variant(0)
        L.s3n_attention_set_variant(-2)


if __name__ == "__main__":
    main()
