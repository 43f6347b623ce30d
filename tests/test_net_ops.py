"""Network kernels (include/s3n.h) vs plain PyTorch fp32 references of the
same op, on the same (fp16-rounded) inputs.  Tolerances are stated per test:
fp16 operands with fp32 MFMA accumulation vs an fp32 matmul of the same
fp16-rounded operands -> only accumulation-order differences (~1e-6 rel),
plus one fp16 rounding when the kernel writes fp16."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def _rand(*shape, scale=1.0, dtype=torch.float16, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, device="cuda", generator=g) * scale).to(dtype)


@pytest.mark.parametrize("M,N,K,groups", [(768, 3072, 1024, 1), (200, 96, 72, 2), (37, 1536, 96, 4),
                                          (4096, 256, 2304, 1), (768, 6400, 64, 2)])
def test_gemm_dense_bias_residual(M, N, K, groups):
    from splatt3r_amd import ops, _lib
    A = [_rand(M, K, seed=g) for g in range(groups)]
    W = [_rand(N, K, scale=K ** -0.5, seed=10 + g) for g in range(groups)]
    b = [_rand(N, dtype=torch.float32, seed=20 + g) for g in range(groups)]
    R = [_rand(M, N, dtype=torch.float32, seed=30 + g) for g in range(groups)]
    C = [torch.empty(M, N, device="cuda") for _ in range(groups)]
    ops.gemm(A, W, C, M, N, K, lda=K, bias=b, R1=R, ldr1=N)(_lib.stream())
    for g in range(groups):
        ref = A[g].float() @ W[g].float().T + b[g] + R[g]
        assert rel_err(C[g], ref) < 1e-5, (g, rel_err(C[g], ref))


@pytest.mark.parametrize("M,N,K,groups,split,tile", [
    (768, 1024, 4096, 1, 3, 0), (768, 768, 768, 2, 2, 1), (200, 96, 200, 2, 5, 0),
    (130, 300, 1000, 1, 7, 2), (300, 256, 2304, 4, 4, 3), (768, 1024, 1024, 1, 1, 3),
    (700, 200, 960, 2, 1, 4), (520, 384, 640, 1, 2, 5), (768, 6400, 512, 2, 1, 4),
    (300, 200, 1000, 1, 1, 6), (130, 96, 2000, 2, 1, 7), (600, 256, 200, 1, 1, 8),
    (768, 1024, 1000, 1, 1, 9), (300, 200, 1000, 2, 3, 10), (130, 300, 968, 1, 2, 11),
    (700, 256, 2304, 2, 1, 12), (64, 64, 136, 1, 1, 9), (700, 256, 1000, 2, 2, 14),
    (520, 300, 640, 1, 1, 14), (300, 500, 1000, 1, 3, 14),
    # in-workgroup K-groups (tiles 15-20), incl. K-tile counts not divisible
    # by the group count, a single K tile, and global split-K on top
    (768, 1024, 1024, 1, 1, 15), (768, 1024, 4096, 1, 1, 16), (300, 200, 1000, 2, 1, 16),
    (768, 768, 768, 2, 1, 17), (700, 256, 2304, 1, 1, 18), (130, 300, 968, 1, 1, 19),
    (768, 1024, 1088, 1, 1, 20), (64, 64, 64, 1, 1, 16), (520, 384, 640, 2, 2, 16),
    (300, 256, 200, 1, 1, 20),
    # v_mfma_f32_16x16x32 tiles (21-31): ragged M / N / K tails, global split-K
    # (N % 8 == 0: these tiles need the vector epilogue, see
    # test_gemm_mf16_tiles_reject_unaligned_n)
    (768, 3072, 1024, 1, 1, 21), (130, 296, 968, 2, 1, 21), (768, 768, 768, 2, 1, 22),
    (300, 200, 1000, 1, 3, 22), (768, 4096, 1024, 1, 1, 23), (520, 296, 640, 2, 2, 23),
    (768, 3072, 768, 2, 1, 24), (700, 256, 2304, 1, 1, 24), (768, 1600, 1792, 2, 1, 25),
    (300, 136, 520, 1, 1, 25), (768, 1024, 1024, 1, 1, 26), (64, 64, 136, 1, 2, 26),
    (768, 2304, 768, 2, 1, 27), (130, 96, 2000, 2, 1, 27), (600, 256, 200, 1, 1, 28),
    (768, 768, 3072, 2, 3, 29), (300, 496, 1000, 1, 1, 29), (768, 3072, 1024, 1, 1, 30),
    (200, 96, 200, 2, 5, 30), (768, 1024, 4096, 1, 2, 31), (130, 296, 968, 1, 1, 31),
    (1536, 2304, 768, 2, 1, 32), (130, 296, 968, 1, 2, 32), (6144, 1024, 1024, 1, 1, 34),
    (300, 200, 1000, 2, 3, 34), (1536, 768, 3072, 1, 1, 35), (520, 300, 640, 1, 1, 35),
    (6144, 4096, 1024, 1, 1, 36), (130, 96, 2000, 2, 2, 36), (1536, 3072, 768, 2, 1, 37),
    (64, 64, 136, 1, 1, 37),
    # k_gemm_pp tiles (63, 65, 68: half-K-tile fragment pipeline): ragged M / N,
    # K % 64 != 0, global split-K 2 and 3
    (1536, 2304, 768, 2, 1, 63), (300, 200, 1000, 2, 3, 63), (130, 300, 968, 1, 2, 65),
    (1536, 3072, 768, 2, 2, 65), (768, 6400, 1792, 2, 2, 68), (520, 296, 640, 1, 1, 68),
    (300, 136, 520, 1, 3, 68)])
def test_gemm_split_k_and_tiles(M, N, K, groups, split, tile):
    """Split-K partials + ordered reduce + the full epilogue (bias, GELU,
    fp32 residual, fp16 out + fp16 copy) for every tile shape."""
    from splatt3r_amd import ops, _lib
    A = [_rand(M, K, seed=g) for g in range(groups)]
    W = [_rand(N, K, scale=K ** -0.5, seed=10 + g) for g in range(groups)]
    b = [_rand(N, dtype=torch.float32, seed=20 + g) for g in range(groups)]
    R = [_rand(M, N, dtype=torch.float32, seed=30 + g) for g in range(groups)]
    C = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(groups)]
    C2 = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(groups)]
    ops.gemm(A, W, C, M, N, K, lda=K, bias=b, act="gelu", R1=R, ldr1=N, C2=C2, ldc2=N,
             split_k=split, tile=tile)(_lib.stream())
    for g in range(groups):
        ref = F.gelu(A[g].float() @ W[g].float().T + b[g]) + R[g]
        assert rel_err(C[g], ref) < 2e-3, (g, rel_err(C[g], ref))
        assert torch.equal(C[g], C2[g])


@pytest.mark.parametrize("split,tile,Cin", [(3, 1, 768), (9, 0, 768), (2, 3, 768), (1, 4, 768),
                                            (1, 5, 768), (1, 9, 768), (2, 10, 768), (1, 11, 96),
                                            (1, 12, 768), (1, 9, 96), (2, 9, 136), (1, 15, 768),
                                            (1, 16, 96), (1, 17, 768), (2, 18, 256), (1, 19, 136),
                                            (1, 20, 768), (1, 21, 768), (2, 23, 256),
                                            (1, 24, 96), (1, 25, 136), (1, 27, 768),
                                            (1, 29, 256), (1, 31, 768), (1, 32, 768),
                                            (2, 34, 256), (1, 35, 136), (1, 36, 768),
                                            (1, 37, 96), (1, 63, 768), (2, 65, 256),
                                            (1, 68, 136), (3, 63, 96)])
def test_gemm_implicit_conv_split_k(split, tile, Cin):
    from splatt3r_amd import ops, _lib
    B, H, W, Cout, k, stride, pad = 1, 12, 16, 256, 3, 1, 1
    x = _rand(B, H, W, Cin, seed=13)
    w = _rand(Cout, Cin, k, k, scale=(Cin * k * k) ** -0.5, seed=14)
    out = torch.empty(B, H, W, Cout, device="cuda")
    wk = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous()
    conv = dict(H=H, W=W, C=Cin, k=k, stride=stride, pad=pad, oH=H, oW=W, relu_in=True)
    ops.gemm([x], [wk], [out], B * H * W, Cout, k * k * Cin, lda=0, conv=conv, split_k=split,
             tile=tile)(_lib.stream())
    ref = F.conv2d(x.float().permute(0, 3, 1, 2).clamp_min(0), w.float(), padding=pad)
    assert rel_err(out, ref.permute(0, 2, 3, 1)) < 1e-5


@pytest.mark.parametrize("pp,ref,M,N,K,groups,split", [
    (63, 32, 1536, 2304, 768, 2, 1), (63, 26, 300, 200, 1000, 2, 3), (65, 3, 130, 300, 968, 1, 2),
    (65, 3, 1536, 768, 3072, 2, 1), (68, 36, 768, 6400, 1792, 2, 2), (68, 25, 520, 296, 640, 1, 1)])
def test_gemm_pp_tiles_bitexact_vs_same_reduction_class(pp, ref, M, N, K, groups, split):
    """k_gemm_pp (net_gemm_t8.hip: its own two-half register pipeline and
    stage reuse) computes every element with the same
    MFMA k order as a k_gemm tile of the same ops.reduction_class:
    bit-identical outputs, with the full epilogue, ragged tails and split-K
    (ADVICE r04)."""
    from splatt3r_amd import ops, _lib
    assert ops.reduction_class(K, pp, split) == ops.reduction_class(K, ref, split)
    A = [_rand(M, K, seed=g) for g in range(groups)]
    W = [_rand(N, K, scale=K ** -0.5, seed=10 + g) for g in range(groups)]
    b = [_rand(N, dtype=torch.float32, seed=20 + g) for g in range(groups)]
    R = [_rand(M, N, dtype=torch.float32, seed=30 + g) for g in range(groups)]
    outs = []
    for tile in (pp, ref):
        C = [torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
             for _ in range(groups)]
        ops.gemm(A, W, C, M, N, K, lda=K, bias=b, act="gelu", R1=R, ldr1=N, split_k=split,
                 tile=tile)(_lib.stream())
        outs.append(C)
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("bd,ref,M,N,K,groups", [
    (70, 32, 1536, 3072, 768, 2), (71, 26, 6144, 1024, 1024, 1), (72, 22, 300, 200, 1056, 2),
    (73, 26, 130, 296, 992, 1), (74, 32, 1536, 2304, 768, 2), (75, 28, 520, 296, 640, 1),
    (76, 32, 300, 136, 544, 2), (77, 26, 768, 1024, 4096, 1), (70, 32, 64, 40, 96, 1),
    (71, 32, 1, 24, 32, 1), (72, 26, 200, 1040, 2080, 3), (78, 22, 1536, 768, 768, 2),
    (79, 32, 130, 296, 992, 1), (78, 26, 64, 40, 96, 1)])
def test_gemm_bdirect_tiles_bitexact_vs_same_reduction_class(bd, ref, M, N, K, groups):
    """The B-direct tiles (net_gemm_t9.hip: B fragments from the packed
    weights, ops.packed_b, straight into registers) compute every element
    in the reduction class of the LDS-staged 16x16x32 tiles: bit-identical
    outputs with the full epilogue (bias, GELU, fp32 residual, fp16 out +
    copy), ragged M, N % 16 != 0 (zero-padded packed rows), K % 64 == 32,
    a single row and K tile; and correct against torch."""
    from splatt3r_amd import ops, _lib
    assert ops.reduction_class(K, bd, 1) == ops.reduction_class(K, ref, 1)
    A = [_rand(M, K, seed=g) for g in range(groups)]
    W = [_rand(N, K, scale=K ** -0.5, seed=10 + g) for g in range(groups)]
    b = [_rand(N, dtype=torch.float32, seed=20 + g) for g in range(groups)]
    R = [_rand(M, N, dtype=torch.float32, seed=30 + g) for g in range(groups)]
    outs = []
    for tile in (bd, ref):
        C = [torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
             for _ in range(groups)]
        C2 = [torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
              for _ in range(groups)]
        ops.gemm(A, W, C, M, N, K, lda=K, bias=b, act="gelu", R1=R, ldr1=N, C2=C2, ldc2=N,
                 split_k=1, tile=tile)(_lib.stream())
        outs.append((C, C2))
    for g in range(groups):
        assert torch.equal(outs[0][0][g], outs[1][0][g])
        assert torch.equal(outs[0][0][g], outs[0][1][g])
        ref_ = F.gelu(A[g].float() @ W[g].float().T + b[g]) + R[g]
        assert rel_err(outs[0][0][g], ref_) < 2e-3


@pytest.mark.parametrize("bd,ref,M,N,K,groups,split", [
    (73, 26, 1536, 768, 3072, 2, 3), (72, 22, 1536, 768, 3072, 2, 2),
    (74, 32, 6144, 1024, 4096, 1, 2), (77, 26, 300, 136, 2080, 1, 4),
    (70, 32, 520, 296, 1056, 3, 3), (75, 28, 1, 24, 640, 1, 2), (78, 26, 1536, 768, 3072, 2, 2)])
def test_gemm_bdirect_split_k_bitexact_vs_same_reduction_class(bd, ref, M, N, K, groups, split):
    """Split-K on the B-direct tiles: each split's K tiles in order into an
    fp32 plane, the planes added in split order by k_splitk_reduce -- the
    same bits as an LDS-staged tile of the class with the same split
    (ragged M and N, K % 64 == 32 at the last split, three groups), and
    correct against torch."""
    from splatt3r_amd import ops, _lib
    assert ops.reduction_class(K, bd, split) == ops.reduction_class(K, ref, split)
    A = [_rand(M, K, seed=g) for g in range(groups)]
    W = [_rand(N, K, scale=K ** -0.5, seed=10 + g) for g in range(groups)]
    b = [_rand(N, dtype=torch.float32, seed=20 + g) for g in range(groups)]
    R = [_rand(M, N, dtype=torch.float32, seed=30 + g) for g in range(groups)]
    outs = []
    for tile in (bd, ref):
        C = [torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
             for _ in range(groups)]
        ops.gemm(A, W, C, M, N, K, lda=K, bias=b, act="gelu", R1=R, ldr1=N, split_k=split,
                 tile=tile)(_lib.stream())
        outs.append(C)
    for g in range(groups):
        assert torch.equal(outs[0][g], outs[1][g])
        ref_ = F.gelu(A[g].float() @ W[g].float().T + b[g]) + R[g]
        assert rel_err(outs[0][g], ref_) < 2e-3


@pytest.mark.parametrize("tile", [70, 71, 72, 73, 74, 75, 76, 77, 78, 79])
def test_gemm_bdirect_rope_and_scatter_epilogues(tile):
    """The B-direct tiles share the LDS-staged epilogue: the fused RoPE2D
    columns and the ConvTranspose scatter store equal tile 32's bits."""
    from splatt3r_amd import ops, _lib
    from splatt3r_amd.net import positions, rope_tables
    B, ht, wt, K = 1, 24, 32, 128
    M, Nout = B * ht * wt, 16 * 64
    cos, sin = rope_tables(64, "cuda")
    pos = [positions(B, ht, wt, "cuda")]
    A, W = [_rand(M, K, seed=41)], [_rand(Nout, K, scale=K ** -0.5, seed=51)]
    b = [_rand(Nout, dtype=torch.float32, seed=61)]
    got = []
    for t in (tile, 32):
        C = [torch.empty(M, Nout, device="cuda")]
        ops.gemm(A, W, C, M, Nout, K, lda=K, bias=b, rope=(cos, sin), rope_pos=pos,
                 rope_ncols=1024, tile=t)(_lib.stream())
        got.append(C[0])
    assert torch.equal(got[0], got[1])
    s, cout, K2 = 2, 64, 256
    A2, W2 = [_rand(M, K2, seed=42)], [_rand(s * s * cout, K2, scale=K2 ** -0.5, seed=52)]
    got = []
    for t in (tile, 32):
        C = [torch.empty(B, ht * s, wt * s, cout, device="cuda")]
        ops.gemm(A2, W2, C, M, s * s * cout, K2, lda=K2, store=("convt", ht, wt, s, cout),
                 tile=t)(_lib.stream())
        got.append(C[0])
    assert torch.equal(got[0], got[1])


def test_gemm_bdirect_tiles_need_a_packed_b():
    """Without a packed B (B given as a raw pointer) the B-direct tiles fail
    instead of running another tile."""
    from splatt3r_amd import ops, _lib
    M, N, K = 256, 256, 256
    A, W = [_rand(M, K)], _rand(N, K, scale=K ** -0.5, seed=1)
    C = [torch.empty(M, N, device="cuda")]
    with pytest.raises(RuntimeError, match="B-direct"):
        ops.gemm(A, [W.data_ptr()], C, M, N, K, lda=K, split_k=1, tile=70)(_lib.stream())


@pytest.mark.parametrize("tile", [21, 26, 32, 36, 63, 68])
def test_gemm_mf16_tiles_reject_unaligned_n(tile):
    """A 16x16x32 tile stages its fp32 tile through LDS (vector epilogue:
    N % 8 == 0, aligned operands); with N % 8 != 0 the launch fails instead of
    silently running another tile (which would change its reduction class,
    ops.reduction_class)."""
    from splatt3r_amd import ops, _lib
    M, N, K = 130, 300, 968
    A, W = [_rand(M, K)], [_rand(N, K, scale=K ** -0.5, seed=1)]
    C = [torch.empty(M, N, device="cuda")]
    with pytest.raises(RuntimeError, match="vector epilogue"):
        ops.gemm(A, W, C, M, N, K, lda=K, split_k=1, tile=tile)(_lib.stream())


def test_gemm_gelu_erf_accuracy():
    """The GELU epilogue's erf (Abramowitz & Stegun 7.1.26 on v_rcp / v_exp,
    net_gemm_kernel.hpp erf_fast) over x in [-12, 12]: |gelu - exact| <=
    0.5 |x| 5e-7 + 2 ulp, i.e. far below the fp16 quantum the network stores
    GELU outputs in."""
    from splatt3r_amd import ops, _lib
    M, N, K = 64 * 1024, 8, 8
    x = torch.linspace(-12, 12, M, device="cuda")
    A = torch.zeros(M, K, device="cuda", dtype=torch.float16)
    A[:, 0] = x.half()
    xv = A[:, 0].double()                      # the exact fp16 inputs
    W = torch.zeros(N, K, device="cuda", dtype=torch.float16)
    W[:, 0] = 1.0
    C = torch.empty(M, N, device="cuda")
    ops.gemm([A], [W], [C], M, N, K, lda=K, act="gelu")(_lib.stream())
    ref = 0.5 * xv * (1.0 + torch.erf(xv / 2 ** 0.5))
    err = (C[:, 0].double() - ref).abs()
    bound = 0.5 * xv.abs() * 5e-7 + 6e-7 * ref.abs() + 1e-12
    assert bool((err <= bound).all()), float((err / bound).max())


def test_gemm_split_k_is_deterministic():
    from splatt3r_amd import ops, _lib
    M, N, K = 768, 1024, 4096
    A, W = _rand(M, K), _rand(N, K, scale=K ** -0.5, seed=1)
    outs = []
    for _ in range(3):
        C = torch.empty(M, N, device="cuda")
        ops.gemm([A], [W], [C], M, N, K, lda=K, split_k=4)(_lib.stream())
        outs.append(C)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def test_gemm_gelu_fp16_out_and_copy():
    from splatt3r_amd import ops, _lib
    M, N, K = 300, 512, 256
    A, W, b = _rand(M, K), _rand(N, K, scale=K ** -0.5, seed=1), _rand(N, dtype=torch.float32, seed=2)
    C = torch.empty(M, N, device="cuda", dtype=torch.float16)
    C2 = torch.empty(M, N, device="cuda", dtype=torch.float16)
    ops.gemm([A], [W], [C], M, N, K, lda=K, bias=[b], act="gelu", C2=[C2], ldc2=N)(_lib.stream())
    ref = F.gelu(A.float() @ W.float().T + b)
    assert rel_err(C, ref) < 2e-3
    assert torch.equal(C, C2)


def test_gemm_transposed_operand_layout_catches_swaps():
    """A = I, asymmetric B (guide §3): C must equal B^T exactly."""
    from splatt3r_amd import ops, _lib
    n = 128
    A = torch.eye(n, device="cuda", dtype=torch.float16)
    B = (torch.arange(n * n, device="cuda").view(n, n) % 61).to(torch.float16)
    C = torch.empty(n, n, device="cuda")
    ops.gemm([A], [B], [C], n, n, n, lda=n)(_lib.stream())
    assert torch.equal(C, B.float().T)


@pytest.mark.parametrize("H,W,Cin,Cout,k,stride,relu", [(24, 32, 96, 256, 3, 1, False),
                                                          (12, 16, 768, 768, 3, 2, False),
                                                          (96, 128, 256, 256, 3, 1, True),
                                                          (7, 9, 16, 40, 3, 2, True),
                                                          (10, 12, 128, 16, 1, 1, False)])
def test_gemm_implicit_conv(H, W, Cin, Cout, k, stride, relu):
    from splatt3r_amd import ops, _lib
    B, pad = 2, k // 2
    x = _rand(B, H, W, Cin, seed=3)
    w = _rand(Cout, Cin, k, k, scale=(Cin * k * k) ** -0.5, seed=4)
    b = _rand(Cout, dtype=torch.float32, seed=5)
    oh, ow = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = torch.empty(B, oh, ow, Cout, device="cuda")
    wk = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous()
    conv = dict(H=H, W=W, C=Cin, k=k, stride=stride, pad=pad, oH=oh, oW=ow, relu_in=relu)
    ops.gemm([x], [wk], [out], B * oh * ow, Cout, k * k * Cin, lda=0, bias=[b], conv=conv)(_lib.stream())
    xin = x.float().permute(0, 3, 1, 2)
    if relu:
        xin = xin.clamp_min(0)
    ref = F.conv2d(xin, w.float(), b, stride=stride, padding=pad).permute(0, 2, 3, 1)
    assert rel_err(out, ref) < 1e-5


@pytest.mark.parametrize("s", [4, 2])
def test_gemm_convtranspose_scatter(s):
    from splatt3r_amd import ops, _lib
    B, ht, wt, Cin, Cout = 2, 6, 8, 96, 96
    x = _rand(B, ht, wt, Cin, seed=6)
    w = _rand(Cin, Cout, s, s, scale=Cin ** -0.5, seed=7)
    b = _rand(Cout, dtype=torch.float32, seed=8)
    wk = w.permute(2, 3, 1, 0).reshape(s * s * Cout, Cin).contiguous()
    out = torch.empty(B, ht * s, wt * s, Cout, device="cuda", dtype=torch.float16)
    ops.gemm([x], [wk], [out], B * ht * wt, s * s * Cout, Cin, lda=Cin, bias=[b.repeat(s * s)],
             store=("convt", ht, wt, s, Cout))(_lib.stream())
    ref = F.conv_transpose2d(x.float().permute(0, 3, 1, 2), w.float(), b, stride=s).permute(0, 2, 3, 1)
    assert rel_err(out, ref) < 2e-3


def test_gemm_pixel_shuffle_scatter():
    from splatt3r_amd import ops, _lib
    B, ht, wt, K, p, c = 1, 3, 4, 64, 16, 25
    N = c * p * p
    x = _rand(B * ht * wt, K, seed=9)
    w = _rand(N, K, scale=K ** -0.5, seed=10)
    out = torch.empty(B, ht * p, wt * p, c, device="cuda")
    ops.gemm([x], [w], [out], B * ht * wt, N, K, lda=K, store=("pixshuf", ht, wt, p, c))(_lib.stream())
    lf = (x.float() @ w.float().T).view(B, ht * wt, N).transpose(-1, -2).reshape(B, N, ht, wt)
    ref = F.pixel_shuffle(lf, p).permute(0, 2, 3, 1)  # catmlp_dpt_head.py:263-265
    assert rel_err(out, ref) < 1e-5


def rope_ref(t, pos, cos, sin):
    """croco/models/pos_embed.py:142-159 on [B, H, N, 64]."""
    def rot(x):
        x1, x2 = x[..., :16], x[..., 16:]
        return torch.cat((-x2, x1), -1)

    def r1d(x, p):
        c = F.embedding(p, torch.cat([cos, cos], -1))[:, None]
        s = F.embedding(p, torch.cat([sin, sin], -1))[:, None]
        return x * c + rot(x) * s

    y, xx = t.chunk(2, dim=-1)
    return torch.cat((r1d(y, pos[:, :, 0]), r1d(xx, pos[:, :, 1])), -1)


@pytest.mark.parametrize("B,ht,wt,heads,ncol_heads,groups,tile", [
    (1, 24, 32, 16, 32, 1, 0), (2, 6, 8, 12, 12, 2, 0), (1, 5, 7, 2, 4, 2, 0),
    (1, 24, 32, 16, 32, 1, 21), (1, 24, 32, 12, 12, 2, 24), (2, 6, 8, 12, 12, 2, 30),
    (1, 24, 32, 16, 32, 1, 23)])
def test_gemm_rope_epilogue_vs_torch(B, ht, wt, heads, ncol_heads, groups, tile):
    """QKV projection with RoPE2D fused into the epilogue == linear then
    pos_embed.py's rope on each head of the first rope_ncols columns."""
    from splatt3r_amd import ops, _lib
    from splatt3r_amd.net import positions, rope_tables
    N_tok = ht * wt
    M, K = B * N_tok, 128
    Nout = heads * 64 + 64 * 2          # rotated heads + 2 untouched heads
    ncols = ncol_heads * 64 if ncol_heads <= heads else heads * 64
    ncols = min(ncols, heads * 64)
    cos, sin = rope_tables(64, "cuda")
    pos = [positions(B, ht, wt, "cuda") for _ in range(groups)]
    if groups > 1:
        pos[1] = pos[1].flip(1).contiguous()     # different positions per group
    A = [_rand(M, K, seed=40 + g) for g in range(groups)]
    W = [_rand(Nout, K, scale=K ** -0.5, seed=50 + g) for g in range(groups)]
    b = [_rand(Nout, dtype=torch.float32, seed=60 + g) for g in range(groups)]
    C = [torch.empty(M, Nout, device="cuda") for _ in range(groups)]
    ops.gemm(A, W, C, M, Nout, K, lda=K, bias=b, rope=(cos, sin), rope_pos=pos,
             rope_ncols=ncols, tile=tile)(_lib.stream())
    for g in range(groups):
        lin = A[g].float() @ W[g].float().T + b[g]
        ref = lin.clone()
        hr = ncols // 64
        t = lin[:, :ncols].view(B, N_tok, hr, 64).transpose(1, 2)
        ref[:, :ncols] = rope_ref(t, pos[g], cos, sin).transpose(1, 2).reshape(M, ncols)
        assert rel_err(C[g], ref) < 1e-5, (g, rel_err(C[g], ref))


@pytest.mark.parametrize("B,N,Nk,H,cross", [(1, 768, 768, 16, False), (2, 12, 12, 2, False),
                                             (1, 640, 640, 12, True), (3, 100, 70, 4, True)])
def test_attention_rope_vs_torch(B, N, Nk, H, cross):
    from splatt3r_amd import ops, _lib
    from splatt3r_amd.net import positions, rope_tables
    D = 64
    q = _rand(B * N, H * D, seed=11)
    k = _rand(B * Nk, H * D, seed=12)
    v = _rand(B * Nk, H * D, seed=13)
    o = torch.empty(B * N, H * D, device="cuda", dtype=torch.float16)
    cos, sin = rope_tables(512, "cuda")
    qpos = positions(B, 24, 32, "cuda")[:, :N].contiguous() if N <= 768 else None
    kpos = positions(B, 24, 32, "cuda")
    kpos = (kpos.flip(1) if cross else kpos)[:, :Nk].contiguous()
    if not cross:
        kpos = qpos
    ops.attention([q], [k], [v], [o], B=B, Nq=N, Nk=Nk, H=H, q_stride=H * D, k_stride=H * D,
                  v_stride=H * D, o_stride=H * D, qpos=[qpos], kpos=[kpos], rope=(cos, sin),
                  scale=D ** -0.5)(_lib.stream())
    Q = rope_ref(q.float().view(B, N, H, D).transpose(1, 2), qpos, cos, sin)
    K = rope_ref(k.float().view(B, Nk, H, D).transpose(1, 2), kpos, cos, sin)
    V = v.float().view(B, Nk, H, D).transpose(1, 2)
    ref = ((Q @ K.transpose(-2, -1)) * D ** -0.5).softmax(-1) @ V
    ref = ref.transpose(1, 2).reshape(B * N, H * D)
    # Q/K rotated in fp16 and P rounded to fp16 before P.V: ~1e-3 relative
    assert rel_err(o, ref) < 5e-3, rel_err(o, ref)


@pytest.mark.parametrize("B,N,Nk,H,groups,strided", [(1, 768, 768, 16, 1, True),
                                                     (1, 768, 768, 12, 2, False),
                                                     (2, 100, 70, 4, 1, False),
                                                     (3, 5, 130, 2, 2, True),
                                                     (1, 200, 330, 3, 1, False)])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_attention_no_rope_dma_path(B, N, Nk, H, groups, strided, variant):
    """The LDS-DMA ring kernel (q/k pre-rotated by the GEMM epilogue): plain
    softmax(QK^T s)V, K/V read from strided views like the fused QKV buffer."""
    from splatt3r_amd import ops, _lib
    D = 64
    Qs, Ks, Vs, Os, refs = [], [], [], [], []
    for g in range(groups):
        if strided:
            qkv = _rand(B * max(N, Nk), 3 * H * D, seed=70 + g)
            q, k, v = qkv[:B * N, :H * D], qkv[:B * Nk, H * D:2 * H * D], qkv[:B * Nk, 2 * H * D:]
            qs = ks = vs = 3 * H * D
        else:
            q, k, v = (_rand(B * N, H * D, seed=80 + g), _rand(B * Nk, H * D, seed=90 + g),
                       _rand(B * Nk, H * D, seed=100 + g))
            qs = ks = vs = H * D
        o = torch.empty(B * N, H * D, device="cuda", dtype=torch.float16)
        Qs.append(q); Ks.append(k); Vs.append(v); Os.append(o)
        Qf = q.float().reshape(B, N, H, D).transpose(1, 2)
        Kf = k.float().reshape(B, Nk, H, D).transpose(1, 2)
        Vf = v.float().reshape(B, Nk, H, D).transpose(1, 2)
        r = ((Qf @ Kf.transpose(-2, -1)) * D ** -0.5).softmax(-1) @ Vf
        refs.append(r.transpose(1, 2).reshape(B * N, H * D))
    if strided:   # the sliced views must keep the fused buffer's row stride
        Qs = [t.as_strided((B * N, H * D), (qs, 1)) for t in Qs]
    _lib.lib().s3n_attention_set_variant(variant)
    try:
        ops.attention(Qs, Ks, Vs, Os, B=B, Nq=N, Nk=Nk, H=H, q_stride=qs, k_stride=ks,
                      v_stride=vs, o_stride=H * D, scale=D ** -0.5)(_lib.stream())
    finally:
        _lib.lib().s3n_attention_set_variant(0)
    for g in range(groups):
        assert rel_err(Os[g], refs[g]) < 5e-3, (g, rel_err(Os[g], refs[g]))


def test_layernorm_vs_torch():
    from splatt3r_amd import ops, _lib
    for C in (1024, 768, 128):
        x = _rand(300, C, dtype=torch.float32, seed=14) * 3 + 1
        g = _rand(C, dtype=torch.float32, seed=15)
        b = _rand(C, dtype=torch.float32, seed=16)
        o16 = torch.empty(300, C, device="cuda", dtype=torch.float16)
        o32 = torch.empty(300, C, device="cuda")
        ops.layernorm([x], [g], [b], rows=300, C=C, ldx=C, eps=1e-6, out16=[o16], ld16=C,
                      out32=[o32], ld32=C)(_lib.stream())
        ref = F.layer_norm(x, (C,), g, b, eps=1e-6)
        assert rel_err(o32, ref) < 1e-5
        assert rel_err(o16, ref) < 1e-3


@pytest.mark.parametrize("H,W,oh,ow", [(12, 16, 24, 32), (5, 7, 9, 14), (192, 256, 384, 512)])
def test_upsample_align_corners_vs_torch(H, W, oh, ow):
    from splatt3r_amd import ops, _lib
    x = _rand(2, H, W, 128, seed=17)
    out = torch.empty(2, oh, ow, 128, device="cuda", dtype=torch.float16)
    ops.upsample2x([x], [out], B=2, H=H, W=W, C=128, oh=oh, ow=ow)(_lib.stream())
    ref = F.interpolate(x.float().permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                        align_corners=True)[:, :, :oh, :ow].permute(0, 2, 3, 1)
    assert rel_err(out, ref) < 1e-3


def test_prng_fill_bitexact_vs_numpy():
    from splatt3r_amd import ops
    from splatt3r_amd.weights import prng_numpy, tensor_seed
    t = torch.empty(100_003, device="cuda")
    seed = tensor_seed(1234, "enc_blocks.0.attn.qkv.weight")
    ops.prng_fill(t, seed, 0.0541, 0.0)
    np.testing.assert_array_equal(t.cpu().numpy(), prng_numpy(seed, 100_003, 0.0541, 0.0))


@pytest.mark.parametrize("n", [5000, 1, 256, 257])
def test_gaussian_postprocess_vs_torch(n):
    from splatt3r_amd import ops, _lib
    pts = _rand(n, 16, dtype=torch.float32, seed=18)
    feat = _rand(n, 25, dtype=torch.float32, seed=19)
    gs = _rand(n, 16, dtype=torch.float32, seed=20)
    out = {k: torch.empty(n, c, device="cuda").squeeze(-1) for k, c in
           dict(pts3d=3, conf=1, desc=24, desc_conf=1, scales=3, rotations=4, sh=3,
                opacities=1, means=3).items()}
    desc16 = torch.full((n + 1, 24), 7.0, device="cuda", dtype=torch.float16)
    ops.gaussian_postprocess(n, pts, 16, feat, gs, 16, True, out, desc16=desc16)(_lib.stream())
    # the fp16 copy is the fp32 descriptor rounded, and nothing past row n
    assert torch.equal(desc16[:n], out["desc"].half())
    assert bool((desc16[n] == 7.0).all())
    xyz = pts[:, :3]
    d = xyz.norm(dim=-1, keepdim=True)
    p3 = xyz / d.clip(min=1e-8) * torch.expm1(d)
    off = gs[:, :3]
    od = off.norm(dim=-1, keepdim=True)
    offs = off / od.clip(min=1e-8) * (torch.exp(od - 6) - torch.exp(torch.zeros_like(od) - 6))
    rot = gs[:, 6:10]
    ref = dict(pts3d=p3, conf=1 + pts[:, 3].exp(), desc=feat[:, :24] / feat[:, :24].norm(dim=-1, keepdim=True),
               desc_conf=1 + feat[:, 24].exp(), scales=gs[:, 3:6].exp(),
               rotations=rot / (rot.norm(dim=-1, keepdim=True) + 1e-8), sh=gs[:, 10:13],
               opacities=gs[:, 13].sigmoid(), means=p3 + offs)
    for k, v in ref.items():
        assert rel_err(out[k], v) < 1e-5, k


@pytest.mark.parametrize("case", ["plain", "res16", "split", "rope", "convt", "tile3", "tile4",
                                  "tile16", "tile17_rope", "tile20", "tile65", "tile65_split"])
def test_gemm_vector_epilogue_matches_register_epilogue(case):
    """The LDS-staged 8-column epilogue and the per-register epilogue
    (s3n_gemm_set_debug(16)) apply the same operations in the same order:
    bit-identical outputs."""
    from splatt3r_amd import ops, _lib
    from splatt3r_amd.net import positions, rope_tables
    M, N, K, g = 300, 384, 320, 2
    A = [_rand(M, K, seed=40 + i) for i in range(g)]
    W = [_rand(N, K, scale=K ** -0.5, seed=50 + i) for i in range(g)]
    b = [_rand(N, dtype=torch.float32, seed=60 + i) for i in range(g)]
    kw = dict(lda=K, bias=b, act="gelu")
    out_dt = torch.float32
    if case == "res16":
        kw.update(R1=[_rand(M, N, dtype=torch.float32, seed=70 + i) for i in range(g)], ldr1=N,
                  R2=[_rand(M, N, seed=80 + i) for i in range(g)], ldr2=N, act="none")
        out_dt = torch.float16
    if case == "split":
        kw.update(split_k=3, R1=[_rand(M, N, dtype=torch.float32, seed=70 + i) for i in range(g)],
                  ldr1=N)
    if case == "rope":
        cos, sin = rope_tables(64, "cuda")
        pos = [positions(3, 10, 10, "cuda").reshape(-1, 2) for _ in range(g)]
        kw.update(rope=(cos, sin), rope_pos=pos, rope_ncols=256, act="none")
        out_dt = torch.float16
    if case == "tile3":
        kw.update(tile=3, split_k=1)
    if case == "tile4":
        kw.update(tile=4, split_k=1)
    if case in ("tile16", "tile20", "tile65"):
        kw.update(tile=int(case[4:]), split_k=1)
    if case == "tile65_split":
        kw.update(tile=65, split_k=2, R1=[_rand(M, N, dtype=torch.float32, seed=70 + i)
                                          for i in range(g)], ldr1=N)
    if case == "tile17_rope":
        cos, sin = rope_tables(64, "cuda")
        pos = [positions(3, 10, 10, "cuda").reshape(-1, 2) for _ in range(g)]
        kw.update(rope=(cos, sin), rope_pos=pos, rope_ncols=256, act="none", tile=17)
        out_dt = torch.float16
    if case == "convt":
        s, cout = 2, 96                                  # N = s*s*cout = 384
        kw.update(store=("convt", 15, 20, s, cout), act="none")
        C = [torch.empty(1, 30, 40, cout, device="cuda", dtype=out_dt) for _ in range(g)]
    else:
        C = [torch.empty(M, N, device="cuda", dtype=out_dt) for _ in range(g)]
    C2 = [torch.empty(M, N, device="cuda", dtype=torch.float16) for _ in range(g)]
    if case != "convt":
        kw.update(C2=C2, ldc2=N)
    L = _lib.lib()
    outs = []
    for dbg in (16, 0):
        for c in C:
            c.fill_(0)
        L.s3n_gemm_set_debug(dbg)
        try:
            ops.gemm(A, W, C, M, N, K, **kw)(_lib.stream())
        finally:
            L.s3n_gemm_set_debug(0)
        outs.append([c.clone() for c in C] + ([c.clone() for c in C2] if case != "convt" else []))
    for x, y in zip(*outs):
        if case in ("rope", "tile17_rope"):   # the paths may contract x*cos -/+ x'*sin differently
            assert rel_err(y, x.float()) < 2e-3
        else:
            assert torch.equal(x, y)


@pytest.mark.parametrize("tile,tn,store_c", [(3, 16, False), (2, 16, True), (4, 8, False),
                                             (0, 16, False), (63, 16, False), (65, 8, True)])
def test_gemm_conv_fused_1x1_tail(tile, tn, store_c):
    """conv3x3 + bias + ReLU with the 1x1 conv fused in the epilogue (the DPT
    head's last two convs, dpt_block.py:321-323) vs torch fp32."""
    from splatt3r_amd import ops, _lib
    B, H, W, Cin, Cout, g = 1, 20, 28, 128, 128, 2
    xs = [_rand(B, H, W, Cin, seed=31 + i) for i in range(g)]
    ws = [_rand(Cout, Cin, 3, 3, scale=(Cin * 9) ** -0.5, seed=41 + i) for i in range(g)]
    bs = [_rand(Cout, dtype=torch.float32, seed=51 + i) for i in range(g)]
    tw = [_rand(tn, Cout, scale=Cout ** -0.5, seed=61 + i) for i in range(g)]
    tb = [_rand(tn, dtype=torch.float32, seed=71 + i) for i in range(g)]
    out = [torch.empty(B * H * W, tn, device="cuda") for _ in range(g)]
    C = [torch.empty(B, H, W, Cout, device="cuda", dtype=torch.float16) if store_c else None
         for _ in range(g)]
    wk = [w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous() for w in ws]
    conv = dict(H=H, W=W, C=Cin, k=3, stride=1, pad=1, oH=H, oW=W)
    ops.gemm(xs, wk, C, B * H * W, Cout, 9 * Cin, lda=0, conv=conv, bias=bs, act="relu",
             tile=tile, tail=(tw, tb, out, tn, tn))(_lib.stream())
    for i in range(g):
        y = F.relu(F.conv2d(xs[i].float().permute(0, 3, 1, 2), ws[i].float(), bs[i], padding=1))
        ref = y.permute(0, 2, 3, 1).reshape(-1, Cout) @ tw[i].float().T + tb[i]
        assert rel_err(out[i], ref) < 2e-3, (i, rel_err(out[i], ref))
        if store_c:
            assert rel_err(C[i], y.permute(0, 2, 3, 1)) < 2e-3


@pytest.mark.parametrize("tile,B,H,W,Cin,Cout,relu,res,tail", [
    (40, 2, 5, 256, 128, 128, True, False, False), (41, 1, 4, 256, 128, 128, False, True, False),
    (42, 1, 6, 128, 256, 256, True, True, False), (40, 1, 7, 128, 64, 128, False, False, True),
    (42, 2, 3, 256, 128, 128, True, False, True), (41, 1, 3, 512, 128, 64, False, False, False),
    (43, 2, 5, 256, 128, 128, True, True, True), (43, 1, 4, 256, 256, 128, True, False, False),
    (45, 1, 6, 128, 128, 128, False, True, True), (46, 2, 3, 256, 128, 128, True, True, True),
    (47, 1, 4, 256, 256, 128, True, False, False), (48, 1, 5, 128, 128, 128, True, True, True),
    (49, 2, 4, 128, 256, 128, False, True, True), (50, 1, 3, 256, 128, 64, True, False, False),
    (51, 2, 5, 256, 128, 128, True, True, True), (52, 1, 4, 128, 256, 128, False, False, True),
    (53, 1, 3, 512, 128, 128, True, True, False)])
def test_gemm_halo_conv_vs_torch(tile, B, H, W, Cin, Cout, relu, res, tail):
    """Halo-reuse 3x3 conv tiles (net_gemm_t6.hip: one input row segment per
    (ky, channel chunk) serves the three kx taps) vs torch fp32: bias, ReLU on
    the input, residual operands, the fused 1x1 tail, image edges (top and
    bottom rows, the first and last column of every segment), two images."""
    from splatt3r_amd import ops, _lib
    g = 2
    xs = [_rand(B, H, W, Cin, seed=81 + i) for i in range(g)]
    ws = [_rand(Cout, Cin, 3, 3, scale=(Cin * 9) ** -0.5, seed=83 + i) for i in range(g)]
    bs = [_rand(Cout, dtype=torch.float32, seed=85 + i) for i in range(g)]
    r1 = [_rand(B, H, W, Cout, dtype=torch.float32, seed=87 + i) for i in range(g)] if res else None
    wk = [w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous() for w in ws]
    out = [torch.empty(B, H, W, Cout, device="cuda") for _ in range(g)]
    conv = dict(H=H, W=W, C=Cin, k=3, stride=1, pad=1, oH=H, oW=W, relu_in=relu)
    kw = dict(lda=0, conv=conv, bias=bs, act="relu" if tail else "none", tile=tile, split_k=1)
    if res:
        kw.update(R1=r1, ldr1=Cout)
    tn = 16
    if tail:
        tw = [_rand(tn, Cout, scale=Cout ** -0.5, seed=89 + i) for i in range(g)]
        tb = [_rand(tn, dtype=torch.float32, seed=91 + i) for i in range(g)]
        tout = [torch.empty(B * H * W, tn, device="cuda") for _ in range(g)]
        kw["tail"] = (tw, tb, tout, tn, tn)
    ops.gemm(xs, wk, out, B * H * W, Cout, 9 * Cin, **kw)(_lib.stream())
    for i in range(g):
        xin = xs[i].float().permute(0, 3, 1, 2)
        if relu:
            xin = xin.clamp_min(0)
        y = F.conv2d(xin, ws[i].float(), bs[i], padding=1).permute(0, 2, 3, 1)
        if tail:
            y = F.relu(y)
        if res:
            y = y + r1[i]
        assert rel_err(out[i], y) < 1e-5, (i, rel_err(out[i], y))
        if tail:
            ref = y.reshape(-1, Cout) @ tw[i].float().T + tb[i]
            assert rel_err(tout[i], ref) < 2e-5, (i, rel_err(tout[i], ref))


def test_gemm_halo_conv_rejects_unsupported_shapes():
    """A halo tile on a shape it cannot tile (segment not dividing the width,
    stride 2, Cin % 64 != 0, dense A) fails loudly; the tuner skips it."""
    from splatt3r_amd import ops, _lib
    x = _rand(1, 4, 96, 128, seed=1)
    w = _rand(128, 9 * 128, scale=0.03, seed=2)
    out = torch.empty(1, 4, 96, 128, device="cuda")
    conv = dict(H=4, W=96, C=128, k=3, stride=1, pad=1, oH=4, oW=96)
    with pytest.raises(RuntimeError):
        ops.gemm([x], [w], [out], 4 * 96, 128, 9 * 128, lda=0, conv=conv, tile=40,
                 split_k=1)(_lib.stream())
    with pytest.raises(RuntimeError):
        ops.gemm([x.view(384, 128)], [w[:, :128].contiguous()], [out.view(384, 128)], 384, 128,
                 128, lda=128, tile=40, split_k=1)(_lib.stream())


def test_gemm_and_layernorm_fp16_range_guard():
    """fp16 activations saturate at +-65504 (not inf) and raise the device
    flag s3n_f16_saturations reports; in-range outputs leave it clear."""
    from splatt3r_amd import ops, _lib
    ops.f16_saturations(reset=True)
    M, N, K = 128, 128, 64
    A = torch.full((M, K), 60.0, device="cuda", dtype=torch.float16)
    W = torch.full((N, K), 60.0, device="cuda", dtype=torch.float16)   # dot = 230400
    C = torch.empty(M, N, device="cuda", dtype=torch.float16)
    ops.gemm([A], [W * 0.001], [C], M, N, K, lda=K)(_lib.stream())
    assert ops.f16_saturations(reset=True) == 0
    assert torch.isfinite(C).all()
    ops.gemm([A], [W], [C], M, N, K, lda=K)(_lib.stream())
    assert ops.f16_saturations(reset=True) == 1
    assert float(C.float().max()) == 65504.0 and torch.isfinite(C).all()
    assert ops.f16_saturations() == 0
    x = torch.zeros(4, 256, device="cuda")
    x[:, 0] = 1.0
    g = torch.full((256,), 1e5, device="cuda")
    o = torch.empty(4, 256, device="cuda", dtype=torch.float16)
    ops.layernorm([x], [g], [torch.zeros(256, device="cuda")], rows=4, C=256, ldx=256,
                  out16=[o], ld16=256)(_lib.stream())
    assert ops.f16_saturations(reset=True) == 1 and torch.isfinite(o).all()
