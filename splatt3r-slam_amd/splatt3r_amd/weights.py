"""MASt3RGaussians weights: state_dict manifest, portable PRNG init, checkpoint
loading, and repacking into the kernel layouts.

There is no network here and the Splatt3R checkpoint is not in the image, so
benchmarks and parity tests use *portable-PRNG* weights: every state_dict
tensor (reference names, splatt3r_core/main.py:54-71 architecture) is
filled by a counter-based splitmix64 stream seeded from the tensor's name,
w = (2u - 1) a + c.  The same stream is produced on the GPU
(s3n_prng_fill) and in numpy (prng_numpy below, used by
oracle/gen_golden.py to load identical weights into the reference
modules), so the 2.9 GB of weights never has to be shipped.
A real checkpoint (safetensors, or a torch state_dict loadable with
weights_only=True) can be loaded instead with load_state_dict_file().
"""
from __future__ import annotations

import dataclasses
import math
import os

import numpy as np
import torch

GOLDEN = 0x9E3779B97F4A7C15
MASK64 = (1 << 64) - 1


@dataclasses.dataclass(frozen=True)
class NetConfig:
    """Splatt3R's AsymmetricMASt3R arguments (splatt3r_core/main.py:54-71)."""
    enc_dim: int = 1024
    enc_depth: int = 24
    enc_heads: int = 16
    dec_dim: int = 768
    dec_depth: int = 12
    dec_heads: int = 12
    patch: int = 16
    mlp_ratio: float = 4.0
    desc_dim: int = 24
    sh_degree: int = 1
    use_offsets: bool = True
    feature_dim: int = 256
    layer_dims: tuple = (96, 192, 384, 768)
    rope_base: float = 100.0
    ln_eps: float = 1e-6
    # portable-PRNG init of the two final 1x1 convs (not architecture):
    # (channels, xavier gain, bias) per split of the Gaussian head's final
    # conv, and an optional constant added to the pts head's x, y, z bias.
    # The defaults are the reference init (catmlp_dpt_head.py:222-238);
    # N1_INIT is the conditioned variant of the N1 render fixture.
    gauss_splits: tuple = ((3, 0.001, 0.001), (3, 0.00003, -7.0), (4, 1.0, 0.0),
                           (3, 1.0, 0.0), (1, 1.0, -2.0))
    pts_bias: tuple = None

    @property
    def hooks(self):  # catmlp_dpt_head.py:317
        l2 = self.dec_depth
        return (0, l2 * 2 // 4, l2 * 3 // 4, l2)

    @property
    def gauss_channels(self):  # catmlp_dpt_head.py:215
        return 3 + 3 + 4 + 3 * self.sh_degree + 1


FULL = NetConfig()
# The reduced configuration the golden fixtures use (dec_depth > 9 is
# asserted by the reference head factory; head_dim stays 64).
SMALL = NetConfig(enc_dim=128, enc_depth=2, enc_heads=2, dec_dim=128, dec_depth=12, dec_heads=2)


def n1_init(cfg: NetConfig, scale_bias: float) -> NetConfig:
    """The N1 render fixture's init (oracle/gen_golden.py `n1`):
    with the reference init the Gaussian head's scales are a constant e^-7
    (xavier gain 3e-5, bias -7: sub-pixel splats, opacity sigmoid(-2)) and
    the rendered image is a step function of the means.  Trained weights
    give multi-pixel, varying splats; this init gets there with the same
    PRNG streams: scale gain 0.2 and bias `scale_bias` (per resolution:
    splats of ~10-30 px), SH residual gain 0.05 (the colour comes from the
    image, as after training), opacity bias 0, and +0.3 on the pts head's
    z bias (points in front of the camera)."""
    return dataclasses.replace(
        cfg, gauss_splits=((3, 0.001, 0.001), (3, 0.2, scale_bias), (4, 1.0, 0.0),
                           (3, 0.05, 0.0), (1, 1.0, 0.0)), pts_bias=(0.0, 0.0, 0.3))


# ------------------------------------------------------------ manifest ----
def manifest(cfg: NetConfig) -> list[tuple[str, tuple]]:
    """(name, shape) of AsymmetricMASt3R.state_dict(), reference order."""
    E, D, p = cfg.enc_dim, cfg.dec_dim, cfg.patch
    hE, hD = int(E * cfg.mlp_ratio), int(D * cfg.mlp_ratio)
    out = [("mask_token", (1, 1, D)), ("patch_embed.proj.weight", (E, 3, p, p)),
           ("patch_embed.proj.bias", (E,))]

    def lin(pre, o, i, bias=True):
        out.append((pre + ".weight", (o, i)))
        if bias:
            out.append((pre + ".bias", (o,)))

    def ln(pre, c):
        out.append((pre + ".weight", (c,)))
        out.append((pre + ".bias", (c,)))

    for i in range(cfg.enc_depth):
        b = f"enc_blocks.{i}"
        ln(b + ".norm1", E)
        lin(b + ".attn.qkv", 3 * E, E)
        lin(b + ".attn.proj", E, E)
        ln(b + ".norm2", E)
        lin(b + ".mlp.fc1", hE, E)
        lin(b + ".mlp.fc2", E, hE)
    ln("enc_norm", E)
    lin("decoder_embed", D, E)

    def dec_block(b):
        ln(b + ".norm1", D)
        lin(b + ".attn.qkv", 3 * D, D)
        lin(b + ".attn.proj", D, D)
        lin(b + ".cross_attn.projq", D, D)
        lin(b + ".cross_attn.projk", D, D)
        lin(b + ".cross_attn.projv", D, D)
        lin(b + ".cross_attn.proj", D, D)
        ln(b + ".norm2", D)
        ln(b + ".norm3", D)
        lin(b + ".mlp.fc1", hD, D)
        lin(b + ".mlp.fc2", D, hD)
        ln(b + ".norm_y", D)

    for i in range(cfg.dec_depth):
        dec_block(f"dec_blocks.{i}")
    ln("dec_norm", D)
    for i in range(cfg.dec_depth):
        dec_block(f"dec_blocks2.{i}")
    for h in (1, 2):
        hp = f"downstream_head{h}"
        _dpt_manifest(out, hp + ".dpt", cfg, 3 + 1)
        idim = E + D
        lin(hp + ".head_local_features.fc1", int(4 * idim), idim)
        lin(hp + ".head_local_features.fc2", (cfg.desc_dim + 1) * p * p, int(4 * idim))
        _dpt_manifest(out, hp + ".gaussian_dpt.dpt", cfg, cfg.gauss_channels)
    return out


def _dpt_manifest(out, pre, cfg, nch):
    F = cfg.feature_dim
    ld = cfg.layer_dims
    dims = (cfg.enc_dim, cfg.dec_dim, cfg.dec_dim, cfg.dec_dim)
    for i in range(4):
        out.append((f"{pre}.scratch.layer{i + 1}_rn.weight", (F, ld[i], 3, 3)))
    for i in range(4):
        out.append((f"{pre}.scratch.layer_rn.{i}.weight", (F, ld[i], 3, 3)))
    for r in (1, 2, 3, 4):
        rp = f"{pre}.scratch.refinenet{r}"
        out.append((rp + ".out_conv.weight", (F, F, 1, 1)))
        out.append((rp + ".out_conv.bias", (F,)))
        for u in (1, 2):
            for c in (1, 2):
                out.append((f"{rp}.resConfUnit{u}.conv{c}.weight", (F, F, 3, 3)))
                out.append((f"{rp}.resConfUnit{u}.conv{c}.bias", (F,)))
    out.append((f"{pre}.head.0.weight", (F // 2, F, 3, 3)))
    out.append((f"{pre}.head.0.bias", (F // 2,)))
    out.append((f"{pre}.head.2.weight", (F // 2, F // 2, 3, 3)))
    out.append((f"{pre}.head.2.bias", (F // 2,)))
    out.append((f"{pre}.head.4.weight", (nch, F // 2, 1, 1)))
    out.append((f"{pre}.head.4.bias", (nch,)))
    ap = f"{pre}.act_postprocess"
    out.append((f"{ap}.0.0.weight", (ld[0], dims[0], 1, 1)))
    out.append((f"{ap}.0.0.bias", (ld[0],)))
    out.append((f"{ap}.0.1.weight", (ld[0], ld[0], 4, 4)))
    out.append((f"{ap}.0.1.bias", (ld[0],)))
    out.append((f"{ap}.1.0.weight", (ld[1], dims[1], 1, 1)))
    out.append((f"{ap}.1.0.bias", (ld[1],)))
    out.append((f"{ap}.1.1.weight", (ld[1], ld[1], 2, 2)))
    out.append((f"{ap}.1.1.bias", (ld[1],)))
    out.append((f"{ap}.2.0.weight", (ld[2], dims[2], 1, 1)))
    out.append((f"{ap}.2.0.bias", (ld[2],)))
    out.append((f"{ap}.3.0.weight", (ld[3], dims[3], 1, 1)))
    out.append((f"{ap}.3.0.bias", (ld[3],)))
    out.append((f"{ap}.3.1.weight", (ld[3], ld[3], 3, 3)))
    out.append((f"{ap}.3.1.bias", (ld[3],)))


def canonical(name: str) -> str:
    """scratch.layer_rn.{i} is the same tensor as scratch.layer{i+1}_rn."""
    if ".scratch.layer_rn." in name:
        pre, rest = name.split(".scratch.layer_rn.")
        i, tail = rest.split(".", 1)
        return f"{pre}.scratch.layer{int(i) + 1}_rn.{tail}"
    return name


# ---------------------------------------------------------- PRNG spec -----
def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & MASK64
    return h


def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def tensor_seed(global_seed: int, name: str) -> int:
    return mix64(fnv1a64(name) ^ mix64(global_seed & MASK64))


def _fans(shape):
    rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    return shape[1] * rf, shape[0] * rf


# final Gaussian conv: (channels, xavier gain, bias) per split,
# catmlp_dpt_head.py:222-238
GAUSS_SPLITS = FULL.gauss_splits


def init_spec(name: str, shape: tuple, cfg: NetConfig = FULL) -> list[tuple[str, int, float, float]]:
    """List of (stream name, numel, a, c) chunks that fill the tensor in order."""
    n = int(np.prod(shape))
    if cfg.pts_bias is not None and name.endswith(".dpt.head.4.bias") \
            and ".gaussian_dpt." not in name:
        # the same stream and scale as the default; chunk k = one channel
        # with its constant (pts x, y, z, conf)
        off = tuple(cfg.pts_bias) + (0.0,) * (n - len(cfg.pts_bias))
        return [(f"{name}#{k}", 1, 0.02, off[k]) for k in range(n)]
    if name.endswith("gaussian_dpt.dpt.head.4.weight") or name.endswith("gaussian_dpt.dpt.head.4.bias"):
        chunks = []
        per = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        for k, (nc, gain, bias) in enumerate(cfg.gauss_splits):
            if name.endswith("weight"):
                fi, fo = per, nc * int(np.prod(shape[2:]))
                a = gain * math.sqrt(6.0 / (fi + fo))
                chunks.append((f"{name}#{k}", nc * per, a, 0.0))
            else:
                chunks.append((f"{name}#{k}", nc, 0.0, bias))
        return chunks
    leaf = name.rsplit(".", 1)[-1]
    is_norm = any(t in name for t in ("norm", "enc_norm", "dec_norm")) and len(shape) == 1
    if is_norm and leaf == "weight":
        return [(name, n, 0.1, 1.0)]
    if is_norm and leaf == "bias":
        return [(name, n, 0.05, 0.0)]
    if leaf == "bias":
        return [(name, n, 0.02, 0.0)]
    if name == "mask_token":
        return [(name, n, 0.02, 0.0)]
    fi, fo = _fans(shape)
    a = math.sqrt(6.0 / (fi + fo))
    if ".dpt." in name and "head.4" not in name:
        # xavier x 0.7 inside the DPTs keeps the refinenet residual chain at
        # O(1) with the decoder's raw hook tokens (gain 1.0 drives pts3d to
        # ~1e5 via expm1; 0.7 gives ~1 m depths, conf ~2.4, opacity ~0.12).
        a *= DPT_GAIN
    return [(name, n, a, 0.0)]


DPT_GAIN = 0.7


def prng_numpy(seed: int, n: int, a: float, c: float) -> np.ndarray:
    """numpy twin of s3n_prng_fill (bit-exact; float32 arithmetic)."""
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(5.9604644775390625e-08)
    t = u * np.float32(2.0)
    w = t - np.float32(1.0)
    y = w * np.float32(a)
    return y + np.float32(c)


def prng_tensor_numpy(global_seed: int, name: str, shape: tuple, cfg: NetConfig = FULL) -> np.ndarray:
    parts = [prng_numpy(tensor_seed(global_seed, s), n, a, c)
             for s, n, a, c in init_spec(canonical(name), shape, cfg)]
    return np.concatenate(parts).reshape(shape)


def prng_state_dict(cfg: NetConfig, seed: int, device) -> dict[str, torch.Tensor]:
    """All state_dict tensors filled on the GPU by s3n_prng_fill."""
    from splatt3r_amd import ops
    sd = {}
    for name, shape in manifest(cfg):
        cname = canonical(name)
        if cname != name and cname in sd:
            sd[name] = sd[cname]
            continue
        t = torch.empty(int(np.prod(shape)), device=device, dtype=torch.float32)
        off = 0
        for s, n, a, c in init_spec(cname, shape, cfg):
            ops.prng_fill(t[off:off + n], tensor_seed(seed, s), a, c)
            off += n
        sd[name] = t.view(shape)
    return sd


def load_state_dict_file(path: str, device) -> dict[str, torch.Tensor]:
    """Load real weights without executing anything from the file:
    safetensors, or torch.load(weights_only=True).  Accepts the Lightning
    layout (keys under 'state_dict', prefixed 'encoder.')."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path, device="cpu")
    else:
        obj = torch.load(path, map_location="cpu", weights_only=True, mmap=True)
        sd = obj.get("state_dict", obj) if isinstance(obj, dict) else obj
    out = {}
    for k, v in sd.items():
        if k.startswith("encoder."):
            k = k[len("encoder."):]
        out[k] = v.to(device=device, dtype=torch.float32)
    return out


def check_state_dict(cfg: NetConfig, sd: dict) -> None:
    missing = [n for n, _ in manifest(cfg) if n not in sd and n != "mask_token"]
    bad = [(n, tuple(sd[n].shape), s) for n, s in manifest(cfg)
           if n in sd and tuple(sd[n].shape) != tuple(s)]
    if missing or bad:
        raise ValueError(f"state_dict mismatch: missing={missing[:5]}... bad={bad[:5]}")


def tie_symmetric(sd: dict) -> dict:
    """Make the two decoder branches and the two heads share weights
    (dec_blocks2 := dec_blocks, downstream_head2 := downstream_head1).

    Same architecture and the same compute; used by bench.py so that, with
    portable-PRNG weights, the cross prediction of a view agrees with the
    self prediction of a nearby view (as trained weights make it) and the
    tracker's matching/GN run with realistic trip counts.  Parity tests use
    the untied weights."""
    for name in list(sd):
        for a, b in (("dec_blocks2.", "dec_blocks."), ("downstream_head2.", "downstream_head1.")):
            if name.startswith(a):
                sd[name] = sd[b + name[len(a):]]
    return sd
