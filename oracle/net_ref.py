"""ORACLE — test infrastructure only.  Plain-torch fp32 restatement of the
MASt3RGaussians inference forward on a reference-layout state_dict, used
(a) as the `cpu_baseline` leg of bench.py (the reference's own PyTorch-CPU
path cannot travel to the GPU box) and (b) as a second parity reference.
Pinned against the reference modules by tests/test_net_ref.py via
tests/golden/net_small_*.npz.

Restated (splatt3r_core/src/mast3r_src/...):
  dust3r/dust3r/patch_embed.py:42-70, dust3r/dust3r/model.py:121-193,
  dust3r/croco/models/blocks.py:58-191, pos_embed.py:106-159 (RoPE2D),
  dust3r/croco/models/dpt_block.py:20-450, dust3r/dust3r/heads/dpt_head.py:34-65,
  mast3r/catmlp_dpt_head.py:97-278, dust3r/dust3r/heads/postprocess.py:22-58.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _rope(t, pos, base=100.0):
    D = t.shape[-1] // 2
    inv = 1.0 / (base ** (torch.arange(0, D, 2).float() / D))
    tt = torch.arange(int(pos.max()) + 1, dtype=inv.dtype)
    fr = torch.einsum("i,j->ij", tt, inv)
    fr = torch.cat((fr, fr), -1)
    cos, sin = fr.cos(), fr.sin()

    def r1(x, p):
        c = F.embedding(p, cos)[:, None]
        s = F.embedding(p, sin)[:, None]
        x1, x2 = x[..., :x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
        return x * c + torch.cat((-x2, x1), -1) * s

    y, x = t.chunk(2, dim=-1)
    return torch.cat((r1(y, pos[:, :, 0]), r1(x, pos[:, :, 1])), -1)


def _ln(sd, p, x):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps=1e-6)


def _lin(sd, p, x):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


def _attn(q, k, v):
    a = (q @ k.transpose(-2, -1)) * q.shape[-1] ** -0.5
    return a.softmax(-1) @ v


def _self_attn(sd, p, x, pos, heads):
    B, N, C = x.shape
    qkv = _lin(sd, p + ".qkv", x).reshape(B, N, 3, heads, C // heads).transpose(1, 3)
    q, k, v = [qkv[:, :, i] for i in range(3)]
    o = _attn(_rope(q, pos), _rope(k, pos), v).transpose(1, 2).reshape(B, N, C)
    return _lin(sd, p + ".proj", o)


def _cross_attn(sd, p, x, y, xpos, ypos, heads):
    B, N, C = x.shape
    sh = lambda t: t.reshape(B, -1, heads, C // heads).permute(0, 2, 1, 3)
    q = sh(_lin(sd, p + ".projq", x))
    k = sh(_lin(sd, p + ".projk", y))
    v = sh(_lin(sd, p + ".projv", y))
    o = _attn(_rope(q, xpos), _rope(k, ypos), v).transpose(1, 2).reshape(B, N, C)
    return _lin(sd, p + ".proj", o)


def _mlp(sd, p, x):
    return _lin(sd, p + ".fc2", F.gelu(_lin(sd, p + ".fc1", x)))


def encode(sd, cfg, img):
    B, _, H, W = img.shape
    p = cfg.patch
    x = F.conv2d(img, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=p)
    ht, wt = x.shape[-2:]
    x = x.permute(0, 2, 3, 1).flatten(1, 2)
    pos = torch.cartesian_prod(torch.arange(ht), torch.arange(wt)).view(1, -1, 2).expand(B, -1, 2)
    for i in range(cfg.enc_depth):
        b = f"enc_blocks.{i}"
        x = x + _self_attn(sd, b + ".attn", _ln(sd, b + ".norm1", x), pos, cfg.enc_heads)
        x = x + _mlp(sd, b + ".mlp", _ln(sd, b + ".norm2", x))
    return _ln(sd, "enc_norm", x), pos


def decode(sd, cfg, f1, p1, f2, p2):
    out = [(f1, f2)]
    x1, x2 = _lin(sd, "decoder_embed", f1), _lin(sd, "decoder_embed", f2)
    out.append((x1, x2))
    for i in range(cfg.dec_depth):
        pr = out[-1]
        res = []
        for name, (x, y, xp, yp) in (("dec_blocks", (pr[0], pr[1], p1, p2)),
                                     ("dec_blocks2", (pr[1], pr[0], p2, p1))):
            b = f"{name}.{i}"
            x = x + _self_attn(sd, b + ".attn", _ln(sd, b + ".norm1", x), xp, cfg.dec_heads)
            y_ = _ln(sd, b + ".norm_y", y)
            x = x + _cross_attn(sd, b + ".cross_attn", _ln(sd, b + ".norm2", x), y_, xp, yp,
                                cfg.dec_heads)
            x = x + _mlp(sd, b + ".mlp", _ln(sd, b + ".norm3", x))
            res.append(x)
        out.append(tuple(res))
    del out[1]
    out[-1] = (_ln(sd, "dec_norm", out[-1][0]), _ln(sd, "dec_norm", out[-1][1]))
    return [o[0] for o in out], [o[1] for o in out]


def _conv(sd, p, x, stride=1, padding=None):
    w = sd[p + ".weight"]
    pad = w.shape[-1] // 2 if padding is None else padding
    return F.conv2d(x, w, sd.get(p + ".bias"), stride=stride, padding=pad)


def _rcu(sd, p, x):
    out = _conv(sd, p + ".conv1", F.relu(x))
    out = _conv(sd, p + ".conv2", F.relu(out))
    return out + x


def _ffb(sd, p, *xs):
    out = xs[0]
    if len(xs) == 2:
        out = out + _rcu(sd, p + ".resConfUnit1", xs[1])
    out = _rcu(sd, p + ".resConfUnit2", out)
    out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    return _conv(sd, p + ".out_conv", out)


def dpt(sd, p, cfg, tokens, H, W):
    ht, wt = H // cfg.patch, W // cfg.patch
    layers = [tokens[h] for h in cfg.hooks]
    layers = [l.transpose(1, 2).reshape(l.shape[0], -1, ht, wt) for l in layers]
    ap = p + ".act_postprocess"
    l0 = F.conv_transpose2d(_conv(sd, ap + ".0.0", layers[0]), sd[ap + ".0.1.weight"],
                            sd[ap + ".0.1.bias"], stride=4)
    l1 = F.conv_transpose2d(_conv(sd, ap + ".1.0", layers[1]), sd[ap + ".1.1.weight"],
                            sd[ap + ".1.1.bias"], stride=2)
    l2 = _conv(sd, ap + ".2.0", layers[2])
    l3 = _conv(sd, ap + ".3.1", _conv(sd, ap + ".3.0", layers[3]), stride=2, padding=1)
    ls = [_conv(sd, f"{p}.scratch.layer{i + 1}_rn", l) for i, l in enumerate((l0, l1, l2, l3))]
    s = p + ".scratch"
    p4 = _ffb(sd, s + ".refinenet4", ls[3])[:, :, :ls[2].shape[2], :ls[2].shape[3]]
    p3 = _ffb(sd, s + ".refinenet3", p4, ls[2])
    p2 = _ffb(sd, s + ".refinenet2", p3, ls[1])
    p1 = _ffb(sd, s + ".refinenet1", p2, ls[0])
    h = _conv(sd, p + ".head.0", p1)
    h = F.interpolate(h, scale_factor=2, mode="bilinear", align_corners=True)
    h = F.relu(_conv(sd, p + ".head.2", h))
    return _conv(sd, p + ".head.4", h)


def head(sd, cfg, hn, decout, H, W):
    hp = f"downstream_head{hn}"
    pts = dpt(sd, hp + ".dpt", cfg, decout, H, W)
    cat = torch.cat([decout[0], decout[-1]], -1)
    B, S, _ = cat.shape
    lf = _mlp(sd, hp + ".head_local_features", cat)
    lf = lf.transpose(-1, -2).reshape(B, -1, H // cfg.patch, W // cfg.patch)
    lf = F.pixel_shuffle(lf, cfg.patch)
    gs = dpt(sd, hp + ".gaussian_dpt.dpt", cfg, decout, H, W)
    fmap = torch.cat([pts, lf, gs], 1).permute(0, 2, 3, 1)
    pts3d, conf, desc, dconf, off, scales, rot, sh, opac = torch.split(
        fmap, [3, 1, cfg.desc_dim, 1, 3, 3, 4, 3 * cfg.sh_degree, 1], -1)
    d = pts3d.norm(dim=-1, keepdim=True)
    pts3d = pts3d / d.clip(min=1e-8) * torch.expm1(d)
    od = off.norm(dim=-1, keepdim=True)
    off = off / od.clip(min=1e-8) * (torch.exp(od - 6.0) - torch.exp(torch.zeros_like(od) - 6.0))
    res = dict(pts3d=pts3d, conf=1 + conf[..., 0].exp(), desc=desc / desc.norm(dim=-1, keepdim=True),
               desc_conf=1 + dconf[..., 0].exp(), scales=scales.exp(),
               rotations=rot / (rot.norm(dim=-1, keepdim=True) + 1e-8),
               sh=sh.reshape(*sh.shape[:-1], 3, cfg.sh_degree), opacities=opac.sigmoid())
    res["means"] = pts3d + off if cfg.use_offsets else pts3d
    return res


@torch.no_grad()
def frame_forward(sd, cfg, img_f, feat_k, pos_k):
    """One tracked frame's network work (encoder on the new frame, decoder +
    both heads against the cached keyframe features), as
    splatt3r_match_asymmetric does (splatt3r_utils.py:580-644)."""
    H, W = img_f.shape[-2:]
    f, p = encode(sd, cfg, img_f)
    d1, d2 = decode(sd, cfg, f, p, feat_k, pos_k)
    return head(sd, cfg, 1, d1, H, W), head(sd, cfg, 2, d2, H, W)
