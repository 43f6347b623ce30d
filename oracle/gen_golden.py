"""Generate the golden fixtures under tests/golden/ by importing the Python
reference from /root/reference (this container only; the GPU box never reads
/root/reference).  Committed outputs are data only (inputs + expected
outputs), never reference source.

  python oracle/gen_golden.py [section ...]     sections: matching, net, render

matching : splatt3r_slam/image.py img_gradient (imported) driven exactly as
           splatt3r_slam/matching.py:25-49 prep_for_iter_proj does.
net      : see gen_net() — reduced-size MASt3RGaussians forward with
           portable-PRNG weights (oracle/prng.py).
render   : see gen_render() — rasterizer boundary inputs captured through a
           stub diff_gaussian_rasterization module.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _load_file(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def gen_matching():
    img = _load_file("ref_image", os.path.join(REF, "splatt3r_slam", "image.py"))
    g = torch.Generator().manual_seed(0)
    b, h, w = 2, 12, 16
    X11 = torch.randn(b, h, w, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0])
    X21 = torch.randn(b, h, w, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0])
    # matching.py:25-49
    rays_img = F.normalize(X11, dim=-1).permute(0, 3, 1, 2)
    gx, gy = img.img_gradient(rays_img)
    rays_with_grad = torch.cat((rays_img, gx, gy), dim=1).permute(0, 2, 3, 1).contiguous()
    pts = F.normalize(X21.view(b, -1, 3), dim=-1)
    np.savez_compressed(os.path.join(GOLDEN, "matching_prep.npz"),
                        X11=X11.numpy(), X21=X21.numpy(),
                        rays_with_grad=rays_with_grad.numpy(), pts3d_norm=pts.numpy())
    print("wrote matching_prep.npz")


def gen_render():
    """Capture the rasterizer boundary of the reference splat-decoder glue.

    A stub `diff_gaussian_rasterization` is injected into sys.modules; the
    reference's decoder_splatting_cuda.py / cuda_splatting.py / projection.py
    and utils/geometry.py + utils/sh_utils.py are imported from
    /root/reference and driven exactly as splatt3r_slam/splatt3r_utils.py:332-432
    (splatt3r_render) drives them.  Saved: the settings the glue builds and
    the tensors it hands to GaussianRasterizer.
    """
    import types
    captured = {}

    class Settings(tuple):
        def __new__(cls, **kw):
            o = tuple.__new__(cls, tuple(kw.values()))
            o.kw = kw
            return o

    class Rasterizer(torch.nn.Module):
        def __init__(self, rs):
            super().__init__()
            self.rs = rs

        def forward(self, **kw):
            captured["settings"] = self.rs.kw
            captured["inputs"] = kw
            h, w = self.rs.kw["image_height"], self.rs.kw["image_width"]
            return torch.zeros(3, h, w), torch.zeros(kw["means3D"].shape[0], dtype=torch.int32)

    stub = types.ModuleType("diff_gaussian_rasterization")
    stub.GaussianRasterizationSettings = Settings
    stub.GaussianRasterizer = Rasterizer
    sys.modules["diff_gaussian_rasterization"] = stub
    core = os.path.join(REF, "splatt3r_core")
    ps = os.path.join(core, "src", "pixelsplat_src")
    for p in (ps, core):
        if p not in sys.path:
            sys.path.insert(0, p)
    dec = _load_file("ref_decoder_splatting_cuda", os.path.join(ps, "decoder_splatting_cuda.py"))
    geo = _load_file("ref_geometry", os.path.join(core, "utils", "geometry.py"))
    shu = _load_file("ref_sh_utils", os.path.join(core, "utils", "sh_utils.py"))

    g = torch.Generator().manual_seed(3)
    h, w = 16, 24
    out = {}

    def head(seed_off):
        means = torch.randn(1, h, w, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 2.0])
        scales = torch.exp(torch.randn(1, h, w, 3, generator=g) * 0.3 - 4.0)
        rot = torch.randn(1, h, w, 4, generator=g)
        rot = rot / (rot.norm(dim=-1, keepdim=True) + 1e-8)
        sh = torch.randn(1, h, w, 3, 1, generator=g) * 0.3
        opac = torch.rand(1, h, w, 1, generator=g)
        return means, scales, rot, sh, opac

    m1, s1, r1, sh1, o1 = head(0)
    m2, s2, r2, sh2, o2 = head(1)
    img1 = torch.rand(1, 3, h, w, generator=g) * 2 - 1   # ImgNorm space
    img2 = torch.rand(1, 3, h, w, generator=g) * 2 - 1

    def hwc(img):  # splatt3r_utils.py:140-150 _get_original_img_hwc
        return (img * 0.5 + 0.5).clamp(0, 1).permute(0, 2, 3, 1)

    # splatt3r_utils.py:371-407
    cov1 = geo.build_covariance(s1, r1)
    cov2 = geo.build_covariance(s2, r2)
    shr1 = torch.zeros_like(sh1); shr1[..., 0] = shu.RGB2SH(hwc(img1))
    shr2 = torch.zeros_like(sh2); shr2[..., 0] = shu.RGB2SH(hwc(img2))
    pred1 = {"means": m1, "covariances": cov1, "sh": sh1 + shr1, "opacities": o1}
    pred2 = {"means_in_other_view": m2, "covariances": cov2, "sh": sh2 + shr2, "opacities": o2}
    # a non-trivial Sim3 -> 4x4 target pose (splatt3r_utils.py:153-165) and K
    ctx_pose = torch.eye(4)[None]
    tgt = torch.eye(4)[None].clone()
    ang = 0.1
    tgt[0, :3, :3] = torch.tensor([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0],
                                   [-np.sin(ang), 0, np.cos(ang)]], dtype=torch.float32) * 1.1
    tgt[0, :3, 3] = torch.tensor([0.05, -0.02, 0.1])
    K = torch.tensor([[[30.0, 0, 12.0], [0, 30.0, 8.0], [0, 0, 1]]])
    batch = {"context": [{"camera_pose": ctx_pose}],
             "target": [{"camera_pose": tgt, "camera_intrinsics": K}]}
    decoder = dec.DecoderSplattingCUDA(background_color=[0.0, 0.0, 0.0])
    decoder(batch, pred1, pred2, (h, w))
    st = captured["settings"]
    ins = captured["inputs"]
    for k in ("tanfovx", "tanfovy", "scale_modifier", "image_height", "image_width",
              "sh_degree"):
        out["settings_" + k] = np.asarray(st[k])
    for k in ("bg", "viewmatrix", "projmatrix", "campos"):
        out["settings_" + k] = st[k].detach().numpy()
    for k in ("means3D", "shs", "opacities", "cov3D_precomp"):
        out["in_" + k] = ins[k].detach().contiguous().numpy()
    # head outputs (to drive our glue with the same data)
    for name, t in dict(m1=m1, s1=s1, r1=r1, sh1=sh1, o1=o1, m2=m2, s2=s2, r2=r2, sh2=sh2,
                        o2=o2, img1=img1, img2=img2, ctx_pose=ctx_pose, tgt_pose=tgt,
                        K=K).items():
        out["head_" + name] = t.numpy()
    np.savez_compressed(os.path.join(GOLDEN, "render_boundary.npz"), **out)
    del sys.modules["diff_gaussian_rasterization"]
    print("wrote render_boundary.npz", {k: v.shape for k, v in out.items() if k.startswith("in_")})


def build_reference_model(cfg):
    """mast3r.model.AsymmetricMASt3R with the Splatt3R arguments
    (splatt3r_core/main.py:54-71), imported from /root/reference."""
    src = os.path.join(REF, "splatt3r_core", "src", "mast3r_src")
    for p in (os.path.join(src, "dust3r"), src):
        if p not in sys.path:
            sys.path.insert(0, p)
    import mast3r.model as mm
    return mm.AsymmetricMASt3R(
        pos_embed="RoPE100", patch_embed_cls="ManyAR_PatchEmbed", img_size=(512, 512),
        head_type="gaussian_head", output_mode=f"pts3d+gaussian+desc{cfg.desc_dim}",
        depth_mode=("exp", -mm.inf, mm.inf), conf_mode=("exp", 1, mm.inf),
        enc_embed_dim=cfg.enc_dim, enc_depth=cfg.enc_depth, enc_num_heads=cfg.enc_heads,
        dec_embed_dim=cfg.dec_dim, dec_depth=cfg.dec_depth, dec_num_heads=cfg.dec_heads,
        two_confs=True, use_offsets=cfg.use_offsets, sh_degree=cfg.sh_degree).eval()


def load_prng(model, cfg, seed):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "splatt3r-slam_amd"))
    from splatt3r_amd import weights as W
    sd = model.state_dict()
    man = W.manifest(cfg)
    assert [n for n, _ in man] == list(sd.keys()), "manifest order differs from the reference"
    assert all(tuple(sd[n].shape) == tuple(s) for n, s in man), "manifest shapes differ"
    new = {n: torch.from_numpy(W.prng_tensor_numpy(seed, n, s)) for n, s in man}
    model.load_state_dict(new)
    return man


def run_reference(model, img1, img2):
    """dust3r model.py:121-193 driven as splatt3r_utils.decoder() does
    (encode each view, _decoder, heads in fp32)."""
    shape = torch.tensor([list(img1.shape[-2:])], dtype=torch.int32)
    f1, p1, _ = model._encode_image(img1, shape)
    f2, p2, _ = model._encode_image(img2, shape)
    dec1, dec2 = model._decoder(f1, p1, f2, p2)
    dec1, dec2 = list(dec1), list(dec2)
    r1 = model._downstream_head(1, [t.float() for t in dec1], shape)
    r2 = model._downstream_head(2, [t.float() for t in dec2], shape)
    return f1, f2, p1, dec1, dec2, r1, r2


def gen_net():
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "splatt3r-slam_amd"))
    from splatt3r_amd import weights as W
    import dataclasses
    keys = ("pts3d", "conf", "desc", "desc_conf", "scales", "rotations", "sh", "opacities", "means")
    # (a) reduced config, full outputs, both use_offsets values
    for use_off in (True, False):
        cfg = dataclasses.replace(W.SMALL, use_offsets=use_off)
        torch.manual_seed(0)
        model = build_reference_model(cfg)
        man = load_prng(model, cfg, seed=1234)
        g = torch.Generator().manual_seed(5)
        H, Wd = 48, 64
        img1 = torch.rand(1, 3, H, Wd, generator=g) * 2 - 1
        img2 = torch.rand(1, 3, H, Wd, generator=g) * 2 - 1
        # stage captures of head 1's pts DPT (NHWC) to localise divergences
        cap = {}
        dpt = model.downstream_head1.dpt
        named = {"ap0": dpt.act_postprocess[0], "ap1": dpt.act_postprocess[1],
                 "ap2": dpt.act_postprocess[2], "ap3": dpt.act_postprocess[3],
                 "rn0": dpt.scratch.layer_rn[0], "rn1": dpt.scratch.layer_rn[1],
                 "rn2": dpt.scratch.layer_rn[2], "rn3": dpt.scratch.layer_rn[3],
                 "ref4": dpt.scratch.refinenet4, "ref3": dpt.scratch.refinenet3,
                 "ref2": dpt.scratch.refinenet2, "ref1": dpt.scratch.refinenet1,
                 "head0": dpt.head[0], "head3": dpt.head[3], "head4": dpt.head[4],
                 "mlp": model.downstream_head1.head_local_features}
        hooks = []
        for k, m in named.items():
            def fn(mod, inp, outp, k=k):
                if k not in cap:
                    cap[k] = outp.detach().clone()
            hooks.append(m.register_forward_hook(fn))
        f1, f2, p1, dec1, dec2, r1, r2 = run_reference(model, img1, img2)
        for hk_ in hooks:
            hk_.remove()
        out = dict(img1=img1.numpy(), img2=img2.numpy(), feat1=f1.numpy(), feat2=f2.numpy(),
                   pos=p1.numpy())
        for k, v in cap.items():
            out["stage_" + k] = (v.permute(0, 2, 3, 1) if v.dim() == 4 else v).contiguous().numpy()
        for hk in cfg.hooks:
            out[f"dec1_{hk}"] = dec1[hk].numpy()
            out[f"dec2_{hk}"] = dec2[hk].numpy()
        for k in keys:
            out["res1_" + k] = r1[k].numpy()
            out["res2_" + k] = r2[k].numpy()
        tag = "small_off" if use_off else "small_nooff"
        np.savez_compressed(os.path.join(GOLDEN, f"net_{tag}.npz"), **out)
        print(f"wrote net_{tag}.npz")
        if use_off:
            with open(os.path.join(GOLDEN, "manifest_small.txt"), "w") as f:
                f.writelines(f"{n} {list(s)}\n" for n, s in man)
    # (b) full Splatt3R architecture at 384x512: slices + checksums
    cfg = W.FULL
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    man = load_prng(model, cfg, seed=1234)
    with open(os.path.join(GOLDEN, "manifest_full.txt"), "w") as f:
        f.writelines(f"{n} {list(s)}\n" for n, s in man)
    g = torch.Generator().manual_seed(6)
    img1 = torch.rand(1, 3, 384, 512, generator=g) * 2 - 1
    img2 = torch.rand(1, 3, 384, 512, generator=g) * 2 - 1
    f1, f2, p1, dec1, dec2, r1, r2 = run_reference(model, img1, img2)
    out = dict(img1=img1.numpy(), img2=img2.numpy(), feat1_rows=f1[0, ::37].numpy(),
               feat1_sum=f1.double().sum().numpy(), feat1_abs=f1.double().abs().sum().numpy())
    for hk in cfg.hooks:
        out[f"dec1_{hk}_rows"] = dec1[hk][0, ::37].numpy()
        out[f"dec2_{hk}_rows"] = dec2[hk][0, ::37].numpy()
    for k in keys:
        for ri, r in (("1", r1), ("2", r2)):
            v = r[k][0]
            out[f"res{ri}_{k}_sub"] = v[::8, ::8].numpy()
            out[f"res{ri}_{k}_sum"] = v.double().sum().numpy()
            out[f"res{ri}_{k}_abs"] = v.double().abs().sum().numpy()
    np.savez_compressed(os.path.join(GOLDEN, "net_full_384x512.npz"), **out)
    print("wrote net_full_384x512.npz")


SECTIONS = {"matching": gen_matching, "render": gen_render, "net": gen_net}


def main(argv):
    if not os.path.isdir(REF):
        raise SystemExit("/root/reference not present: fixtures are generated in the build container")
    os.makedirs(GOLDEN, exist_ok=True)
    torch.set_grad_enabled(False)
    for s in (argv or list(SECTIONS)):
        SECTIONS[s]()


if __name__ == "__main__":
    main(sys.argv[1:])
