"""Generate the golden fixtures under tests/golden/ by importing the Python
reference from /root/reference (this container only; the GPU box never reads
/root/reference).  Committed outputs are data only (inputs + expected
outputs), never reference source.

  python oracle/gen_golden.py [section ...]     sections: matching, net, net_c4, n1, mono, resize, viz, portrait, render

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
    new = {n: torch.from_numpy(W.prng_tensor_numpy(seed, n, s, cfg)) for n, s in man}
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
    gen_full(384, 512, seed=6, write_manifest=True)


def gen_net_c4():
    """Full architecture at 320x512 (C4: EuRoC 752x480 -> 512x320 by the
    resize_img rule, splatt3r_utils.py:668-679; N = 640 tokens)."""
    gen_full(320, 512, seed=7)


def gen_net_c5():
    """Full architecture at 304x512 (C5 ETH3D shape by the resize_img rule;
    N = 608 tokens, a ragged tile tail for the 64-row attention tiles)."""
    gen_full(304, 512, seed=8)


def gen_full(H, Wd, seed, write_manifest=False):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "splatt3r-slam_amd"))
    from splatt3r_amd import weights as W
    keys = ("pts3d", "conf", "desc", "desc_conf", "scales", "rotations", "sh", "opacities", "means")
    cfg = W.FULL
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    man = load_prng(model, cfg, seed=1234)
    if write_manifest:
        with open(os.path.join(GOLDEN, "manifest_full.txt"), "w") as f:
            f.writelines(f"{n} {list(s)}\n" for n, s in man)
    g = torch.Generator().manual_seed(seed)
    img1 = torch.rand(1, 3, H, Wd, generator=g) * 2 - 1
    img2 = torch.rand(1, 3, H, Wd, generator=g) * 2 - 1
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
    name = f"net_full_{H}x{Wd}.npz"
    np.savez_compressed(os.path.join(GOLDEN, name), **out)
    print("wrote", name)


def gen_mono():
    """splatt3r_inference_mono (splatt3r_utils.py:503-536) on the small
    config: the reference decoder run on (img1, img1) of net_small_off.npz."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "splatt3r-slam_amd"))
    from splatt3r_amd import weights as W
    import dataclasses
    keys = ("pts3d", "conf", "desc", "desc_conf", "scales", "rotations", "sh", "opacities", "means")
    cfg = dataclasses.replace(W.SMALL, use_offsets=True)
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    load_prng(model, cfg, seed=1234)
    img1 = torch.from_numpy(np.load(os.path.join(GOLDEN, "net_small_off.npz"))["img1"])
    _, _, _, _, _, r1, r2 = run_reference(model, img1, img1)
    out = {"img": img1.numpy()}
    for k in keys:
        out["res11_" + k] = r1[k].numpy()
        out["res21_" + k] = r2[k].numpy()
    np.savez_compressed(os.path.join(GOLDEN, "net_small_mono.npz"), **out)
    print("wrote net_small_mono.npz")


RESIZE_CASES = ((480, 640, 512), (480, 752, 512), (512, 512, 512), (640, 480, 512),
                (540, 960, 512), (300, 400, 512), (480, 640, 224))


def resize_input(h, w, seed):
    """Deterministic smooth float image in [0, 1] (also rebuilt by the test)."""
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    img = np.stack([0.45 + 0.45 * np.sin(6 * xx + 4 * yy + k + seed) for k in range(3)], -1)
    iy, ix = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    img += 0.1 * (((ix // 3) + (iy // 3)) % 2)[..., None]   # 3-px checker: resampling detail
    return np.clip(img, 0, 1).astype(np.float32)


def gen_resize():
    """resize_img (splatt3r_utils.py:646-693), the reference's own function
    text compiled from the file (the module itself does not import here:
    lietorch, torchvision); torchvision's ImgNorm is restated as
    ToTensor + Normalize(0.5, 0.5).  Saved: the cropped uint8 image, the
    true_shape and the transformation tuple per case."""
    import ast
    import PIL.Image
    path = os.path.join(REF, "splatt3r_slam", "splatt3r_utils.py")
    tree = ast.parse(open(path).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef)
           and n.name in ("_resize_pil_image", "resize_img")]
    mod = ast.Module(body=fns, type_ignores=[])

    def img_norm(pil):
        a = torch.from_numpy(np.asarray(pil).astype(np.float32) / 255.0).permute(2, 0, 1)
        return (a - 0.5) / 0.5

    ns = {"PIL": PIL, "np": np, "ImgNorm": img_norm}
    exec(compile(mod, path, "exec"), ns)
    out = {}
    for i, (h, w, size) in enumerate(RESIZE_CASES):
        img = resize_input(h, w, i)
        res, tr = ns["resize_img"](img, size, return_transformation=True)
        out[f"case{i}_uimg"] = res["unnormalized_img"]
        out[f"case{i}_true_shape"] = res["true_shape"]
        # res["img"] = ImgNorm(uimg) is not stored: the test derives it from uimg
        out[f"case{i}_transform"] = np.float64(tr)
        print(i, (h, w, size), "->", res["true_shape"].tolist(), tr)
    np.savez_compressed(os.path.join(GOLDEN, "resize_img.npz"), **out)
    print("wrote resize_img.npz")


def _tf32_round(t):
    """fp32 -> TF32 operand (round to nearest even at mantissa bit 13)."""
    if not torch.is_tensor(t) or t.dtype != torch.float32:
        return t
    i = t.contiguous().view(torch.int32)
    i = (i + 0xFFF + ((i >> 13) & 1)) & ~0x1FFF
    return i.view(torch.float32)


def tf32_mode():
    """The reference's CUDA path runs its matrix products in TF32
    (main.py:195 torch.backends.cuda.matmul.allow_tf32 = True; cuDNN convs
    default to TF32): a TorchFunctionMode that rounds both operands of every
    linear / matmul / conv / conv-transpose to TF32 and keeps fp32
    accumulation, so the CPU reference reproduces that precision class."""
    from torch.overrides import TorchFunctionMode

    ops = {F.linear, torch.matmul, torch.bmm, torch.Tensor.__matmul__, F.conv2d,
           F.conv_transpose2d}

    class TF32Mode(TorchFunctionMode):
        def __torch_function__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            if func in ops:
                args = tuple(_tf32_round(a) if i < 2 else a for i, a in enumerate(args))
                if "weight" in kwargs:
                    kwargs["weight"] = _tf32_round(kwargs["weight"])
            elif func is torch.einsum:
                args = (args[0],) + tuple(_tf32_round(a) for a in args[1:])
            return func(*args, **kwargs)

    return TF32Mode()


def gen_viz():
    """Full-map render (A14): the reference's own `_render_gs_interactive`
    (splatt3r_slam/visualization.py:467-600; function text compiled from the
    file -- the module needs moderngl/imgui/in3d) driven with a synthetic
    SharedGaussians map and GL camera, a stub rasterizer capturing what it
    hands GaussianRasterizer, then oracle.raster on the captured inputs.
    Saved: the map, the camera, the captured settings/inputs and the
    clamped HWC image the function returns."""
    import ast
    import types
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle
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
    # import splatt3r_core.src.pixelsplat_src.* without running
    # splatt3r_core/__init__.py (it imports lightning, absent here)
    pkg = types.ModuleType("splatt3r_core")
    pkg.__path__ = [os.path.join(REF, "splatt3r_core")]
    sys.modules["splatt3r_core"] = pkg
    sys.path.insert(0, os.path.join(REF, "splatt3r_core", "src", "pixelsplat_src"))
    path = os.path.join(REF, "splatt3r_slam", "visualization.py")
    tree = ast.parse(open(path).read())
    fn = None
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == "_render_gs_interactive":
            fn = node
    ns = {"torch": torch, "np": np, "math": __import__("math"),
          "GaussianRasterizationSettings": Settings, "GaussianRasterizer": Rasterizer}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)
    render_fn = ns["_render_gs_interactive"]

    rng = np.random.default_rng(11)
    n = 30000
    means = rng.normal(size=(n, 3)).astype(np.float32) * np.float32([0.6, 0.4, 0.5]) \
        + np.float32([0.1, -0.05, 3.0])
    sc = np.exp(rng.uniform(np.log(0.01), np.log(0.05), (n, 3)))
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    x, y, z, w = q.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                  2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                  2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)
    R = R.reshape(n, 3, 3)
    cov = np.einsum("nik,nk,njk->nij", R, sc * sc, R)
    iu = np.triu_indices(3)
    cov6 = cov[:, iu[0], iu[1]].astype(np.float32)
    colors = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    opac = rng.uniform(0.3, 1.0, n).astype(np.float32)
    # OpenCV camera-to-world: small yaw and offset; GL world-to-camera from it
    th = 0.1
    T_WC_cv = np.eye(4)
    T_WC_cv[:3, :3] = [[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]]
    T_WC_cv[:3, 3] = [-0.2, 0.05, -0.3]
    cv2gl = np.diag([1.0, -1.0, -1.0, 1.0])
    T_CW_gl = (cv2gl @ np.linalg.inv(T_WC_cv)).astype(np.float32)
    ns_ = types.SimpleNamespace
    gm = tuple(torch.from_numpy(a) for a in (means, cov6, colors, opac))
    self_ = ns_(shared_gaussians=ns_(get_all=lambda: gm),
                camera=ns_(viewport_size=(640, 480), T_CW=T_CW_gl, proj_mat=ns_(hfov=90.0)),
                gs_resolution_scale=0.5)
    render_fn(self_)
    st, ins = captured["settings"], captured["inputs"]
    sd = {k: (st[k].detach().numpy() if torch.is_tensor(st[k]) else st[k]) for k in st}
    o = oracle.raster(sd, ins["means3D"].numpy(), ins["opacities"].numpy(),
                      colors_precomp=ins["colors_precomp"].numpy(),
                      cov3D_precomp=ins["cov3D_precomp"].numpy(), nthreads=8)
    img = np.clip(o["color"], 0, 1).transpose(1, 2, 0)
    out = dict(means=means, cov6=cov6, colors=colors, opacities=opac, T_CW_gl=T_CW_gl,
               viewport=np.int32([640, 480]), hfov=np.float32(90.0), res_scale=np.float32(0.5),
               image_hwc=img, num_rendered=np.int64(o["num_rendered"]))
    for k in ("tanfovx", "tanfovy", "image_height", "image_width"):
        out["settings_" + k] = np.asarray(sd[k])
    for k in ("bg", "viewmatrix", "projmatrix", "campos"):
        out["settings_" + k] = np.asarray(sd[k], np.float32)
    out["in_means3D"] = ins["means3D"].numpy()
    out["in_cov3D_precomp"] = ins["cov3D_precomp"].numpy()
    np.savez_compressed(os.path.join(GOLDEN, "viz_render.npz"), **out)
    for m in ("diff_gaussian_rasterization", "splatt3r_core"):
        del sys.modules[m]
    print("wrote viz_render.npz", img.shape, "mean", float(img.mean()),
          "num_rendered", o["num_rendered"])


def gen_portrait():
    """Portrait inputs through the reference model API: a landscape-shaped
    image tensor with a portrait true_shape (ManyAR_PatchEmbed transposes it,
    patch_embed.py:42-70; _LandscapeWrapperYes runs the heads on the
    transposed grid and transposes back, utils/misc.py:80-116).  Small
    config, use_offsets."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "splatt3r-slam_amd"))
    from splatt3r_amd import weights as W
    import dataclasses
    keys = ("pts3d", "conf", "desc", "desc_conf", "scales", "rotations", "sh", "opacities", "means")
    cfg = dataclasses.replace(W.SMALL, use_offsets=True)
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    load_prng(model, cfg, seed=1234)
    g = torch.Generator().manual_seed(9)
    img1 = torch.rand(1, 3, 48, 64, generator=g) * 2 - 1
    img2 = torch.rand(1, 3, 48, 64, generator=g) * 2 - 1
    shape = torch.tensor([[64, 48]], dtype=torch.int32)      # portrait true shape
    f1, p1, _ = model._encode_image(img1, shape)
    f2, p2, _ = model._encode_image(img2, shape)
    dec1, dec2 = model._decoder(f1, p1, f2, p2)
    dec1, dec2 = list(dec1), list(dec2)
    r1 = model._downstream_head(1, [t.float() for t in dec1], shape)
    r2 = model._downstream_head(2, [t.float() for t in dec2], shape)
    out = dict(img1=img1.numpy(), img2=img2.numpy(), true_shape=shape.numpy(), feat1=f1.numpy(),
               pos1=p1.numpy())
    for k in keys:
        out["res1_" + k] = r1[k].numpy()
        out["res2_" + k] = r2[k].numpy()
    np.savez_compressed(os.path.join(GOLDEN, "net_small_portrait.npz"), **out)
    print("wrote net_small_portrait.npz", r1["pts3d"].shape)


def _sim3_matrix(T):
    """lietorch Sim3 data [t, q(xyzw), s] -> 4x4 [sR | t] (fp64 -> fp32), the
    matrix splatt3r_utils.py:153-165 builds through SE3.matrix()."""
    T = np.asarray(T, np.float64)
    x, y, z, w = T[3:7] / np.linalg.norm(T[3:7])
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    M = np.eye(4)
    M[:3, :3] = R * T[7]
    M[:3, 3] = T[:3]
    return torch.from_numpy(M.astype(np.float32))[None]


# N1 render cases: (name, context Sim3, target Sim3); the tracked-frame render
# of main.py:491-499 is a self-render (target_T_WC = frame.T_WC)
N1_POSES = {
    "self": ([0.0, 0, 0, 0, 0, 0, 1, 1], [0.0, 0, 0, 0, 0, 0, 1, 1]),
    "moved": ([0.1, -0.05, 0.2, 0.0499792, 0.0, 0.0, 0.99875026, 1.2],
              [0.13, -0.04, 0.15, 0.0499792, 0.0399893, 0.0, 0.99795, 1.2]),
}
# (tag, config, scale bias of weights.n1_init, H, W): the small config and
# the full architecture at the C2 (384x512) and C4 (320x512) sizes
N1_CASES = (("small_off", "small_off", -1.2, 48, 64), ("small_nooff", "small_nooff", -1.2, 48, 64),
            ("full_384x512", "full", -2.5, 384, 512), ("full_320x512", "full", -2.5, 320, 512))
N1_CONTRAST = 0.08
N1_LOOKAT_BACK = 0.3
N1_Q16 = 65535.0          # fp32 image -> uint16 quantum (mean error 3.8e-6)
N1_DQ = float(2 ** 20)    # TF32-minus-fp32 image delta -> int16 quantum ~1e-6


def n1_image(H, W, phase):
    """The N1 input image: a smooth colour field of amplitude N1_CONTRAST
    around mid-grey, as uint8 HxWx3 (a camera frame's type).  Low spatial
    frequency, so splats that land next to each other carry similar
    colours."""
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    ch = [0.5 + N1_CONTRAST * np.sin(5 * xx + 3 * yy + 2.1 * k + phase) * np.cos(2 * yy - xx + k)
          for k in range(3)]
    return np.round(np.stack(ch, -1) * 255).astype(np.uint8)


def n1_normalise(u8):
    """uint8 HxWx3 -> ImgNorm [1,3,H,W] float32 in [-1, 1] (dust3r/utils/image.py:23)."""
    a = torch.from_numpy(u8.astype(np.float32) / np.float32(255.0)).permute(2, 0, 1)[None]
    return ((a - 0.5) / 0.5).contiguous()


def _look_at(means, back=1.0):
    """Sim3 data of a camera at -back * d looking along d = the normalised
    median of `means` (camera +z -> d, shortest-arc quaternion)."""
    d = np.median(means.reshape(-1, 3).numpy().astype(np.float64), axis=0)
    d /= np.linalg.norm(d)
    z = np.array([0.0, 0.0, 1.0])
    axis = np.cross(z, d)
    q = np.concatenate([axis, [1.0 + z @ d]])
    q /= np.linalg.norm(q)
    return [float(v) for v in (-back * d)] + [float(v) for v in q] + [1.0]


def gen_n1():
    """North-star N1 fixture: the reference pipeline's rendered RGB.

    The reference network (imported modules, portable-PRNG weights with the
    conditioned init of weights.n1_init: multi-pixel splats of varying scale,
    the colour from the image) is run on smooth uint8 frames (n1_image), in
    fp32 and with TF32-emulated matrix products (the reference CUDA path's
    arithmetic, main.py:195); its head outputs go through the reference glue
    exactly as splatt3r_render drives it (splatt3r_utils.py:332-432:
    build_covariance, RGB2SH residual, DecoderSplattingCUDA with default
    intrinsics f = max(h, w)), a stub rasterizer captures what the glue hands
    GaussianRasterizer and oracle.raster (oracle/raster_ref.c) renders it.
    Views: self, moved, look-at.  Saved: the frames, poses, images (fp32 as
    uint16, the TF32 image as an int16 delta), subsampled head outputs of the
    conditioned init (the scales check) and, for the small configs, the full
    head outputs (the glue check).  Also kept: the default-init small
    matching on TF32 outputs (tests/test_net.py)."""
    import dataclasses
    import types
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle
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
    decoder = dec.DecoderSplattingCUDA(background_color=[0.0, 0.0, 0.0])

    def render(r1, r2, img1, img2, T_ctx, T_tgt):
        # splatt3r_utils.py:358-432 with frame = view 1, ref_frame = view 2
        hwc = lambda im: (im * 0.5 + 0.5).clamp(0, 1).permute(0, 2, 3, 1)
        h, w = r1["means"].shape[1:3]
        cov1 = geo.build_covariance(r1["scales"], r1["rotations"])
        cov2 = geo.build_covariance(r2["scales"], r2["rotations"])
        sh1 = r1["sh"].clone(); res = torch.zeros_like(sh1); res[..., 0] = shu.RGB2SH(hwc(img1))
        sh1 = sh1 + res
        sh2 = r2["sh"].clone(); res = torch.zeros_like(sh2); res[..., 0] = shu.RGB2SH(hwc(img2))
        sh2 = sh2 + res
        pred1 = {"means": r1["means"], "covariances": cov1, "sh": sh1, "opacities": r1["opacities"]}
        pred2 = {"means_in_other_view": r2["means"], "covariances": cov2, "sh": sh2,
                 "opacities": r2["opacities"]}
        f = float(max(h, w))
        K = torch.tensor([[[f, 0, w / 2.0], [0, f, h / 2.0], [0, 0, 1]]], dtype=torch.float32)
        batch = {"context": [{"camera_pose": _sim3_matrix(T_ctx)}],
                 "target": [{"camera_pose": _sim3_matrix(T_tgt), "camera_intrinsics": K}]}
        decoder(batch, pred1, pred2, (h, w))
        st, ins = captured["settings"], captured["inputs"]
        sd = {k: (st[k].detach().numpy() if torch.is_tensor(st[k]) else st[k]) for k in st}
        o = oracle.raster(sd, ins["means3D"].numpy(), ins["opacities"].numpy(),
                          shs=ins["shs"].numpy(), cov3D_precomp=ins["cov3D_precomp"].numpy(),
                          nthreads=8)
        return o["color"], o["num_rendered"]

    keys = ("means", "scales", "rotations", "sh", "opacities")
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "splatt3r-slam_amd"))
    from splatt3r_amd import weights as W
    out = {"contrast": np.float32(N1_CONTRAST), "lookat_back": np.float32(N1_LOOKAT_BACK),
           "q16": np.float32(N1_Q16), "dq": np.float32(N1_DQ)}
    # default-init small model: matching on the TF32 outputs (test_net.py)
    g = np.load(os.path.join(GOLDEN, "net_small_off.npz"))
    torch.manual_seed(0)
    model = build_reference_model(dataclasses.replace(W.SMALL, use_offsets=True))
    load_prng(model, dataclasses.replace(W.SMALL, use_offsets=True), seed=1234)
    with tf32_mode():
        _, _, _, _, _, t1, t2 = run_reference(model, torch.from_numpy(g["img1"]),
                                              torch.from_numpy(g["img2"]))
    idx_t, valid_t = oracle.match(t1["pts3d"].numpy(), t2["pts3d"].numpy(),
                                  t1["desc"].numpy(), t2["desc"].numpy())
    out["small_off_match_tf32_idx"] = idx_t
    out["small_off_match_tf32_valid"] = valid_t
    only = os.environ.get("N1_ONLY")          # experiments: a subset of the cases
    sb_over = os.environ.get("N1_SMALL_BIAS")
    for tag, kind, scale_bias, H, Wd in N1_CASES:
        if only and tag not in only.split(","):
            continue
        if sb_over and kind != "full":
            scale_bias = float(sb_over)
        base = W.FULL if kind == "full" else dataclasses.replace(
            W.SMALL, use_offsets=(kind == "small_off"))
        cfg = W.n1_init(base, scale_bias)
        torch.manual_seed(0)
        model = build_reference_model(cfg)
        load_prng(model, cfg, seed=1234)
        u1, u2 = n1_image(H, Wd, 0.0), n1_image(H, Wd, 0.4)
        im1, im2 = n1_normalise(u1), n1_normalise(u2)
        _, _, _, _, _, r1, r2 = run_reference(model, im1, im2)
        with tf32_mode():
            _, _, _, _, _, t1, t2 = run_reference(model, im1, im2)
        del model
        out[f"{tag}_u8img1"], out[f"{tag}_u8img2"] = u1, u2
        out[f"{tag}_scale_bias"] = np.float32(scale_bias)
        sub = (slice(None), slice(None, None, 8), slice(None, None, 8)) if kind == "full" \
            else (slice(None),)
        for i, r in ((1, r1), (2, r2)):
            for k in keys + ("pts3d", "conf"):
                out[f"{tag}_res{i}_{k}"] = r[k][sub].contiguous().numpy()
        poses = dict(N1_POSES)
        poses["lookat"] = ([0.0, 0, 0, 0, 0, 0, 1, 1], _look_at(r1["means"], N1_LOOKAT_BACK))
        for pname, (Tc, Tt) in poses.items():
            img, nr = render(r1, r2, im1, im2, Tc, Tt)
            img_t, _ = render(t1, t2, im1, im2, Tc, Tt)
            q = np.round(np.clip(img, 0, 1) * N1_Q16)
            assert np.array_equal(np.clip(img, 0, 1), img), "bg 0 + alpha <= 1: image in [0, 1]"
            out[f"{tag}_{pname}_image_u16"] = q.astype(np.uint16)
            d = np.round((img_t.astype(np.float64) - q / N1_Q16) * N1_DQ)
            out[f"{tag}_{pname}_tf32_delta"] = np.clip(d, -32767, 32767).astype(np.int16)
            out[f"{tag}_{pname}_ctx"] = np.float32(Tc)
            out[f"{tag}_{pname}_tgt"] = np.float32(Tt)
            dref = float(np.abs(img - img_t).mean())
            print(tag, pname, "num_rendered", nr, "mean %.4f" % float(img.mean()),
                  "covered %.3f" % float((img.sum(0) > 0).mean()),
                  "tf32-vs-fp32 mean-L1 %.3e" % dref,
                  "delta clipped", int((np.abs(d) > 32767).sum()), flush=True)
    np.savez_compressed(os.environ.get("N1_OUT", os.path.join(GOLDEN, "n1_render.npz")), **out)
    del sys.modules["diff_gaussian_rasterization"]
    print("wrote n1_render.npz")


# ------------------------------------------------------- host glue (AST) ---
def _ast_defs(path, names, ns, cls=None):
    """Compile the reference's own function (or, with `cls`, method) text
    from `path` into namespace `ns` (the module itself does not import here:
    lietorch / mast3r_slam_backends / cv2 are absent).  Decorators are
    dropped (torch.inference_mode only)."""
    import ast
    tree = ast.parse(open(path).read())
    body = tree.body
    if cls is not None:
        body = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls).body
    fns = [n for n in body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert sorted(f.name for f in fns) == sorted(names), (path, names)
    for f in fns:
        f.decorator_list = []
    exec(compile(ast.Module(body=fns, type_ignores=[]), path, "exec"), ns)
    return ns


def _reference_config():
    """config/base.yaml through the reference's own loader
    (splatt3r_slam/config.py, importable: yaml + re)."""
    cfgmod = _load_file("ref_config", os.path.join(REF, "splatt3r_slam", "config.py"))
    cwd = os.getcwd()
    try:
        os.chdir(REF)
        cfgmod.load_config("config/base.yaml")
    finally:
        os.chdir(cwd)
    return cfgmod.config


class MatSim3:
    """lietorch.Sim3 in matrix form (float64 4x4 [sR | t]) for driving the
    reference's tracker / geometry text: act, inv, compose, matrix.  `retr`
    records the GN step and keeps the pose (one normal-equation step is
    what the fixture pins; lietorch's Exp is not importable)."""

    def __init__(self, M):
        self.M = M

    @staticmethod
    def from_data(T):
        return MatSim3(_sim3_matrix(T)[0].double())

    def act(self, p):
        return p @ self.M[:3, :3].T + self.M[:3, 3]

    def inv(self):
        return MatSim3(torch.linalg.inv(self.M))

    def __mul__(self, o):
        return MatSim3(self.M @ o.M)

    def retr(self, tau):
        self.tau = tau
        return self


def gen_host():
    """Fixtures for the host-side Python of the path, produced by running
    the reference's own function text (AST-extracted) on synthetic inputs:

      gaussians_to_world     splatt3r_utils.py:180-328 (+ _get_original_img_hwc
                             :140-150; build_covariance / RGB2SH imported from
                             splatt3r_core/utils; _sim3_to_4x4 -> MatSim3
                             matrix, i.e. numpy in place of lietorch)
      geometry               geometry.py:5-128 (point_to_ray_dist, act_Sim3,
                             project_calib, constrain_points_to_ray, ...)
      tracker GN step        tracker.py:129-270 (get_points_poses, solve,
                             opt_pose_ray_dist_sim3, opt_pose_calib_sim3 with
                             max_iters 1; H captured at the Cholesky)
      add_factors            global_opt.py:30-99 with splatt3r_match_symmetric
                             stubbed to fixed match tensors
      match_iterative_proj   matching.py:8-90 with mast3r_slam_backends stubbed
                             by the oracle kernels (oracle.iter_proj /
                             refine_matches; the CUDA kernels do not compile)
    -> tests/golden/host_glue.npz."""
    import types
    import einops
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle
    core = os.path.join(REF, "splatt3r_core")
    geo_core = _load_file("ref_geometry_core", os.path.join(core, "utils", "geometry.py"))
    shu = _load_file("ref_sh_utils", os.path.join(core, "utils", "sh_utils.py"))
    nlo = _load_file("ref_nlo", os.path.join(REF, "splatt3r_slam", "nonlinear_optimizer.py"))
    rimg = _load_file("ref_image", os.path.join(REF, "splatt3r_slam", "image.py"))
    cfg = _reference_config()
    out = {}

    # ---- gaussians_to_world
    ns = {"torch": torch, "einops": einops, "RGB2SH": shu.RGB2SH,
          "build_covariance": geo_core.build_covariance,
          "_sim3_to_4x4": lambda T: _sim3_matrix(T.data.reshape(-1)[:8].numpy())}
    _ast_defs(os.path.join(REF, "splatt3r_slam", "splatt3r_utils.py"),
              ["gaussians_to_world", "_get_original_img_hwc"], ns)
    g2w = ns["gaussians_to_world"]

    def pred(H, W, seed):
        g = torch.Generator().manual_seed(seed)
        q = torch.randn(1, H, W, 4, generator=g)
        q = q / q.norm(dim=-1, keepdim=True)
        means = torch.randn(1, H, W, 3, generator=g) * 0.5
        means[..., 2] = torch.rand(1, H, W, generator=g) * 4 - 0.5
        return dict(means=means, scales=torch.exp(torch.randn(1, H, W, 3, generator=g) - 2.5),
                    rotations=q, sh=torch.randn(1, H, W, 3, 1, generator=g) * 0.3,
                    opacities=torch.rand(1, H, W, 1, generator=g),
                    conf=1 + torch.rand(1, H, W, generator=g) * 2)

    G2W_CASES = ((48, 64, 4, True, 0.98, 1.0, 1.5), (48, 64, 1, False, 0.98, 0.5, 1.5),
                 (37, 50, 3, True, 0.9, 0.3, 2.0), (40, 56, 2, False, 1.0, 10.0, 0.0))
    for c, (H, W, stride, cross, q, maxs, minc) in enumerate(G2W_CASES):
        p1, p2 = pred(H, W, 100 + c), pred(H, W, 200 + c)
        img = torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(300 + c)) * 2.2 - 1.1
        T = np.array([0.2, -0.1, 0.5, 0.0, np.sin(0.15), 0.0, np.cos(0.15), 1.3], np.float32)
        fr = types.SimpleNamespace(gaussian_pred=p1, gaussian_pred_cross=p2, img=img,
                                   T_WC=types.SimpleNamespace(data=torch.from_numpy(T)[None]))
        res = g2w(fr, include_cross=cross, spatial_stride=stride, depth_max_percentile=q,
                  max_scale=maxs, min_confidence=minc)
        pre = f"g2w{c}_"
        out[pre + "args"] = np.float64([H, W, stride, cross, q, maxs, minc])
        out[pre + "T"] = T
        out[pre + "img"] = img.numpy()
        for k in p1:
            out[pre + "p1_" + k] = p1[k].numpy()
            out[pre + "p2_" + k] = p2[k].numpy()
        for k, v in zip(("means", "cov", "colors", "opacities"), res):
            out[pre + "out_" + k] = v.numpy()
        print("gaussians_to_world case", c, "kept", res[0].shape[0])

    # ---- geometry (float64)
    gns = {"torch": torch, "lietorch": None}
    _ast_defs(os.path.join(REF, "splatt3r_slam", "geometry.py"),
              ["skew_sym", "point_to_dist", "point_to_ray_dist", "act_Sim3", "decompose_K",
               "project_calib", "backproject", "get_pixel_coords", "constrain_points_to_ray"], gns)
    rng = np.random.default_rng(7)
    X = torch.from_numpy(np.concatenate([rng.uniform(-1, 1, (512, 2)),
                                         rng.uniform(0.5, 4, (512, 1))], 1))
    rd, J = gns["point_to_ray_dist"](X, jacobian=True)
    out["geo_X"], out["geo_rd"], out["geo_rd_J"] = X.numpy(), rd.numpy(), J.numpy()
    Td = np.array([0.1, -0.2, 0.3, 0.1, -0.05, 0.2, 0.0, 1.1])
    Td[6] = np.sqrt(1 - np.sum(Td[3:6] ** 2))
    pW, Ja = gns["act_Sim3"](MatSim3.from_data(Td), X, jacobian=True)
    out["geo_T"], out["geo_act"], out["geo_act_J"] = np.float32(Td), pW.numpy(), Ja.numpy()
    K = torch.tensor([[300.0, 0, 160.0], [0, 310.0, 120.0], [0, 0, 1]], dtype=torch.float64)
    P = X.clone()
    P[::17, 2] = -0.5                                     # behind the camera
    pz, D, valid = gns["project_calib"](P, K, (240, 320), jacobian=True, border=-10, z_eps=1e-6)
    out["geo_K"], out["geo_P"] = K.numpy(), P.numpy()
    out["geo_pz"], out["geo_pz_J"], out["geo_pz_valid"] = pz.numpy(), D.numpy(), valid.numpy()

    # ---- tracker: one normal-equation step, ray/dist and calibrated
    tcfg = dict(cfg["tracking"], max_iters=1)
    captured = {}

    class TorchProxy(types.ModuleType):
        def __getattr__(self, k):
            return getattr(torch, k)

    tp = TorchProxy("torch")
    tp.linalg = types.SimpleNamespace(
        cholesky=lambda H, upper=False: captured.setdefault("H", [H.clone()]) and
        torch.linalg.cholesky(H, upper=upper), norm=torch.linalg.norm)
    tns = dict(gns, torch=tp, huber=nlo.huber, check_convergence=nlo.check_convergence,
               config={"tracking": tcfg})
    _ast_defs(os.path.join(REF, "splatt3r_slam", "tracker.py"),
              ["solve", "opt_pose_ray_dist_sim3", "opt_pose_calib_sim3", "get_points_poses"],
              tns, cls="FrameTracker")
    tracker = types.SimpleNamespace(cfg=tcfg)
    for k in ("solve", "opt_pose_ray_dist_sim3", "opt_pose_calib_sim3", "get_points_poses"):
        setattr(tracker, k, types.MethodType(tns[k], tracker))

    def scene(n, seed, calib_hw=None):
        r = np.random.default_rng(seed)
        if calib_hw is None:
            Xk = np.concatenate([r.uniform(-1, 1, (n, 2)), r.uniform(1, 4, (n, 1))], 1)
        else:
            h, w = calib_hw
            v, u = np.divmod(np.arange(h * w), w)
            z = r.uniform(1, 4, h * w)
            Xk = np.stack([(u - w / 2) / (0.9 * max(h, w)) * z, (v - h / 2) / (0.9 * max(h, w)) * z,
                           z], 1) + r.normal(size=(h * w, 3)) * 0.02
            n = h * w
        T_true = np.array([0.05, -0.02, 0.03, 0.02, -0.01, 0.015, 0.0, 1.02])
        T_true[6] = np.sqrt(1 - np.sum(T_true[3:6] ** 2))
        Xf = MatSim3.from_data(T_true).inv().act(torch.from_numpy(Xk)).numpy() \
            + r.normal(size=(n, 3)) * 0.02
        Q = r.uniform(0.5, 3.0, (n, 1))
        valid = r.uniform(size=(n, 1)) > 0.1
        return Xf, Xk, Q, valid

    Ttr = np.array([0.01, 0.02, -0.01, 0.01, 0.0, -0.01, 0.0, 0.98])
    Ttr[6] = np.sqrt(1 - np.sum(Ttr[3:6] ** 2))
    Xf, Xk, Q, valid = scene(4096, 11)
    captured.clear()
    I = MatSim3.from_data(np.array([0, 0, 0, 0, 0, 0, 1, 1.0]))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    _, Tc = tracker.opt_pose_ray_dist_sim3(t(Xf), t(Xk), MatSim3.from_data(Ttr), I, t(Q),
                                           t(valid))
    H = captured["H"][0].numpy()
    tau = Tc.tau.numpy().reshape(-1)
    out.update(trk_ray_Xf=Xf, trk_ray_Xk=Xk, trk_ray_Q=Q, trk_ray_valid=valid,
               trk_ray_T=np.float32(Ttr), trk_ray_H=H, trk_ray_g=H @ tau, trk_ray_tau=tau)
    # calibrated: get_points_poses (constrain to rays, pixel grid + log z)
    h, w = 24, 32
    Xf, Xk, Q, valid = scene(0, 12, (h, w))
    Kc = torch.tensor([[0.9 * 32, 0, 16.0], [0, 0.9 * 32, 12.0], [0, 0, 1]], dtype=torch.float64)
    idx = np.random.default_rng(13).permutation(h * w)
    frame = types.SimpleNamespace(X_canon=t(Xf), T_WC=MatSim3.from_data(Ttr),
                                  get_average_conf=lambda: torch.ones(h * w, 1, dtype=torch.float64))
    kf = types.SimpleNamespace(X_canon=t(Xk), T_WC=I,
                               get_average_conf=lambda: torch.ones(h * w, 1, dtype=torch.float64))
    Xf_c, Xk_c, T_WCf, T_WCk, _, _, meas, vmeas = tracker.get_points_poses(
        frame, kf, t(idx), (h, w), True, Kc)
    captured.clear()
    _, Tc = tracker.opt_pose_calib_sim3(Xf_c, Xk_c, T_WCf, T_WCk, t(Q), t(valid), meas, vmeas, Kc,
                                        (h, w))
    H = captured["H"][0].numpy()
    tau = Tc.tau.numpy().reshape(-1)
    out.update(trk_cal_Xf=Xf, trk_cal_Xk=Xk, trk_cal_idx=idx, trk_cal_K=Kc.numpy(),
               trk_cal_hw=np.int64([h, w]), trk_cal_Q=Q, trk_cal_valid=valid,
               trk_cal_T=np.float32(Ttr), trk_cal_Xf_c=Xf_c.numpy(), trk_cal_Xk_c=Xk_c.numpy(),
               trk_cal_meas=meas.numpy(), trk_cal_vmeas=vmeas.numpy(), trk_cal_H=H,
               trk_cal_g=H @ tau)
    print("tracker steps: |g| ray", np.abs(out["trk_ray_g"]).max(), "calib", np.abs(H @ tau).max())

    # ---- add_factors (global_opt.py:30-99)
    fns = {"torch": torch}
    _ast_defs(os.path.join(REF, "splatt3r_slam", "global_opt.py"), ["add_factors"], fns,
              cls="FactorGraph")
    hh, ww, b = 12, 16, 4
    r = np.random.default_rng(21)
    dens = np.array([0.05, 0.6, 0.05, 0.3])          # pair 0 consecutive, pair 2 rejected
    m = dict(idx_i2j=r.integers(0, hh * ww, (b, hh * ww)), idx_j2i=r.integers(0, hh * ww, (b, hh * ww)),
             valid_j=r.uniform(size=(b, hh * ww, 1)) < dens[:, None, None],
             valid_i=r.uniform(size=(b, hh * ww, 1)) < dens[:, None, None] + 0.05,
             Qii=r.uniform(0.5, 3.5, (b, hh * ww, 1)), Qjj=r.uniform(0.5, 3.5, (b, hh * ww, 1)),
             Qji=r.uniform(0.5, 3.5, (b, hh * ww, 1)), Qij=r.uniform(0.5, 3.5, (b, hh * ww, 1)))
    m = {k: torch.from_numpy(v.astype(np.float32) if v.dtype == np.float64 else v)
         for k, v in m.items()}
    fns["splatt3r_match_symmetric"] = lambda *a: (m["idx_i2j"], m["idx_j2i"], m["valid_j"],
                                                  m["valid_i"], m["Qii"], m["Qjj"], m["Qji"],
                                                  m["Qij"])
    ii, jj = [0, 0, 1, 2], [1, 2, 3, 4]
    for k, v in m.items():
        out["af_m_" + k] = v.numpy()
    out["af_ii"], out["af_jj"] = np.int64(ii), np.int64(jj)
    for case, reloc in (("add", False), ("reloc", True)):
        L = lambda dt: torch.as_tensor([], dtype=dt)
        fg = types.SimpleNamespace(
            model=None, device="cpu", cfg=cfg["local_opt"],
            frames=[types.SimpleNamespace(feat=torch.zeros(1, 2, 4), pos=torch.zeros(1, 2, 2),
                                          img_true_shape=torch.tensor([[hh, ww]]))] * 5,
            ii=L(torch.long), jj=L(torch.long), idx_ii2jj=L(torch.long), idx_jj2ii=L(torch.long),
            valid_match_j=L(torch.bool), valid_match_i=L(torch.bool),
            Q_ii2jj=L(torch.float32), Q_jj2ii=L(torch.float32))
        ret = fns["add_factors"](fg, ii, jj, cfg["local_opt"]["min_match_frac"], is_reloc=reloc)
        out[f"af_{case}_ret"] = np.bool_(bool(ret))
        for k in ("ii", "jj", "idx_ii2jj", "idx_jj2ii", "valid_match_j", "valid_match_i",
                  "Q_ii2jj", "Q_jj2ii"):
            out[f"af_{case}_{k}"] = getattr(fg, k).numpy()
        print("add_factors", case, "->", bool(ret), "edges", getattr(fg, "ii").tolist())

    # ---- match_iterative_proj glue (matching.py:8-90)
    def iter_proj(rays, pts, p_init, max_iter, lam, thr):
        p, c = oracle.iter_proj(rays.numpy(), pts.numpy(), p_init.numpy(), max_iter, lam, thr)
        return [torch.from_numpy(p), torch.from_numpy(c)]

    def refine(D11, D21, p1, radius, dil):
        return [torch.from_numpy(oracle.refine_matches(D11.numpy(), D21.numpy(), p1.numpy(),
                                                       radius, dil))]

    mns = {"torch": torch, "F": F, "img_utils": rimg, "config": cfg,
           "mast3r_slam_backends": types.SimpleNamespace(iter_proj=iter_proj,
                                                         refine_matches=refine)}
    _ast_defs(os.path.join(REF, "splatt3r_slam", "matching.py"),
              ["match", "pixel_to_lin", "lin_to_pixel", "prep_for_iter_proj",
               "match_iterative_proj"], mns)
    for c, (b, h, w, init) in enumerate(((2, 48, 64, False), (1, 40, 56, True))):
        r = np.random.default_rng(40 + c)
        v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
        X11 = np.stack([(u - w / 2) / w * 2, (v - h / 2) / w * 2, 2 + 0.3 * np.sin(u / 7.0)], -1)
        X11 = np.repeat(X11[None], b, 0) + r.normal(size=(b, h, w, 3)) * 0.002
        X21 = np.roll(X11, (1, 2), axis=(1, 2)) + r.normal(size=(b, h, w, 3)) * 0.002
        D11 = r.normal(size=(b, h, w, 24))
        D11 /= np.linalg.norm(D11, axis=-1, keepdims=True)
        D21 = np.roll(D11, (1, 2), axis=(1, 2)) + r.normal(size=(b, h, w, 24)) * 0.3
        D21 /= np.linalg.norm(D21, axis=-1, keepdims=True)
        X11, X21, D11, D21 = (a.astype(np.float32) for a in (X11, X21, D11, D21))
        idx0 = None
        if init:
            idx0 = torch.from_numpy(np.clip(np.arange(h * w) + r.integers(-3, 4, h * w), 0,
                                            h * w - 1)[None].repeat(b, 0))
        idx, valid = mns["match"](t(X11), t(X21), t(D11), t(D21), idx0)
        pre = f"mt{c}_"
        out.update({pre + "X11": X11, pre + "X21": X21, pre + "D11": D11, pre + "D21": D21,
                    pre + "idx": idx.numpy(), pre + "valid": valid.numpy()})
        if idx0 is not None:
            out[pre + "idx_init"] = idx0.numpy()
        print("match case", c, "valid frac", float(valid.float().mean()),
              "identity frac", float((idx.numpy() == np.arange(h * w)).mean()))
    np.savez_compressed(os.path.join(GOLDEN, "host_glue.npz"), **out)
    print("wrote host_glue.npz")


SECTIONS = {"host": gen_host, "matching": gen_matching, "render": gen_render, "net": gen_net, "net_c4": gen_net_c4, "net_c5": gen_net_c5, "n1": gen_n1, "mono": gen_mono, "resize": gen_resize, "viz": gen_viz, "portrait": gen_portrait}


def main(argv):
    if not os.path.isdir(REF):
        raise SystemExit("/root/reference not present: fixtures are generated in the build container")
    os.makedirs(GOLDEN, exist_ok=True)
    torch.set_grad_enabled(False)
    for s in (argv or list(SECTIONS)):
        SECTIONS[s]()


if __name__ == "__main__":
    main(sys.argv[1:])
