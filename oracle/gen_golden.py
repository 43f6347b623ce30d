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
    gen_full(384, 512, seed=6, write_manifest=True)


def gen_net_c4():
    """Full architecture at 320x512 (C4: EuRoC 752x480 -> 512x320 by the
    resize_img rule, splatt3r_utils.py:668-679; N = 640 tokens)."""
    gen_full(320, 512, seed=7)


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

    Reference head outputs (the committed net_small_* goldens, and the full
    architecture at 384x512 re-run here with the net_full_384x512 inputs) go
    through the reference glue exactly as splatt3r_render drives it
    (splatt3r_utils.py:332-432: build_covariance, RGB2SH residual,
    DecoderSplattingCUDA with default intrinsics f = max(h, w)), with a stub
    rasterizer capturing what the glue hands GaussianRasterizer; the captured
    inputs are rasterized by oracle.raster (the canonical graphdeco forward,
    oracle/raster_ref.c).  Saved: the rendered [3,H,W] images + the poses."""
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
    import dataclasses
    out = {}
    cases = []
    for tag, use_off in (("small_off", True), ("small_nooff", False)):
        g = np.load(os.path.join(GOLDEN, f"net_{tag}.npz"))
        im1, im2 = torch.from_numpy(g["img1"]), torch.from_numpy(g["img2"])
        r1 = {k: torch.from_numpy(g["res1_" + k]) for k in keys}
        r2 = {k: torch.from_numpy(g["res2_" + k]) for k in keys}
        cfg = dataclasses.replace(W.SMALL, use_offsets=use_off)
        torch.manual_seed(0)
        model = build_reference_model(cfg)
        load_prng(model, cfg, seed=1234)
        with tf32_mode():
            _, _, _, _, _, t1, t2 = run_reference(model, im1, im2)
        cases.append((tag, r1, r2, t1, t2, im1, im2))
        # matching on the TF32 reference outputs (splatt3r_match_asymmetric's
        # idx/valid as the reference CUDA path would produce them)
        idx_t, valid_t = oracle.match(t1["pts3d"].numpy(), t2["pts3d"].numpy(),
                                      t1["desc"].numpy(), t2["desc"].numpy())
        out[f"{tag}_match_tf32_idx"] = idx_t
        out[f"{tag}_match_tf32_valid"] = valid_t
    # full architecture at 384x512 (same inputs as net_full_384x512.npz)
    torch.manual_seed(0)
    model = build_reference_model(W.FULL)
    load_prng(model, W.FULL, seed=1234)
    g = torch.Generator().manual_seed(6)
    img1 = torch.rand(1, 3, 384, 512, generator=g) * 2 - 1
    img2 = torch.rand(1, 3, 384, 512, generator=g) * 2 - 1
    full = np.load(os.path.join(GOLDEN, "net_full_384x512.npz"))
    assert np.array_equal(full["img1"], img1.numpy())
    _, _, _, _, _, r1, r2 = run_reference(model, img1, img2)
    with tf32_mode():
        _, _, _, _, _, t1, t2 = run_reference(model, img1, img2)
    del model
    cases.append(("full_384x512", r1, r2, t1, t2, img1, img2))
    for tag, r1, r2, t1, t2, im1, im2 in cases:
        poses = dict(N1_POSES)
        # a target looking at view 1's point cloud from behind the origin
        # (portable-PRNG weights put the full model's points outside the
        # default frustum)
        poses["lookat"] = ([0.0, 0, 0, 0, 0, 0, 1, 1], _look_at(r1["means"]))
        for pname, (Tc, Tt) in poses.items():
            img, nr = render(r1, r2, im1, im2, Tc, Tt)
            img_t, _ = render(t1, t2, im1, im2, Tc, Tt)
            out[f"{tag}_{pname}_image"] = img
            out[f"{tag}_{pname}_image_tf32"] = img_t
            out[f"{tag}_{pname}_ctx"] = np.float32(Tc)
            out[f"{tag}_{pname}_tgt"] = np.float32(Tt)
            print(tag, pname, "num_rendered", nr, "mean", float(img.mean()),
                  "covered", float((img.sum(0) > 0).mean()),
                  "tf32-vs-fp32 mean-L1", float(np.abs(img - img_t).mean()))
    np.savez_compressed(os.path.join(GOLDEN, "n1_render.npz"), **out)
    del sys.modules["diff_gaussian_rasterization"]
    print("wrote n1_render.npz")


SECTIONS = {"matching": gen_matching, "render": gen_render, "net": gen_net, "net_c4": gen_net_c4, "n1": gen_n1, "mono": gen_mono, "resize": gen_resize, "viz": gen_viz, "portrait": gen_portrait}


def main(argv):
    if not os.path.isdir(REF):
        raise SystemExit("/root/reference not present: fixtures are generated in the build container")
    os.makedirs(GOLDEN, exist_ok=True)
    torch.set_grad_enabled(False)
    for s in (argv or list(SECTIONS)):
        SECTIONS[s]()


if __name__ == "__main__":
    main(sys.argv[1:])
