"""Where the frame loop's device copies come from (diagnostic): torch
profiler (CPU ops with Python stacks) over `--steps` frames of the bench's
default frame loop; every aten copy-like op counted per frame, grouped by
its innermost call site inside the package.

  python -m tools.copy_sites [--steps 20]
"""
from __future__ import annotations

import argparse
import collections

import torch

from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL

OPS = ("aten::copy_", "aten::clone", "aten::cat", "aten::stack", "aten::contiguous",
       "aten::_to_copy", "aten::fill_", "aten::zero_", "aten::index", "aten::where",
       "aten::nonzero", "aten::item", "aten::_local_scalar_dense")


def site(stack):
    for fr in stack or []:
        if any(k in fr for k in ("splatt3r_amd/", "diff_gaussian_rasterization/", "lietorch/",
                                 "mast3r_slam_backends/")):
            return fr.split("splatt3r-slam_amd/")[-1]
    return (stack or ["?"])[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    n = 24 + a.steps
    frames = tum_like_sequence(n + 16, 384, 512, seed=0, step_px=2.0, device=dev)
    fe = Frontend(model, device=dev, spatial_stride=4, render=True, enc_batch=8,
                  enc_ahead=8, decode_ahead=True, main_priority=-1)
    nxt = lambda i: [frames[j] for j in range(i + 1, i + 17)]
    for i in range(24):
        fe.step(i, frames[i], next_img=nxt(i))
    torch.cuda.synchronize()
    import traceback
    cnt = collections.Counter()

    def where():
        for fr in reversed(traceback.extract_stack()[:-2]):
            f = fr.filename
            if any(k in f for k in ("splatt3r_amd/", "diff_gaussian_rasterization/", "lietorch/",
                                    "mast3r_slam_backends/")):
                return f"{f.split('splatt3r-slam_amd/')[-1]}:{fr.lineno}"
        return "?"

    T = torch.Tensor
    orig = {"clone": T.clone, "copy_": T.copy_, "contiguous": T.contiguous, "item": T.item,
            "cat": torch.cat, "stack": torch.stack}

    def wrap(name, fn, method=True):
        def w(*args, **kw):
            t = args[0] if method else (args[0][0] if args and len(args[0]) else None)
            if torch.is_tensor(t) and t.is_cuda and not (name == "contiguous" and t.is_contiguous()):
                src = args[1] if name == "copy_" and len(args) > 1 else None
                kind = name
                if name == "copy_" and torch.is_tensor(src):
                    kind = f"copy_ {src.device.type}->{t.device.type}"
                cnt[(kind, where())] += 1
            elif name == "copy_" and torch.is_tensor(t) and len(args) > 1 and \
                    torch.is_tensor(args[1]) and args[1].is_cuda:
                cnt[("copy_ cuda->cpu", where())] += 1
            return fn(*args, **kw)
        return w

    for k in ("clone", "copy_", "contiguous", "item"):
        setattr(T, k, wrap(k, orig[k]))
    torch.cat = wrap("cat", orig["cat"], method=False)
    torch.stack = wrap("stack", orig["stack"], method=False)
    try:
        for i in range(24, n):
            fe.step(i, frames[i], next_img=nxt(i))
        torch.cuda.synchronize()
    finally:
        for k in ("clone", "copy_", "contiguous", "item"):
            setattr(T, k, orig[k])
        torch.cat, torch.stack = orig["cat"], orig["stack"]
    for (name, s), c in cnt.most_common(40):
        print(f"{c / a.steps:6.2f}/frame  {name:20s} {s}", flush=True)


if __name__ == "__main__":
    main()
