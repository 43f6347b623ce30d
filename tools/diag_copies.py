"""Where the frame loop's device copies come from: the headline frontend
(encoder batch 8, 8 ahead, decode-ahead) runs 24 frames, the last 16 under
torch.profiler with Python stacks; every aten copy-like op (copy_, clone,
contiguous, cat, to, index ...) is counted per frame by its innermost
call site in splatt3r_amd.  GPU only; prints a table."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "splatt3r-slam_amd"))

from splatt3r_amd.slam import Frontend  # noqa: E402
from splatt3r_amd.splatt3r_utils import load_splatt3r  # noqa: E402
from splatt3r_amd.synthetic import tum_like_sequence  # noqa: E402
from splatt3r_amd.weights import FULL  # noqa: E402

OPS = ("aten::copy_", "aten::clone", "aten::cat", "aten::contiguous", "aten::to",
       "aten::_to_copy", "aten::index", "aten::stack", "aten::fill_", "aten::zero_",
       "aten::zeros", "aten::ones", "aten::full", "aten::index_put_", "aten::masked_fill_")


def main():
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    n, warm = 24, 8
    frames = tum_like_sequence(n + 10, 384, 512, seed=3, step_px=2.0, device=dev)
    fe = Frontend(model, device=dev, spatial_stride=4, render=True, enc_batch=8, enc_ahead=8,
                  decode_ahead=True, main_priority=-1)
    for i in range(warm):
        fe.step(i, frames[i], next_img=[frames[j] for j in range(i + 1, min(n, i + 9))])
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                            torch.profiler.ProfilerActivity.CUDA],
                                with_stack=True, record_shapes=True) as prof:
        for i in range(warm, n):
            fe.step(i, frames[i], next_img=[frames[j] for j in range(i + 1, min(n, i + 9))])
        torch.cuda.synchronize()
    nf = n - warm
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        stack = [s for s in (ev.stack or []) if "splatt3r_amd" in s]
        site = stack[0] if stack else "(no splatt3r_amd frame)"
        site = site.split("splatt3r_amd/")[-1]
        sites[(ev.name, site, str(ev.input_shapes)[:60])] += 1
    gpu = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and ("copy" in ev.name.lower()
                                                                  or "Memcpy" in ev.name):
            gpu[ev.name[:60]] += 1
    print(f"GPU copy kernels per frame over {nf} frames:")
    for k, c in gpu.most_common(12):
        print(f"  {c / nf:6.2f}  {k}")
    print("aten copy-like ops per frame by call site:")
    for (name, site, shp), c in sites.most_common(45):
        print(f"  {c / nf:6.2f}  {name:18s} {site[:70]:70s} {shp}")
    fe.close()


if __name__ == "__main__":
    main()
