"""GPU-side per-frame spans of the pipelined frontend (tuning harness):
the encoder span on the side stream, the main-chain span (decoder, heads,
matching, tracking, render) on the current stream, and how much of the
frame period they overlap.  HIP events only, no profiler attached, so the
overlap is the one bench.py gets.

  python -m tools.profile_spans [--steps 20]
"""
from __future__ import annotations

import argparse
import time

import torch

from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    n = a.steps + 7
    frames = tum_like_sequence(n + 1, 384, 512, seed=0, step_px=2.0, device=dev)
    fe = Frontend(model, device=dev, spatial_stride=4, render=True)
    for i in range(5):
        fe.step(i, frames[i], next_img=frames[i + 1])
    torch.cuda.synchronize()
    # event marks at stage boundaries on the main stream (no syncs added)
    import splatt3r_amd.splatt3r_utils as su
    import splatt3r_amd.slam as sl
    import splatt3r_amd.tracker as trk
    marks = []

    def wrap(mod, name):
        fn = getattr(mod, name)

        def w(*x, **k):
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*x, **k)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            marks.append((name, e0, e1))
            return r
        setattr(mod, name, w)

    for mod, names in ((su, ["splatt3r_asymmetric_inference", "_extract_gaussian_params"]),
                       (su.matching, ["match"]),
                       (trk.FrameTracker, ["_gn_finish"]),
                       (sl, ["world_records", "splatt3r_render"])):
        for nm in names:
            wrap(mod, nm)
    fe.spans = []
    t0 = time.perf_counter()
    for i in range(5, 5 + a.steps):
        fe.step(i, frames[i], next_img=frames[i + 1])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    enc = {i: (e0, e1) for k, i, e0, e1 in fe.spans if k == "enc"}
    main_ = {i: (e0, e1) for k, i, e0, e1 in fe.spans if k == "main"}
    ref = main_[5][0]
    rows = []
    for i in range(6, 5 + a.steps):
        m0, m1 = main_[i]
        e0, e1 = enc[i + 1] if (i + 1) in enc else (None, None)
        r = dict(i=i, m0=ref.elapsed_time(m0), m1=ref.elapsed_time(m1))
        if e0 is not None:
            r["e0"], r["e1"] = ref.elapsed_time(e0), ref.elapsed_time(e1)
        rows.append(r)
    for r in rows:
        s = f"frame {r['i']:3d}: main {r['m0']:8.3f} -> {r['m1']:8.3f} ({r['m1'] - r['m0']:6.3f} ms)"
        if "e0" in r:
            s += f" | enc(next) {r['e0']:8.3f} -> {r['e1']:8.3f} ({r['e1'] - r['e0']:6.3f} ms)"
        print(s)
    ms = [r["m1"] - r["m0"] for r in rows]
    es = [r["e1"] - r["e0"] for r in rows if "e0" in r]
    per = [rows[j + 1]["m0"] - rows[j]["m0"] for j in range(len(rows) - 1)]
    gap = [rows[j + 1]["m0"] - rows[j]["m1"] for j in range(len(rows) - 1)]
    avg = lambda x: sum(x) / max(len(x), 1)
    agg = {}
    for nm, e0, e1 in marks:
        agg[nm] = agg.get(nm, 0.0) + e0.elapsed_time(e1)
    for nm, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"   stage {nm:36s} {v / a.steps:7.3f} ms/frame (GPU span, main stream)")
    print(f"host wall {wall:.3f} ms/frame; GPU frame period {avg(per):.3f} ms; "
          f"main span {avg(ms):.3f} ms; encoder span {avg(es):.3f} ms; "
          f"main idle between frames {avg(gap):.3f} ms")


if __name__ == "__main__":
    main()
