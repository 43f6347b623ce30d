"""HBM traffic of the network kernels from rocprofv3 PMC counters.

Two steps (gpurun_traffic.sh runs both):

  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D1 -- \\
      python3 -m tools.pmc_traffic run
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D2 -- \\
      python3 -m tools.pmc_traffic run
  python -m tools.pmc_traffic summarize D1 D2 --out traffic.json

`run` builds the full-size network plans (512x384, the bench's model),
warms them, then replays one frame's network (encoder plan + pair plan)
`--reps` times eagerly, each replay bracketed by a GPU sleep (`spin`)
kernel so the summary can cut the dispatch stream into frames.

`run --workload raster` replays the C3 rasterizer microbench instead
(4,194,304 splats at 960x540, forward + backward through
GaussianRasterizer), one replay per frame marker.

`summarize` applies the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports
half the bytes of wide coalesced reads -> x2; WRITE_SIZE is exact for
16-B/lane stores.  FETCH_SIZE/WRITE_SIZE are in KiB.  Output: per kernel
family, HBM bytes per frame and per launch (mean over the replays).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def _family(name: str) -> str:
    if "k_gemm_bd<" in name:          # B-direct tiles: dense A only
        return "gemm_dense"
    # k_gemm / k_gemm_pp <BM, BN, NWM, NWN, AMODE, ...>: AMODE 0 = dense
    m = re.search(r"k_gemm(?:_pp)?<(\d+), (\d+), \d+, \d+, (\d+),", name)
    if m:
        return "gemm_dense" if m.group(3) == "0" else "gemm_conv"
    if "k_conv3_halo" in name:        # halo-reuse conv tiles: the conv GEMM family
        return "gemm_conv"
    m = re.search(r"\b(k_\w+)", name)
    return m.group(1) if m else name[:40]


def run_raster(reps: int) -> None:
    import torch
    from tools.bench_raster import prepare
    from diff_gaussian_rasterization import GaussianRasterizer
    sc, rs, inputs, grad = prepare(4_194_304)
    rast = GaussianRasterizer(rs)
    leaf = {k: v.clone().requires_grad_(True) for k, v in inputs.items()}

    def step():
        for v in leaf.values():
            v.grad = None
        m2 = torch.zeros_like(leaf["means3D"], requires_grad=True)
        img, _ = rast(means3D=leaf["means3D"], means2D=m2, opacities=leaf["opacities"],
                      shs=leaf["shs"], cov3D_precomp=leaf["cov3D_precomp"])
        (img * grad).sum().backward()

    step()
    torch.cuda.synchronize()
    for _ in range(reps):
        torch.cuda._sleep(1000)
        step()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print("pmc_traffic run: done", reps, "raster forward+backward")


def run(reps: int, kb: int = 1, bp: int = 1, mix=None) -> None:
    """One rep = kb frames: one encoder replay of kb images and kb / bp
    replays of the Bp = bp pair plan (the bench's frame composition with
    --enc-batch kb and, for bp = 2, --decode-ahead with every slot used).
    mix = (frames, encoder replays, Bp=2 replays, Bp=1 replays) per rep
    instead: the bench's timed composition (frame_breakdown.decode_ahead:
    paired frames share a Bp = 2 replay, the others decode alone)."""
    if mix is not None:
        return _run_mix(reps, kb, mix)
    import torch
    from splatt3r_amd import weights as W
    from splatt3r_amd.net import Splatt3RNet
    if kb % bp:
        raise SystemExit("kb must be a multiple of bp")
    H, Wd = 384, 512
    net = Splatt3RNet(W.FULL, seed=1234, graphs=False)
    img = torch.rand(kb, 3, H, Wd, device="cuda") * 2 - 1
    f, p, _ = net._encode_image(img)
    fb, pb = f[:1].expand(bp, -1, -1), p[:1].expand(bp, -1, -1)
    net.infer_pair(fb, pb, fb, pb, (H, Wd))
    enc = net.encoder_plan(kb, H, Wd).plan
    pair = net.pair_plan(bp, H, Wd)
    plans = [enc] + [pair.decoder_plan, pair.head_plan] * (kb // bp)
    torch.cuda.synchronize()
    for plan in plans:
        plan.run()
    torch.cuda.synchronize()
    for _ in range(reps):
        torch.cuda._sleep(1000)
        for plan in plans:
            plan.run()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print("pmc_traffic run: done", reps, "reps of", kb, "frames")


def _run_mix(reps: int, kb: int, mix) -> None:
    import torch
    from splatt3r_amd import weights as W
    from splatt3r_amd.net import Splatt3RNet
    frames, n_enc, n_p2, n_p1 = mix
    H, Wd = 384, 512
    net = Splatt3RNet(W.FULL, seed=1234, graphs=False)
    img = torch.rand(kb, 3, H, Wd, device="cuda") * 2 - 1
    f, p, _ = net._encode_image(img)
    for bp in (1, 2):
        fb, pb = f[:1].expand(bp, -1, -1), p[:1].expand(bp, -1, -1)
        net.infer_pair(fb, pb, fb, pb, (H, Wd))
    enc = net.encoder_plan(kb, H, Wd).plan
    p2, p1 = net.pair_plan(2, H, Wd), net.pair_plan(1, H, Wd)
    plans = ([enc] * n_enc + [p2.decoder_plan, p2.head_plan] * n_p2
             + [p1.decoder_plan, p1.head_plan] * n_p1)
    torch.cuda.synchronize()
    for plan in plans:
        plan.run()
    torch.cuda.synchronize()
    for _ in range(reps):
        torch.cuda._sleep(1000)
        for plan in plans:
            plan.run()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print("pmc_traffic run: done", reps, "reps of", frames, "frames (mix)")


def _load(d: str, counter: str):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = {}
    for path in paths:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                key = int(r["Dispatch_Id"])
                v = disp.setdefault(key, [r["Kernel_Name"], 0.0])
                v[1] += float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def _frames(rows, reps: int, marker: str):
    idx = [i for i, (n, _) in enumerate(rows) if re.search(marker, n)]
    if len(idx) < reps + 1:
        names = sorted({n for n, _ in rows})
        raise SystemExit(f"found {len(idx)} marker dispatches; kernel names: {names[:60]}")
    idx = idx[-(reps + 1):]
    return [rows[a + 1:b] for a, b in zip(idx[:-1], idx[1:])]


def summarize(fetch_dir: str, write_dir: str, reps: int, marker: str, workload: str = "network",
              kb: int = 1, bp: int = 1, mix=None):
    out = {}
    for counter, d, scale in (("FETCH_SIZE", fetch_dir, 2.0), ("WRITE_SIZE", write_dir, 1.0)):
        frames = _frames(_load(d, counter), reps, marker)
        agg = defaultdict(lambda: [0, 0.0])
        for fr in frames:
            for name, kib in fr:
                a = agg[_family(name)]
                a[0] += 1
                a[1] += kib * 1024.0 * scale
        nf = reps * (mix[0] if mix else kb)     # frames
        for fam, (n, b) in agg.items():
            o = out.setdefault(fam, {"launches_per_frame": n / nf})
            o[("read" if counter == "FETCH_SIZE" else "write") + "_bytes_per_frame"] = b / nf
    for o in out.values():
        o["bytes_per_frame"] = o.get("read_bytes_per_frame", 0.0) + o.get("write_bytes_per_frame", 0.0)
        o["bytes_per_launch"] = o["bytes_per_frame"] / max(1e-9, o["launches_per_frame"])
    return {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                      "FETCH_SIZE x2 (gfx950 correction), KiB -> bytes",
            "workload": ((f"512x384 frames of the network (encoder + decoder + 2 heads), eager; "
                          f"the bench's timed composition: per {mix[0]} frames {mix[1]} encoder "
                          f"replays of batch {kb}, {mix[2]} Bp=2 and {mix[3]} Bp=1 pair replays; "
                          f"per frame") if mix else
                         (f"512x384 frames of the network (encoder + decoder + 2 heads), eager; "
                          f"encoder batch {kb}, pair plan Bp={bp} ({kb // bp} pair replays per "
                          f"encoder replay), per frame")
                         if workload == "network" else
                         "C3 rasterizer: 4,194,304 splats at 960x540, forward + backward "
                         "(GaussianRasterizer, torch elementwise kernels included)"),
            "frames": reps, "families": dict(sorted(out.items(), key=lambda kv: -kv[1]["bytes_per_frame"]))}


def _mix(v):
    return tuple(int(x) for x in v.split(",")) if v else None


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--reps", type=int, default=3)
    r.add_argument("--workload", choices=("network", "raster"), default="network")
    r.add_argument("--kb", type=int, default=1, help="encoder batch (frames per rep)")
    r.add_argument("--bp", type=int, default=1, help="pairs per pair-plan replay")
    r.add_argument("--mix", default=None,
                   help="frames,encoder replays,Bp=2 replays,Bp=1 replays per rep")
    s = sub.add_parser("summarize")
    s.add_argument("--kb", type=int, default=1)
    s.add_argument("--bp", type=int, default=1)
    s.add_argument("--mix", default=None)
    s.add_argument("fetch_dir")
    s.add_argument("write_dir")
    s.add_argument("--reps", type=int, default=3)
    s.add_argument("--marker", default=r"spin|sleep")
    s.add_argument("--out", default=None)
    s.add_argument("--workload", choices=("network", "raster"), default="network")
    a = ap.parse_args()
    if a.cmd == "run":
        if a.workload == "raster":
            run_raster(a.reps)
        else:
            run(a.reps, a.kb, a.bp, _mix(a.mix))
        return
    res = summarize(a.fetch_dir, a.write_dir, a.reps, a.marker, a.workload, a.kb, a.bp,
                    _mix(a.mix))
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
