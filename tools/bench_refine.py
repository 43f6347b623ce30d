"""refine_matches on the tracking loop's own inputs:
the (D11, D21, p1) of the tracked frames' refine calls are captured from a
Frontend run, then every (lanes, window-centre binning) variant is timed on
each of them (HIP graph of `reps` calls on one stream, binning included) and
its output compared with the default's.  python -m tools.bench_refine"""
from __future__ import annotations

import torch

from splatt3r_amd import _lib, matching
from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL

# (16, 0) and (3, 0) run first and again last (clock drift check); the
# summary averages over every run of a variant
VARIANTS = [(16, 0), (3, 0), (3, 0x33), (3, 0x42), (3, 0x22), (16, 0x33), (1, 0x33), (4, 0x42),
            (16, 0), (3, 0)]


def timeit(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def main():
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    frames = tum_like_sequence(16, 384, 512, seed=0, step_px=2.0, device=dev)
    seen = []
    orig = matching.refine_matches

    def spy(D11, D21, p1, radius, dilation_max):
        seen.append((D11.clone(), D21.clone(), p1.clone(), radius, dilation_max))
        return orig(D11, D21, p1, radius, dilation_max)

    matching.refine_matches = spy
    fe = Frontend(model, device=dev, spatial_stride=4, render=False)
    for i in range(12):
        fe.step(i, frames[i])
    torch.cuda.synchronize()
    matching.refine_matches = orig
    L = _lib.lib()
    tot = {v: 0.0 for v in VARIANTS}
    runs = {v: 0 for v in VARIANTS}
    calls = seen[2:10]
    for c, (D11, D21, p1, r, dil) in enumerate(calls):
        b, h, w, f = D11.shape
        n = D21.shape[1]
        out = torch.empty_like(p1)

        def fn():
            _lib.call("s3m_refine_matches", D11.data_ptr(), D21.data_ptr(), p1.data_ptr(),
                      out.data_ptr(), b, h, w, n, f, r, dil, _lib.stream())

        L.s3m_refine_set_lanes(16)
        L.s3m_refine_set_sort(0)
        fn()
        ref = out.clone()
        line = f"call {c} b={b} n={n} r={r} dil={dil}:"
        for lanes, mode in VARIANTS:
            L.s3m_refine_set_lanes(lanes)
            L.s3m_refine_set_sort(mode)
            out.fill_(-1)
            fn()
            same = bool(torch.equal(out, ref))
            t = timeit(fn)
            tot[(lanes, mode)] += t
            runs[(lanes, mode)] += 1
            line += f" [{lanes},{mode:#x}] {t:6.1f}{'' if same else ' DIFF'}"
        print(line, flush=True)
    L.s3m_refine_set_lanes(-1)
    L.s3m_refine_set_sort(-1)
    for v, t in sorted(tot.items(), key=lambda kv: kv[1] / runs[kv[0]]):
        print(f"lanes {v[0]:2d} sort {v[1]:#04x}: mean {t / runs[v]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
