"""Live-camera leg A/B (diagnostic): the same bench_live run fresh, after
another live run, after the end-to-end leg, and with normal stream
priority.  python -m tools.live_ab"""
from __future__ import annotations

import torch

import bench
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def main():
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    frames = tum_like_sequence(64, 384, 512, seed=0, step_px=2.0, device=dev)

    def live(tag, prio=-1):
        r = bench.bench_live(model, dev, frames, 20, 5, prio)
        print(f"{tag:28s} live {r['frames_per_s']:6.1f} fps  p50 {r['latency_ms']['p50']:6.2f} ms",
              flush=True)

    live("fresh")
    live("second live run")
    live("priority 0", prio=0)
    e = bench.bench_end_to_end(model, dev, 20, 5, -1, enc_batch=8, enc_ahead=8, decode_ahead=True)
    print(f"end_to_end {e['frames_per_s']:.1f}", flush=True)
    live("after e2e")
    live("after e2e, priority 0", prio=0)
    torch.cuda.empty_cache()
    live("after e2e + empty_cache")


if __name__ == "__main__":
    main()
