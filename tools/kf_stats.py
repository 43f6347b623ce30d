"""Keyframe statistics of the synthetic C2 sequence (diagnostic).

  python -m tools.kf_stats [--frames 40] [--step 2.0 1.0 0.5]

For each pan speed (px per frame) runs the frontend over the synthetic
TUM-shaped sequence and prints, per tracked frame, the tracker's match
fractions (valid_opt, match_frac_k, unique_frac_f; new keyframe when
min(match_frac_k, unique_frac_f) < match_frac_thresh) and the keyframe rate."""
from __future__ import annotations

import argparse

import torch

from splatt3r_amd.slam import Frontend
from splatt3r_amd.splatt3r_utils import load_splatt3r
from splatt3r_amd.synthetic import tum_like_sequence
from splatt3r_amd.weights import FULL


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--step", type=float, nargs="+", default=[2.0, 1.0, 0.5])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    for step in a.step:
        frames = tum_like_sequence(a.frames, 384, 512, seed=0, step_px=step, device=dev)
        fe = Frontend(model, device=dev, spatial_stride=4, render=False)
        rows = []
        for i in range(a.frames):
            nkf = fe.stats["keyframes"]
            fe.step(i, frames[i])
            if i > 0:
                fr = getattr(fe.tracker, "last_fracs", (float("nan"),) * 3)
                rows.append((i, fe.stats["keyframes"] > nkf) + tuple(fr))
        st = fe.stats
        print(f"step_px {step}: keyframes {st['keyframes']} of {a.frames} frames, "
              f"reloc {st['reloc']}, gn_iters_avg {st['gn_iters'] / max(1, st['tracked']):.2f}")
        for i, kf, fo, fk, fu in rows:
            print(f"  frame {i:3d} kf={int(kf)} valid_opt={fo:.3f} match_k={fk:.3f} unique_f={fu:.3f}")


if __name__ == "__main__":
    main()
