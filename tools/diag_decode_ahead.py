"""Localise a decode-ahead mismatch (tests/test_slam.py::
test_decode_ahead_frontend_matches_sequential): run the frame-by-frame
frontend and the decode-ahead + batch-2 encoder frontend on the same
sequence and, per tracked frame, compare the tracker's decoder inputs
(both frames' encoder features) and outputs (X, C, D, Q).  The records are
stream-ordered clones taken where the tracker reads them (no host syncs, so
the timing under test is not perturbed).  GPU only; prints one line per frame.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "splatt3r-slam_amd"))

from splatt3r_amd import splatt3r_utils as U  # noqa: E402
from splatt3r_amd.slam import Frontend  # noqa: E402
from splatt3r_amd.splatt3r_utils import load_splatt3r  # noqa: E402
from splatt3r_amd.synthetic import tum_like_sequence  # noqa: E402
from splatt3r_amd.weights import FULL  # noqa: E402

REC = []
_orig = U._tracker_decode


def _rec(model, frame_i, frame_j, ahead=None):
    out = _orig(model, frame_i, frame_j, ahead)
    res_self, res_cross, d16 = out
    r = {"fi": frame_i.feat.clone(), "fj": frame_j.feat.clone(), "id": frame_i.frame_id,
         "kf": frame_j.frame_id}
    for n, res in (("s", res_self), ("c", res_cross)):
        for k in ("pts3d", "conf", "desc", "desc_conf"):
            if k in res:
                r[n + k] = res[k].clone()
    REC.append(r)
    return out


U._tracker_decode = _rec

MREC = []
_orig_match = U.matching.match


def _mrec(X1, X2, D1, D2, idx_1_to_2_init=None):
    out = _orig_match(X1, X2, D1, D2, idx_1_to_2_init=idx_1_to_2_init)
    r = {"X1": X1.clone(), "X2": X2.clone(), "D1": D1.clone(), "D2": D2.clone(),
         "idx": out[0].clone(), "valid": out[1].clone()}
    if idx_1_to_2_init is not None:
        r["init"] = idx_1_to_2_init.clone()
    MREC.append(r)
    return out


U.matching.match = _mrec

from splatt3r_amd import tracker as T  # noqa: E402

PREC = []
_orig_prep = T.track_prep


def _prec(idx, valid, Xf_all, Cf_all, Ck, Qff, Qkf, *a):
    out = _orig_prep(idx, valid, Xf_all, Cf_all, Ck, Qff, Qkf, *a)
    r = {"in_Xf": Xf_all.clone(), "in_Cf": Cf_all.clone(), "in_Ck": Ck.clone(),
         "in_Qff": Qff.clone(), "in_Qkf": Qkf.clone()}
    for k, v in zip(("Xf", "Qk", "valid_opt", "stats"), out):
        r[k] = v.clone()
    PREC.append(r)
    return out


T.track_prep = _prec

if os.environ.get("DIAG_ENC_SLEEP"):
    # delay every encoder batch on its stream (GPU sleep of N cycles queued
    # ahead of it): same kernels, shifted overlap with the main chain
    _orig_prefetch0 = Frontend._prefetch
    _cycles = int(os.environ["DIAG_ENC_SLEEP"])

    def _sleep_prefetch(self, i, imgs):
        with torch.cuda.stream(self.enc_stream):
            torch.cuda._sleep(_cycles)
        _orig_prefetch0(self, i, imgs)

    Frontend._prefetch = _sleep_prefetch

if os.environ.get("DIAG_ENC_SERIAL") == "1":
    # the main chain waits for every encoder batch as soon as it is queued:
    # no encoder replay overlaps main-stream work
    _orig_prefetch = Frontend._prefetch

    def _serial_prefetch(self, i, imgs):
        _orig_prefetch(self, i, imgs)
        torch.cuda.current_stream(self.device).wait_stream(self.enc_stream)

    Frontend._prefetch = _serial_prefetch


def run(model, frames, n, ahead, kb):
    REC.clear()
    MREC.clear()
    PREC.clear()
    mp = os.environ.get("DIAG_MAIN_PRIORITY")
    fe = Frontend(model, device=frames[0].device, spatial_stride=4, render=True,
                  enc_batch=kb, enc_ahead=3 if kb > 1 else None, decode_ahead=ahead,
                  main_priority=None if mp is None else int(mp))
    poses = []
    for i in range(n):
        nxt = [frames[j] for j in range(i + 1, min(n, i + 6))]
        f = fe.step(i, frames[i], next_img=nxt)
        poses.append(f.T_WC.data.clone())
    torch.cuda.synchronize()
    fe.close()
    return poses, list(REC), list(MREC), list(PREC)


def recheck(mrec, tag):
    """Recompute each recorded matching call from its recorded inputs on an
    idle device; report the calls whose live outputs differ."""
    torch.cuda.synchronize()
    for j, r in enumerate(mrec):
        idx, valid = _orig_match(r["X1"], r["X2"], r["D1"], r["D2"],
                                 idx_1_to_2_init=r.get("init"))
        torch.cuda.synchronize()
        bad_i = (idx != r["idx"]).reshape(-1)
        bad_v = (valid != r["valid"]).reshape(-1)
        if bad_i.any() or bad_v.any():
            pos = torch.nonzero(bad_i | bad_v).reshape(-1)
            print(f"  {tag} match {j}: live != recomputed at {int(pos.numel())} of "
                  f"{bad_i.numel()} pixels (first {pos[:8].tolist()}, idx {int(bad_i.sum())}, "
                  f"valid {int(bad_v.sum())})", flush=True)


def main():
    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    n = 12
    frames = tum_like_sequence(n + 6, 384, 512, seed=3, step_px=2.0, device=dev)
    p0, r0, m0, q0 = run(model, frames, n, False, 1)
    recheck(m0, "sequential")
    for trial in range(int(os.environ.get("DIAG_TRIALS", "2"))):
        p1, r1, m1, q1 = run(model, frames, n, True, 2)
        recheck(m1, f"trial {trial}")
        print(f"trial {trial}: pose diffs", [f"{float((a - b).abs().max()):.1e}" for a, b in zip(p0, p1)])
        for a, b in zip(r0, r1):
            diffs = {k: float((a[k].float() - b[k].float()).abs().max()) for k in a
                     if isinstance(a[k], torch.Tensor) and k in b}
            bad = {k: f"{v:.1e}" for k, v in diffs.items() if v != 0.0}
            print(f"  frame {a['id']} (kf {a['kf']} / {b['kf']}):", bad or "identical", flush=True)
        for j, (a, b) in enumerate(zip(m0, m1)):
            diffs = {k: float((a[k].float() - b[k].float()).abs().max()) for k in a if k in b}
            bad = {k: f"{v:.1e}" for k, v in diffs.items() if v != 0.0}
            print(f"  match {j}:", bad or "identical", flush=True)
        for j, (a, b) in enumerate(zip(q0, q1)):
            diffs = {k: float((a[k].float() - b[k].float()).abs().max()) for k in a if k in b}
            bad = {k: f"{v:.1e}" for k, v in diffs.items() if v != 0.0}
            print(f"  prep {j}:", bad or "identical", flush=True)


if __name__ == "__main__":
    main()
