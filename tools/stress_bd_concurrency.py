"""Cross-stream interference check without the frontend: the encoder plan
(batch 2, C2 size) replays back to back on a side stream while the main
stream runs the dense matching pipeline (matching.match) on fixed inputs
again and again; every main-stream result is compared with the result of
the same call on an idle device.  Prints the number of mismatching calls /
pixels.  Run once with the default tiles and once with
S3_GEMM_BDIRECT_OFF=enc (no B-direct tiles in the encoder plans).  GPU only.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "splatt3r-slam_amd"))

from splatt3r_amd import matching  # noqa: E402
from splatt3r_amd import weights as W  # noqa: E402
from splatt3r_amd.net import Splatt3RNet  # noqa: E402


def make_side(dev, g):
    """The side-stream aggressor (STRESS_SIDE): enc = the encoder plan
    (batch 2); torch = fp16 matmuls + elementwise ops (no library kernel);
    gemm<T> = one library GEMM 1536x4096x1024 forced to tile T."""
    kind = os.environ.get("STRESS_SIDE", "enc")
    if kind == "enc":
        net = Splatt3RNet(W.FULL, seed=1234, device=dev)
        img = torch.rand(2, 3, 384, 512, device=dev, generator=g) * 2 - 1
        net._encode_image(img)                   # build + capture the batch-2 plan
        return kind, lambda: net._encode_image(img)
    if kind == "torch":
        a = torch.randn(4096, 4096, device=dev, generator=g).half()
        b = torch.randn(4096, 4096, device=dev, generator=g).half()

        def run():
            c = a @ b
            (c * 0.5 + 1.0).relu_()
        return kind, run
    if kind == "torchs":
        a = torch.randn(1536, 1024, device=dev, generator=g).half()
        b = torch.randn(1024, 4096, device=dev, generator=g).half() * 0.03

        def run():
            for _ in range(8):
                torch.nn.functional.gelu(a @ b)
        return kind, run
    if kind.startswith("gemm"):
        from splatt3r_amd import _lib, ops
        tile = int(kind[4:])
        M, N, K = 1536, 4096, 1024
        A = torch.randn(M, K, device=dev, generator=g).half()
        Bw = torch.randn(N, K, device=dev, generator=g).half() * 0.03
        C = torch.empty(M, N, device=dev).half()
        bias = torch.zeros(N, device=dev)
        call = ops.gemm([A], [Bw], [C], M, N, K, lda=K, bias=[bias], act="gelu", tile=tile,
                        split_k=1)

        dbg = int(os.environ.get("STRESS_GEMM_DEBUG", "0"))
        if dbg:
            # k_gemm debug bits: 1 no MFMA, 2 no LDS-DMA, 4 no epilogue, 8 no K loop
            _lib.lib().s3n_gemm_set_debug(dbg)
            kind += f"/debug{dbg}"

        def run():
            for _ in range(8):
                call(_lib.stream())
        return kind, run
    raise ValueError(kind)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    side_kind, side_run = make_side(dev, g)
    h, w = 384, 512
    yy, xx = torch.meshgrid(torch.arange(h, device=dev, dtype=torch.float32),
                            torch.arange(w, device=dev, dtype=torch.float32), indexing="ij")
    X11 = torch.stack((xx / w - 0.5, yy / h - 0.5, torch.ones_like(xx)), -1)[None]
    X21 = X11 + 0.002 * torch.randn(X11.shape, device=dev, generator=g)
    D11 = torch.randn(1, h, w, 24, device=dev, generator=g).half()
    D21 = D11 + 0.05 * torch.randn(D11.shape, device=dev, generator=g).half()
    victim = os.environ.get("STRESS_VICTIM", "match")
    xv = torch.randn(1 << 23, device=dev, generator=g)
    q = torch.nn.functional.normalize(torch.randn(2, 4, device=dev, generator=g), dim=-1)
    Tv = torch.cat([torch.randn(2, 3, device=dev, generator=g), q,
                    torch.rand(2, 1, device=dev, generator=g) + 0.5], -1)
    Pts = torch.randn(1, h * w, 3, device=dev, generator=g)

    # fixed inputs of each matching stage (victim = stage_<name>)
    from splatt3r_amd import _lib
    from splatt3r_amd.config import config
    cfg = config["matching"]
    npx = h * w
    rays0, pts0, pinit0 = matching.prep_for_iter_proj(X11, X21, None)
    p0 = torch.empty(1, npx, 2, device=dev)
    conv0 = torch.empty(1, npx, device=dev, dtype=torch.bool)
    _lib.call("s3m_iter_proj", rays0.data_ptr(), pts0.data_ptr(), pinit0.data_ptr(),
              p0.data_ptr(), conv0.data_ptr(), 1, h, w, npx, int(cfg["max_iter"]),
              float(cfg["lambda_init"]), float(cfg["convergence_thresh"]), _lib.stream(dev))
    p1_0 = torch.empty(1, npx, 2, device=dev, dtype=torch.int64)
    valid0 = torch.empty(1, npx, device=dev, dtype=torch.bool)
    _lib.call("s3m_occlusion", p0.data_ptr(), conv0.data_ptr(), X11.data_ptr(),
              X21.data_ptr(), p1_0.data_ptr(), valid0.data_ptr(), 1, h, w,
              float(cfg["dist_thresh"]), _lib.stream(dev))
    D21r = D21.reshape(1, npx, -1).contiguous()

    def stage(name):
        st = _lib.stream(dev)
        if name == "prep":
            r, q, pi = matching.prep_for_iter_proj(X11, X21, None)
            return torch.cat((r.reshape(-1), q.reshape(-1), pi.reshape(-1))), None
        if name == "iter":
            p = torch.empty(1, npx, 2, device=dev)
            c = torch.empty(1, npx, device=dev, dtype=torch.bool)
            _lib.call("s3m_iter_proj", rays0.data_ptr(), pts0.data_ptr(), pinit0.data_ptr(),
                      p.data_ptr(), c.data_ptr(), 1, h, w, npx, int(cfg["max_iter"]),
                      float(cfg["lambda_init"]), float(cfg["convergence_thresh"]), st)
            return p, c
        if name == "occl":
            q = torch.empty(1, npx, 2, device=dev, dtype=torch.int64)
            v = torch.empty(1, npx, device=dev, dtype=torch.bool)
            _lib.call("s3m_occlusion", p0.data_ptr(), conv0.data_ptr(), X11.data_ptr(),
                      X21.data_ptr(), q.data_ptr(), v.data_ptr(), 1, h, w,
                      float(cfg["dist_thresh"]), st)
            return q, v
        if name == "refine":
            return matching.refine_matches(D11, D21r, p1_0, int(cfg["radius"]),
                                           int(cfg["dilation_max"])), None
        raise ValueError(name)

    def victim_run():
        if victim.startswith("stage_"):
            a, b = stage(victim[6:])
            return a, (b if b is not None else a[:1])
        if victim == "torch":
            y = torch.sin(xv) * 1.5 + xv * xv
            return y, (y > 0.5)
        if victim == "lie":
            # the frame loop's pose algebra (lietorch Sim3 compose / inverse /
            # act on a pointmap) and small torch glue, as on the main chain
            import lietorch
            Ta = lietorch.Sim3(Tv[0:1])
            Tb = lietorch.Sim3(Tv[1:2])
            Tc = Ta.inv() * Tb
            Xw = Tc.act(Pts)
            return Xw.contiguous(), (Tc.data * 1.0)
        if victim == "torch64":
            xd = xv.double()
            y = (1.0 / (xd + 4.0)) * 1.5 + xd * xd
            return y, (y > 0.5)
        return matching.match(X11, X21, D11, D21)

    torch.cuda.synchronize()
    ref_idx, ref_valid = victim_run()
    torch.cuda.synchronize()

    side = torch.cuda.Stream(device=dev)
    secs = float(os.environ.get("STRESS_SECONDS", "20"))
    t_end = time.time() + secs
    calls = bad_calls = bad_px = enc_runs = 0
    outs = []
    while time.time() < t_end:
        with torch.cuda.stream(side):
            for _ in range(2):
                side_run()
                enc_runs += 1
        for _ in range(8):
            outs.append(victim_run())
        if len(outs) >= 64:
            torch.cuda.synchronize()
            for idx, valid in outs:
                calls += 1
                n = int((idx != ref_idx).sum()) + int((valid != ref_valid).sum())
                if n:
                    bad_calls += 1
                    bad_px += n
            outs = []
            print(f"[stress] {calls} calls, {bad_calls} corrupted ({bad_px} px), "
                  f"{enc_runs} encoder replays", flush=True)
    torch.cuda.synchronize()
    for idx, valid in outs:
        calls += 1
        n = int((idx != ref_idx).sum()) + int((valid != ref_valid).sum())
        if n:
            bad_calls += 1
            bad_px += n
    print(f"RESULT side={side_kind} victim={victim} bdirect_off={os.environ.get('S3_GEMM_BDIRECT_OFF', '')!r}: "
          f"{calls} matching calls, {bad_calls} corrupted ({bad_px} px), {enc_runs} side runs",
          flush=True)


if __name__ == "__main__":
    main()
