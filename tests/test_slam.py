"""Frontend (main.py:395-535 loop body) on the GPU: the side-stream encoder
pipelining must not change a single output bit."""
import pytest
import torch


@pytest.mark.gpu
def test_pipelined_frontend_matches_sequential():
    from splatt3r_amd.slam import Frontend
    from splatt3r_amd.splatt3r_utils import load_splatt3r
    from splatt3r_amd.synthetic import tum_like_sequence
    from splatt3r_amd.weights import FULL

    dev = torch.device("cuda", 0)
    model = load_splatt3r(None, device=dev, cfg=FULL, seed=1234, symmetric=True)
    n = 7
    frames = tum_like_sequence(n + 1, 384, 512, seed=3, step_px=2.0, device=dev)

    def run(pipelined):
        fe = Frontend(model, device=dev, spatial_stride=4, render=True)
        poses, renders = [], []
        for i in range(n):
            f = fe.step(i, frames[i], next_img=frames[i + 1] if pipelined else None)
            poses.append(f.T_WC.data.clone())
            renders.append(fe.last_render.clone())
        torch.cuda.synchronize()
        return poses, renders, list(fe.new_kf_frames), dict(fe.stats)

    p0, r0, kf0, st0 = run(False)
    p1, r1, kf1, st1 = run(True)
    assert st0["tracked"] == n - 1 and st0["reloc"] == 0
    assert kf0 == kf1
    assert st0 == st1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    for a, b in zip(r0, r1):
        assert torch.equal(a, b)
