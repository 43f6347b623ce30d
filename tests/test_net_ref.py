"""Pin the torch-CPU restatement (oracle/net_ref.py) against the reference
modules' golden outputs (same PRNG weights, both fp32 on CPU)."""
import os

import numpy as np
import pytest
import torch

import oracle.net_ref as R
from conftest import GOLDEN


@pytest.mark.parametrize("tag,use_offsets", [("small_off", True), ("small_nooff", False)])
def test_net_ref_matches_reference_golden(tag, use_offsets):
    import dataclasses
    from splatt3r_amd import weights as W
    g = np.load(os.path.join(GOLDEN, f"net_{tag}.npz"))
    cfg = dataclasses.replace(W.SMALL, use_offsets=use_offsets)
    sd = {n: torch.from_numpy(W.prng_tensor_numpy(1234, n, s)) for n, s in W.manifest(cfg)}
    with torch.no_grad():
        f1, p1 = R.encode(sd, cfg, torch.from_numpy(g["img1"]))
        f2, p2 = R.encode(sd, cfg, torch.from_numpy(g["img2"]))
        np.testing.assert_allclose(f1.numpy(), g["feat1"], rtol=1e-4, atol=1e-4)
        d1, d2 = R.decode(sd, cfg, f1, p1, f2, p2)
        for hk in cfg.hooks[1:]:
            np.testing.assert_allclose(d1[hk].numpy(), g[f"dec1_{hk}"], rtol=1e-4, atol=1e-4)
        r1 = R.head(sd, cfg, 1, d1, 48, 64)
        r2 = R.head(sd, cfg, 2, d2, 48, 64)
    for k in ("pts3d", "conf", "desc", "desc_conf", "scales", "rotations", "sh", "opacities", "means"):
        np.testing.assert_allclose(r1[k].numpy(), g["res1_" + k], rtol=1e-3, atol=1e-4, err_msg=k)
        np.testing.assert_allclose(r2[k].numpy(), g["res2_" + k], rtol=1e-3, atol=1e-4, err_msg=k)
