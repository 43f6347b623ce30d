"""Configuration dictionary mirroring splatt3r_slam/config.py.

`config` is a module-global dict pre-filled with the keys the hot path reads
(values of config/base.yaml:1-58).  `load_config(path)` merges a YAML file
with recursive `inherit:` support, like splatt3r_slam/config.py:7-54.
"""
from __future__ import annotations

import copy
import os

import yaml

BASE = {
    "use_calib": False,
    "single_thread": False,
    "dataset": {"subsample": 1, "img_downsample": 1, "center_principle_point": True},
    "matching": {
        "max_iter": 10,
        "lambda_init": 1e-8,
        "convergence_thresh": 1e-6,
        "dist_thresh": 1e-1,
        "radius": 3,
        "dilation_max": 5,
    },
    "tracking": {
        "min_match_frac": 0.05,
        "max_iters": 50,
        "C_conf": 0.0,
        "Q_conf": 1.5,
        "rel_error": 1e-3,
        "delta_norm": 1e-3,
        "huber": 1.345,
        "match_frac_thresh": 0.333,
        "sigma_ray": 0.003,
        "sigma_dist": 1e1,
        "sigma_pixel": 1.0,
        "sigma_depth": 1e1,
        "sigma_point": 0.05,
        "pixel_border": -10,
        "depth_eps": 1e-6,
        "filtering_mode": "weighted_pointmap",
        "filtering_score": "median",
    },
    "local_opt": {
        "pin": 1,
        "window_size": 1e6,
        "C_conf": 0.0,
        "Q_conf": 1.5,
        "min_match_frac": 0.1,
        "pixel_border": -10,
        "depth_eps": 1e-6,
        "max_iters": 10,
        "sigma_ray": 0.003,
        "sigma_dist": 1e1,
        "sigma_pixel": 1.0,
        "sigma_depth": 1e1,
        "sigma_point": 0.05,
        "delta_norm": 1e-8,
        "use_cuda": True,
    },
    "retrieval": {"k": 3, "min_thresh": 5e-3},
    "reloc": {"min_match_frac": 0.3, "strict": True},
}

config: dict = copy.deepcopy(BASE)


def _merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = v
    return dst


def _load(path: str) -> dict:
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    parent = cfg.pop("inherit", None)
    if parent:
        base = _load(parent if os.path.isabs(parent) else
                     os.path.join(os.path.dirname(path), os.path.basename(parent))
                     if not os.path.exists(parent) else parent)
        return _merge(base, cfg)
    return cfg


def load_config(path: str) -> dict:
    """Reset to base defaults, then merge `path` (with inherit: chain)."""
    config.clear()
    config.update(copy.deepcopy(BASE))
    _merge(config, _load(path))
    return config
