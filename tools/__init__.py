"""Benchmark, profiling and diagnostic scripts (not product code).

Run from the repository root as `python -m tools.<name>`; the package puts
the repository and the product package on sys.path."""
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_REPO, os.path.join(_REPO, "splatt3r-slam_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
