import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "splatt3r-slam_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


# ------------------------------------------------- measured parity errors ---
# Tests call parity(key, err=..., tol=..., ...) for every numeric comparison;
# the values are printed in the terminal summary (so they land in the
# committed test log) and written to gpurun_out/parity_errors.json.
_PARITY: list = []


@pytest.fixture
def parity(request):
    def record(key, **vals):
        row = {"test": request.node.name, "key": key}
        row.update({k: (float(v) if not isinstance(v, str) else v) for k, v in vals.items()})
        _PARITY.append(row)
        return row
    return record


def pytest_terminal_summary(terminalreporter):
    if not _PARITY:
        return
    import json
    terminalreporter.section("parity: measured errors vs stated tolerances")
    for r in _PARITY:
        terminalreporter.write_line(json.dumps(r, sort_keys=False))
    out = os.path.join(REPO, "gpurun_out")
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_errors.json"), "w") as f:
            json.dump(_PARITY, f, indent=1)
    except OSError:
        pass


@pytest.fixture(autouse=True)
def _progress_marker(request):
    """Append the running test's name to gpurun_out/progress.log (long GPU
    tests otherwise write nothing until they finish)."""
    try:
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", "progress.log"), "a") as f:
            f.write(f"start {request.node.nodeid}\n")
    except OSError:
        pass
    yield
