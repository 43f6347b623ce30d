"""Build libsplatt3r_hip.so (all HIP kernels + the C ABI) for gfx950, in-tree.

Plain hipcc, no cmake: every .hip file is compiled to an object with its own
flags (parity-critical files are built with -ffp-contract=off so they evaluate
the reference arithmetic strictly), then linked into one shared library at
splatt3r-slam_amd/splatt3r_amd/_native/libsplatt3r_hip.so.  Incremental:
an object is rebuilt only when its source or any header is newer.

Usage: python splatt3r-slam_amd/csrc/build.py [-j N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
INCLUDE = os.path.join(REPO, "include")
OBJ_DIR = os.path.join(PKG, "build", "obj")
OUT_DIR = os.path.join(PKG, "splatt3r_amd", "_native")
LIB_NAME = "libsplatt3r_hip.so"
ARCH = os.environ.get("S3_OFFLOAD_ARCH", "gfx950")

STRICT = ["-ffp-contract=off"]
FAST = ["-ffp-contract=fast"]
# No packed-FP32 VALU instructions (v_pk_{mul,add,fma}_f32) in any kernel.
# On the MI355X boxes they return wrong values while MFMA instructions of
# another kernel run on the same CU: a concurrent GEMM on another stream --
# ours or hipBLASLt's -- corrupted 30-93 % of the matching kernels' launches
# (tools/stress_bd_concurrency.py, profiles/r06_packed_fp32_mfma.log); built
# without them, 0 of ~160k.  The results are the same IEEE values (each
# packed op is two scalar ops; contraction is set per file above).
# S3_PACKED_FP32=1 builds the packed variant beside it (_pk suffix, A/B only).
NO_PACKED_FP32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
_VARIANT = "_pk" if os.environ.get("S3_PACKED_FP32", "0") == "1" else ""
OBJ_DIR += _VARIANT
LIB_NAME = LIB_NAME.replace(".so", _VARIANT + ".so")


def device_flags(src: str) -> list[str]:
    """Every compile flag of `src` beyond the common ones (tests use it)."""
    return SOURCES[src] + ([] if _VARIANT else NO_PACKED_FP32)

# source file -> extra flags
SOURCES = {
    "common.hip": [],
    "sim3.hip": STRICT,
    "matching.hip": STRICT,
    "tracker.hip": STRICT,
    "raster.hip": STRICT,
    "splat_pack.hip": STRICT,
    "gaussians.hip": STRICT,
    "net_gemm.hip": FAST,
    "net_gemm_t1.hip": FAST,
    "net_gemm_t2.hip": FAST,
    "net_gemm_t3.hip": FAST,
    "net_gemm_t4.hip": FAST,
    "net_gemm_t5.hip": FAST,
    "net_gemm_t6.hip": FAST,
    "net_gemm_t7.hip": FAST,
    "net_gemm_t8.hip": FAST,
    "net_gemm_t9.hip": FAST,
    "net_attn.hip": FAST,
    "net_ops.hip": STRICT,
    "gn_backend.hip": STRICT,
    "retrieval.hip": STRICT,
}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _headers_mtime() -> float:
    m = 0.0
    for d in (INCLUDE, HERE):
        for f in os.listdir(d):
            if f.endswith((".h", ".hpp", ".inc")):
                m = max(m, os.path.getmtime(os.path.join(d, f)))
    return m


def _compile(src: str, flags: list[str], force: bool, hdr_mtime: float) -> str:
    path = os.path.join(HERE, src)
    obj = os.path.join(OBJ_DIR, src.replace(".hip", ".o"))
    cmd = [hipcc(), "-c", path, "-o", obj, "-fPIC", "-O3", "-std=c++17",
           f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", HERE,
           "-Wno-unused-result", "-munsafe-fp-atomics"] + flags + ([] if _VARIANT else NO_PACKED_FP32)
    # the command is stamped beside the object: a flag change rebuilds it
    stamp = obj + ".cmd"
    same_cmd = os.path.exists(stamp) and open(stamp).read() == " ".join(cmd[1:])
    if (not force and same_cmd and os.path.exists(obj)
            and os.path.getmtime(obj) >= max(os.path.getmtime(path), hdr_mtime)):
        return obj
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(" ".join(cmd[1:]))
    return obj


def build(jobs: int | None = None, force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = {s: f for s, f in SOURCES.items() if os.path.exists(os.path.join(HERE, s))}
    hdr = _headers_mtime()
    jobs = jobs or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda kv: _compile(kv[0], kv[1], force, hdr), srcs.items()))
    out = os.path.join(OUT_DIR, LIB_NAME)
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(out) or os.path.getmtime(out) < newest:
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[build] {out} ({len(objs)} objects, arch {ARCH})")
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    try:
        build(a.j, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
