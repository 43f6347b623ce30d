"""The C-ABI library loads and exports every entry point include/*.h declares
(CPU-only: no kernel is launched)."""
import ctypes
import glob
import os
import re

from conftest import REPO

DECL = re.compile(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([a-z][a-z0-9_]*)\s*\(", re.M)


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"//.*", "", txt)
        body = txt.split('extern "C" {', 1)[-1]
        for m in DECL.finditer(body):
            name = m.group(1)
            if name.startswith(("s3", "gsr", "s3n", "s3t")):
                names.add(name)
    return names


def test_headers_declare_entry_points():
    names = declared_symbols()
    assert "s3m_iter_proj" in names and "s3lie_sim3_act" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    from splatt3r_amd import _lib
    lib = _lib.lib()
    missing = [n for n in sorted(declared_symbols()) if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"


def test_every_declared_symbol_has_a_ctypes_signature():
    from splatt3r_amd import _lib
    import importlib
    for mod in ("splatt3r_amd.net", "splatt3r_amd.tracker", "diff_gaussian_rasterization",
                "splatt3r_amd.render", "splatt3r_amd.splatt3r_utils", "mast3r_slam_backends",
                "splatt3r_amd.retrieval_database", "splatt3r_amd.gaussian_map"):
        try:
            importlib.import_module(mod)  # registers its signatures
        except ModuleNotFoundError:
            pass
    missing = [n for n in sorted(declared_symbols()) if n not in _lib.SIGNATURES]
    assert not missing, f"no ctypes signature for: {missing}"


def declared_param_counts():
    counts = {}
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"//.*", "", txt)
        body = txt.split('extern "C" {', 1)[-1]
        for m in re.finditer(r"\b([a-z][a-z0-9_]*)\s*\(([^;{]*?)\)\s*;", body, flags=re.S):
            name, params = m.group(1), m.group(2).strip()
            if not name.startswith(("s3", "gsr")):
                continue
            counts[name] = 0 if params in ("", "void") else params.count(",") + 1
    return counts


def test_ctypes_signatures_match_header_arity():
    """Every ctypes argtypes list has exactly as many entries as the C
    declaration has parameters (catches binding drift without a GPU)."""
    from splatt3r_amd import _lib
    import importlib
    for mod in ("splatt3r_amd.net", "splatt3r_amd.tracker", "diff_gaussian_rasterization",
                "splatt3r_amd.render", "splatt3r_amd.splatt3r_utils", "mast3r_slam_backends",
                "splatt3r_amd.retrieval_database", "splatt3r_amd.gaussian_map"):
        try:
            importlib.import_module(mod)
        except ModuleNotFoundError:
            pass
    counts = declared_param_counts()
    bad = {n: (len(_lib.SIGNATURES[n][1]), c) for n, c in counts.items()
           if n in _lib.SIGNATURES and len(_lib.SIGNATURES[n][1]) != c}
    assert not bad, f"argtypes arity (ctypes, header) mismatch: {bad}"


def test_abi_metadata():
    from splatt3r_amd import _lib
    lib = _lib.lib()
    assert lib.s3_abi_version() >= 1
    assert lib.s3_arch() == b"gfx950"
    assert lib.s3_last_error() == b""


def test_error_path_reports_message():
    from splatt3r_amd import _lib
    lib = _lib.lib()
    # negative count is rejected before any device work
    st = lib.s3lie_sim3_inv(None, None, -1, None)
    assert st == 1
    assert b"n < 0" in lib.s3_last_error()


def test_gemm_args_layout_matches_the_c_header():
    """ops.GemmArgs (ctypes) has the size and B-direct field offset of the C
    s3n_gemm_args (include/s3n.h), compiled here with gcc."""
    import ctypes
    import os
    import subprocess
    import tempfile
    from splatt3r_amd import ops
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "s3n.h"\n'
           'int main(void) { printf("%zu %zu %zu\\n", sizeof(s3n_gemm_args), '
           'offsetof(s3n_gemm_args, Bp), offsetof(s3n_gemm_args, ld_tail)); return 0; }\n')
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        with open(c, "w") as f:
            f.write(src)
        subprocess.run(["gcc", "-I", inc, c, "-o", exe], check=True)
        size, bp, ldt = (int(x) for x in subprocess.run([exe], capture_output=True, text=True,
                                                       check=True).stdout.split())
    assert ctypes.sizeof(ops.GemmArgs) == size
    assert ops.GemmArgs.Bp.offset == bp and ops.GemmArgs.ld_tail.offset == ldt


def test_shipped_library_has_no_packed_fp32_instructions(tmp_path):
    """Every kernel is built without v_pk_{mul,add,fma}_f32 (csrc/build.py
    NO_PACKED_FP32): on the MI355X boxes those return wrong values while
    MFMAs of another kernel run on the same CU (a GEMM on another stream
    corrupted 30-93 % of the matching kernels' launches,
    tools/stress_bd_concurrency.py).  Checked on the library that ships:
    every device bundle of its .hip_fatbin section is disassembled."""
    import shutil
    import subprocess
    import pytest
    llvm = "/opt/rocm/lib/llvm/bin"
    tools = [os.path.join(llvm, t) for t in ("llvm-objcopy", "clang-offload-bundler",
                                              "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools):
        pytest.skip("ROCm LLVM tools not found")
    lib = os.path.join(REPO, "splatt3r-slam_amd", "splatt3r_amd", "_native", "libsplatt3r_hip.so")
    fat = tmp_path / "fatbin.bin"
    subprocess.run([tools[0], f"--dump-section=.hip_fatbin={fat}", lib, str(tmp_path / "copy.so")],
                   check=True, capture_output=True)
    blob = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = [m.start() for m in re.finditer(re.escape(magic), blob)]
    assert len(offs) >= 10, offs
    packed, disassembled = 0, 0
    for k, o in enumerate(offs):
        part = tmp_path / f"b{k}.bin"
        part.write_bytes(blob[o:offs[k + 1] if k + 1 < len(offs) else len(blob)])
        co = tmp_path / f"d{k}.co"
        r = subprocess.run([tools[1], "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                            f"--output={co}"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        d = subprocess.run([tools[2], "-d", str(co)], capture_output=True, text=True).stdout
        disassembled += d.count("\n")
        packed += len(re.findall(r"\bv_pk_(?:mul|add|fma)_f32", d))
    shutil.rmtree(tmp_path, ignore_errors=True)
    assert disassembled > 100000
    assert packed == 0
