"""Thin Python plans over the network entry points of include/s3n.h.

Every op is built once into a ctypes argument struct (`Call`) and then run
many times; the model composes these into a `Plan` (a list of prebuilt
calls over static buffers) that is replayed per frame, optionally captured
into a HIP graph.  No op has a torch fallback.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Sequence

import torch

from splatt3r_amd import _lib

P = ctypes.c_void_p
G = 4  # S3N_MAX_GROUPS
I64 = ctypes.c_int64


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("groups", ctypes.c_int),
        ("A", P * G), ("lda", I64),
        ("B", P * G), ("ldb", I64),
        ("bias", P * G),
        ("R1", P * G), ("ldr1", I64), ("r1_f16", ctypes.c_int),
        ("R2", P * G), ("ldr2", I64), ("r2_f16", ctypes.c_int),
        ("C", P * G), ("ldc", I64), ("c_f16", ctypes.c_int),
        ("C2", P * G), ("ldc2", I64),
        ("act", ctypes.c_int), ("store_mode", ctypes.c_int), ("a_mode", ctypes.c_int),
        ("cH", ctypes.c_int), ("cW", ctypes.c_int), ("cC", ctypes.c_int), ("ksize", ctypes.c_int),
        ("stride", ctypes.c_int), ("pad", ctypes.c_int), ("oH", ctypes.c_int), ("oW", ctypes.c_int),
        ("relu_in", ctypes.c_int),
        ("sH", ctypes.c_int), ("sW", ctypes.c_int), ("sS", ctypes.c_int), ("sCout", ctypes.c_int),
        ("split_k", ctypes.c_int), ("tile", ctypes.c_int), ("workspace", P),
        ("rope_cos", P), ("rope_sin", P), ("rope_maxpos", ctypes.c_int),
        ("rope_ncols", ctypes.c_int), ("rope_pos", P * G),
        ("tail_w", P * G), ("tail_b", P * G), ("tail_out", P * G), ("tail_n", ctypes.c_int),
        ("ld_tail", I64),
        ("Bp", P * G),
    ]


class AttnArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("Nq", ctypes.c_int), ("Nk", ctypes.c_int), ("H", ctypes.c_int),
        ("groups", ctypes.c_int),
        ("Q", P * G), ("K", P * G), ("V", P * G),
        ("q_stride", I64), ("k_stride", I64), ("v_stride", I64),
        ("qpos", P * G), ("kpos", P * G),
        ("rope_cos", P), ("rope_sin", P), ("rope_maxpos", ctypes.c_int),
        ("O", P * G), ("o_stride", I64),
        ("scale", ctypes.c_float),
    ]


_GP = ctypes.POINTER(GemmArgs)
_AP = ctypes.POINTER(AttnArgs)
_PP = ctypes.POINTER(P)
_lib.register({
    "s3n_gemm": (ctypes.c_int, [_GP, P]),
    "s3n_gemm_workspace_bytes": (ctypes.c_size_t, [_GP]),
    "s3n_gemm_set_debug": (None, [ctypes.c_int]),
    "s3n_gemm_set_xcd_flags": (None, [ctypes.c_int]),
    "s3n_attention_set_variant": (None, [ctypes.c_int]),
    "s3n_attention": (ctypes.c_int, [_AP, P]),
    "s3n_layernorm": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _PP, I64, _PP, _PP,
                                     ctypes.c_float, _PP, I64, _PP, I64, P]),
    "s3n_patch_im2col": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        P, P]),
    "s3n_upsample2x": (ctypes.c_int, [ctypes.c_int, _PP, _PP, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]),
    "s3n_gaussian_postprocess": (ctypes.c_int, [I64, P, ctypes.c_int, P, P, ctypes.c_int,
                                                ctypes.c_int] + [P] * 10 + [P]),
    "s3n_prng_fill": (ctypes.c_int, [P, I64, ctypes.c_uint64, ctypes.c_float, ctypes.c_float, P]),
    "s3n_cast_f16": (ctypes.c_int, [P, I64, P, I64, I64, ctypes.c_int, P]),
    "s3n_f16_saturations": (ctypes.c_int, [ctypes.c_int]),
})


def f16_saturations(reset: bool = False) -> int:
    """How many fp16-store guards fired (GEMM epilogue, LayerNorm) since the
    last reset: > 0 means some activation exceeded the fp16 range (+-65504)
    and was saturated instead of becoming inf.  Synchronises the device."""
    torch.cuda.synchronize()
    n = _lib.lib().s3n_f16_saturations(int(bool(reset)))
    if n < 0:
        raise RuntimeError("s3n_f16_saturations: HIP error")
    return n

ACT = {"none": 0, "gelu": 1, "relu": 2}

# S3_SYNC_DEBUG=1: run plans op by op with a device sync after each (fault
# localisation); S3_GRAPHS=0 disables HIP-graph capture.
DEBUG_SYNC = os.environ.get("S3_SYNC_DEBUG", "0") == "1"
# tuning overrides for experiments: S3_GEMM_TILE=<1..8> replaces the
# library's automatic tile choice (only where a call leaves tile=0)
TILE_OVERRIDE = int(os.environ.get("S3_GEMM_TILE", "0"))
GRAPHS_ENABLED = os.environ.get("S3_GRAPHS", "1") != "0"
# S3_ATTN_VARIANT=<n>: the no-RoPE attention kernel variant (net_attn.hip
# s3n_attention_set_variant; experiments only)
ATTN_VARIANT = int(os.environ["S3_ATTN_VARIANT"]) if "S3_ATTN_VARIANT" in os.environ else None
# S3_ATTN_XCD=0: attention workgroups in plain grid order (A/B of the
# XCD-aware order; experiments only)
if os.environ.get("S3_ATTN_XCD", "1") == "0":
    _lib.lib().s3n_attention_set_variant(-1)
# S3_GEMM_XCD=1: tiles placed on the XCDs by the band split only (A/B of the
# 2-D XCD partition, net_gemm.hip; experiments only)
if os.environ.get("S3_GEMM_XCD", "0") == "1":
    _lib.lib().s3n_gemm_set_xcd_flags(1)


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _parr(items: Sequence, n=G):
    arr = (P * n)()
    for i, t in enumerate(items):
        arr[i] = _ptr(t)
    return arr


class Call:
    """A prebuilt library call: fn(*args) with status check."""
    __slots__ = ("fn", "args", "name", "keep", "kind", "flops", "desc", "nbytes")

    def __init__(self, name, *args, keep=(), kind=None, flops=0, desc="", nbytes=0):
        self.desc = desc             # shape string for per-launch profiles
        self.name = name
        self.kind = kind or name     # roofline bucket (bench.py)
        self.flops = flops           # algorithmic flops of one launch
        self.nbytes = nbytes         # algorithmic HBM bytes of one launch (operands once)
        self.fn = getattr(_lib.lib(), name)
        self.args = args
        # Everything the call points into must outlive it: the ctypes
        # arrays/structs AND the tensors behind the raw pointers (a plan
        # buffer held only by pointer is freed, and torch.cuda.graph's
        # empty_cache() then unmaps it under the captured kernels).
        self.keep = keep

    def __call__(self, stream):
        st = self.fn(*self.args, stream)
        if st != 0:
            _lib.check(st, self.name)


def auto_split_k(M, N, K, groups) -> int:
    """Split K only when the 64x64 tile grid is far too small for the chip
    (the 12x16 / 24x32 DPT levels): ~256 workgroups, >= 4 K tiles each."""
    tiles64 = groups * -(-M // 64) * -(-N // 64)
    kt = -(-K // 64)
    if tiles64 < 256 and kt >= 32:   # e.g. the encoder fc2 (768x1024x4096): 2 halves
        return 2
    if tiles64 >= 128:      # the combine launch costs more than it saves
        return 1
    return max(1, min(kt // 4, -(-256 // tiles64)))


# Per-shape launch configuration measured on the device (S3_GEMM_TUNE=0
# falls back to the static policy).  Candidates are timed on scratch
# operands of the call's exact shape, layout and epilogue (the weights and
# tables are the real ones; they are only read), so tuning never touches
# plan buffers.  The choice is cached per process and shape.  Each timed
# launch starts from flushed caches (S3_GEMM_TUNE_COLD=0: six warm
# back-to-back launches instead): inside the frame graph every GEMM reads its
# weights cold, and choosing by cold time gave 3.78 vs 3.93 ms/frame of
# gemm.dense and 144 vs 141.5 fps (profiles/r02g_tune_ab.log).
TUNE = os.environ.get("S3_GEMM_TUNE", "1") != "0"
_TUNE_CACHE: dict = {}
TUNE_LOG = os.environ.get("S3_GEMM_TUNE_LOG", "0") == "1"
TUNE_COLD = os.environ.get("S3_GEMM_TUNE_COLD", "1") == "1"
_FLUSH: dict = {}
# Tuning database: choices of an earlier process, keyed like _TUNE_CACHE and
# stamped with a digest of the tile tables below (a changed table voids the
# file).  S3_GEMM_TUNE_DB = path ("" = none; default tune_gfx950.json beside
# this module); shapes it lacks are timed as usual, so a run with the file
# makes the same launch choices -- and computes the same bits -- as the run
# that wrote it.  S3_GEMM_TUNE_DB_SAVE = path: write this process's choices
# (merged over the loaded file) there at exit.
TUNE_DB = os.environ.get("S3_GEMM_TUNE_DB",
                         os.path.join(os.path.dirname(os.path.abspath(__file__)), "tune_gfx950.json"))
TUNE_DB_SAVE = os.environ.get("S3_GEMM_TUNE_DB_SAVE", "")
# Cache and database keys start with the gfx target of the device that was
# tuned; "loaded" holds the targets whose database entries were read.
_DB_STATE = {"loaded": set(), "entries": {}}


def _kernel_abi() -> str:
    """Digest of the GEMM kernel sources (csrc/net_gemm*.hip, the kernel
    template header and common.hpp): any edit of a kernel or of a launch
    precondition changes it, and a database written under another digest
    (its "abi" field) is ignored -- no stale tile choice is replayed after a
    kernel change.  "unknown" when the sources are not beside the package."""
    import glob
    import hashlib
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "net_gemm*.hip")) +
                   glob.glob(os.path.join(csrc, "net_gemm*.hpp")) +
                   [os.path.join(csrc, "common.hpp")])
    if not all(os.path.isfile(f) for f in files) or len(files) < 3:
        return "unknown"
    h = hashlib.sha1()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


_KERNEL_ABI = _kernel_abi()


def _flush_buffer(dev):
    """512 MiB of int32, twice the MALL: touching it evicts L2 and MALL."""
    if dev not in _FLUSH:
        _FLUSH[dev] = torch.zeros(128 << 20, dtype=torch.int32, device=dev)
    return _FLUSH[dev]


_TILE_SHAPES = {1: (64, 64), 2: (64, 128), 3: (128, 128), 4: (256, 128), 5: (128, 128),
                6: (64, 64), 8: (64, 128), 9: (64, 64), 10: (64, 64), 11: (64, 128),
                12: (128, 128), 14: (256, 256),
                # in-workgroup K-groups (net_gemm.hip KG > 1)
                15: (64, 64), 16: (64, 64), 17: (64, 128), 18: (128, 128), 19: (64, 64),
                20: (64, 128),
                # v_mfma_f32_16x16x32 tiles, 4 waves (net_gemm_t4/t5.hip)
                21: (64, 160), 22: (96, 64), 23: (128, 96), 24: (160, 128), 25: (256, 128),
                26: (64, 64), 27: (128, 128), 28: (64, 128), 29: (96, 128), 30: (64, 192),
                31: (64, 64),
                # 8 / 16 waves per workgroup (net_gemm_t7.hip)
                32: (128, 128), 34: (256, 128), 35: (128, 256), 36: (256, 128), 37: (128, 128),
                # 3x3 conv with halo reuse of the input row segment (net_gemm_t6.hip)
                40: (128, 128), 41: (256, 64), 42: (128, 128), 43: (128, 128), 45: (128, 128),
                46: (128, 128), 47: (256, 64), 48: (128, 128), 49: (128, 128), 50: (256, 64),
                51: (128, 128), 52: (128, 128), 53: (256, 64),
                # k_gemm_pp: fragment reads of half a K tile overlap the MFMAs
                # of the other half (net_gemm_t8.hip)
                63: (128, 128), 65: (128, 128), 68: (256, 128),
                # B fragments straight from the packed weights into registers,
                # A through the LDS ring (net_gemm_t9.hip)
                70: (64, 128), 71: (64, 128), 72: (64, 64), 73: (64, 64), 74: (128, 128),
                75: (128, 128), 76: (128, 128), 77: (64, 128), 78: (64, 64), 79: (64, 128)}
# the B-direct tiles: dense A, a packed B (packed_b), no fused tail
_BDIRECT = set(range(70, 80))
_TAIL_OK = {1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 14, 40, 42, 43, 45, 46, 48, 49, 51, 52, 63, 65}
# S3_GEMM_MF16=0: leave the 16x16x32 tile family out of the tuner (A/B)
_EXCLUDED = set(range(21, 32)) if os.environ.get("S3_GEMM_MF16", "1") == "0" else set()



# Reduction structure of each tile (net_gemm_t*.hip launch<BM, BN, S, NWM,
# NWN, BK, KG, MF> arguments): K tile, in-workgroup K-groups, MFMA shape
# (32 = 32x32x16, 16 = 16x16x32), and whether the fp32 tile fits the LDS
# ring (vector epilogue) or takes the per-register epilogue.
_TILE_RED = {1: (64, 1, 32), 2: (64, 1, 32), 3: (64, 1, 32), 4: (64, 1, 32), 5: (64, 1, 32),
             6: (64, 1, 32), 8: (64, 1, 32), 9: (128, 1, 32), 10: (128, 1, 32),
             11: (128, 1, 32), 12: (128, 1, 32), 14: (64, 1, 32),
             15: (64, 2, 32), 16: (64, 4, 32), 17: (64, 2, 32), 18: (64, 2, 32),
             19: (128, 2, 32), 20: (64, 3, 32),
             **{t: (64, 1, 16) for t in range(21, 31)}, 31: (128, 1, 16),
             32: (64, 1, 16), 34: (64, 1, 32), 35: (64, 1, 32), 36: (64, 1, 16), 37: (64, 1, 16),
             40: (64, 1, 16), 41: (64, 1, 16), 42: (64, 1, 32), 43: (64, 1, 16),
             45: (64, 1, 32), 46: (64, 1, 16), 47: (64, 1, 16), 48: (64, 1, 32), 49: (64, 1, 16),
             50: (64, 1, 16), 51: (64, 1, 16), 52: (64, 1, 32), 53: (64, 1, 16),
             63: (64, 1, 16), 65: (64, 1, 32), 68: (64, 1, 16),
             **{t: (64, 1, 16) for t in range(70, 80)}}
_REGS_EPILOGUE = {14, 34, 35}   # the fp32 tile does not fit the LDS ring
# K tiles in (ky, channel chunk, kx) order instead of (ky, kx, channel chunk)
_HALO = set(range(40, 54)) - {44}
# S3_GEMM_HALO=0: leave the halo-reuse conv tiles out of the tuner (A/B)
if os.environ.get("S3_GEMM_HALO", "1") == "0":
    _EXCLUDED |= _HALO
# S3_GEMM_BDIRECT=0: leave the B-direct tiles out of the tuner (A/B)
if os.environ.get("S3_GEMM_BDIRECT", "1") == "0":
    _EXCLUDED |= _BDIRECT
# S3_GEMM_BDIRECT_OFF=enc,pair: no packed B (so no B-direct tile) for the
# GEMMs of the plans built in those scopes (plan_scope; diagnostic A/B)
_BD_OFF = set(filter(None, os.environ.get("S3_GEMM_BDIRECT_OFF", "").split(",")))
_SCOPE = [None]


@contextlib.contextmanager
def plan_scope(name):
    """Name the plan being built (net.py: "enc" / "pair") for S3_GEMM_BDIRECT_OFF."""
    prev, _SCOPE[0] = _SCOPE[0], name
    try:
        yield
    finally:
        _SCOPE[0] = prev


def _db_digest() -> str:
    import hashlib
    tables = (sorted(_TILE_SHAPES.items()), sorted(_TILE_RED.items()), sorted(_REGS_EPILOGUE),
              sorted(_HALO), sorted(_TAIL_OK), sorted(_BDIRECT))
    return hashlib.sha1(repr(tables).encode()).hexdigest()[:16]


def _db_decode(k):
    like = k[-1]
    return tuple(k[:-1]) + (tuple(like) if like is not None else None,)


def _device_arch(dev) -> str:
    """gfx target of `dev` without feature suffixes ("gfx950:sramecc+" -> "gfx950")."""
    try:
        return torch.cuda.get_device_properties(dev).gcnArchName.split(":")[0]
    except Exception:
        return ""


def _db_load(dev=None):
    """Fill _TUNE_CACHE from TUNE_DB once per gfx target (cold-tuned entries
    only, none whose tile this process excludes).  The file is ignored when
    its tile tables, kernel sources (abi) or gfx target differ from this
    process's / `dev`'s."""
    arch = _device_arch(dev) if dev is not None else ""
    tag = arch or "*"
    if tag in _DB_STATE["loaded"]:
        return
    _DB_STATE["loaded"].add(tag)
    if not TUNE_DB or not TUNE_COLD or not os.path.isfile(TUNE_DB):
        return
    import json
    with open(TUNE_DB) as f:
        db = json.load(f)
    db_arch = db.get("arch", "gfx950")
    why = None
    if db.get("digest") != _db_digest():
        why = "tile tables changed"
    elif str(db.get("abi", 1)) != _KERNEL_ABI:
        why = f"kernel sources {db.get('abi', 1)} != {_KERNEL_ABI}"
    elif arch and db_arch != arch:
        why = f"written for {db_arch}, device is {arch}"
    if why is not None:
        if TUNE_LOG:
            print(f"[gemm-tune] {TUNE_DB}: {why}, database ignored", flush=True)
        return
    for k, v in db["entries"]:
        key, val = (db_arch,) + _db_decode(k), (int(v[0]), int(v[1]))
        if val[0] in _EXCLUDED or (val[0] and val[0] not in _TILE_SHAPES):
            continue
        _DB_STATE["entries"][key] = val
        _TUNE_CACHE.setdefault(key, val)


def save_tune_db(path: str, arch: str = ""):
    """Write the loaded database merged with this process's choices, for the
    gfx target the choices were tuned on (`arch`; by default the only target
    this process tuned or loaded, gfx950 when there is none)."""
    import json
    merged = dict(_DB_STATE["entries"])
    merged.update(_TUNE_CACHE)
    if not arch:
        archs = sorted({k[0] for k in merged})
        if len(archs) > 1:
            raise ValueError(f"tuning choices for several targets {archs}: pass arch=")
        arch = archs[0] if archs else "gfx950"
    entries = [[list(k[1:-1]) + [list(k[-1]) if k[-1] is not None else None], list(v)]
               for k, v in merged.items() if k[0] == arch]
    entries.sort(key=repr)
    with open(path, "w") as f:
        json.dump({"digest": _db_digest(), "abi": _KERNEL_ABI, "arch": arch,
                   "entries": entries}, f)


if TUNE_DB_SAVE:
    import atexit
    atexit.register(lambda: save_tune_db(TUNE_DB_SAVE))


def reduction_class(K: int, tile: int, split_k: int):
    """What fixes the summation order of every output element of a launch:
    the MFMA shape, the K-group interleave (K-groups take every KG-th K
    tile), the split-K boundaries (k_splitk_reduce adds the planes in split
    order) and the epilogue form.  Two launches of one class compute
    bit-identical elements whatever their M or tile footprint (BM, BN only
    decide which workgroup computes an element)."""
    bk, kg, mf = _TILE_RED[tile]
    kt = -(-K // bk)
    per = -(-kt // max(1, split_k))
    bound = per * bk if -(-kt // per) > 1 else 0
    return (mf, kg, bk if kg > 1 else 0, bound, tile in _REGS_EPILOGUE, tile in _HALO)


def _tune_key(a):
    f = ("M", "N", "K", "groups", "lda", "ldb", "ldc", "act", "r1_f16", "r2_f16", "c_f16",
         "ldr1", "ldr2", "ldc2", "store_mode", "sS", "sCout", "a_mode", "cH", "cW", "cC", "ksize",
         "stride", "pad", "oH", "oW", "relu_in", "rope_ncols", "tail_n", "ld_tail")
    return tuple(getattr(a, k) for k in f) + (bool(a.R1[0]), bool(a.R2[0]), bool(a.C2[0]),
                                               bool(a.bias[0]), bool(a.C[0]), bool(a.Bp[0]))


def _tune_candidates(a, split_ok, like=None):
    kt = -(-a.K // 64)
    out = []
    for tile, (bm, bn) in _TILE_SHAPES.items():
        if tile in _EXCLUDED:
            continue
        if a.tail_n and (bn != a.N or tile not in _TAIL_OK):
            continue
        if tile in _HALO and not (a.a_mode == 1 and a.ksize == 3 and a.stride == 1 and
                                  a.oW % bm == 0 and a.cC % 64 == 0):
            continue
        if tile in _BDIRECT and not (a.Bp[0] and a.a_mode == 0 and not a.tail_n and a.K % 32 == 0):
            continue
        tiles = a.groups * -(-a.M // bm) * -(-a.N // bn)
        for sk in (1, 2, 3, 4, 6, 8):
            if sk > 1 and tile in _HALO:
                continue
            if like is not None:
                # batch-invariant plan: only launches whose elements equal
                # those of the one-item plan's choice (like = (tile, split))
                if ((tile, sk) != like and (sk > 1 and not split_ok or
                        reduction_class(a.K, tile, sk) != reduction_class(a.K, *like))):
                    continue
            elif sk > 1 and (not split_ok or kt // sk < 4 or tiles * sk > 4096):
                continue
            out.append((tile, sk))
    return out


def _tuned(a, A, B, bias, rope, rope_pos, split_ok, like=None):
    dev = next(t.device for t in (*A, *B) if isinstance(t, torch.Tensor))
    _db_load(dev)
    key = (_device_arch(dev) or "gfx950",) + _tune_key(a) + (like,)
    if key in _TUNE_CACHE:
        return _TUNE_CACHE[key]
    g = a.groups
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)

    def scratch(n, dt):
        t = torch.empty(int(n), device=dev, dtype=dt)
        if dt == torch.float16 or dt == torch.float32:
            t.normal_(0.0, 0.1, generator=gen)
        return t

    if a.a_mode == 0:
        a_elems = (a.M - 1) * a.lda + a.K
    else:
        a_elems = a.M // (a.oH * a.oW) * a.cH * a.cW * a.cC
    if a.store_mode == 0:
        c_elems = (a.M - 1) * a.ldc + a.N
    else:
        c_elems = a.M * a.sS * a.sS * a.sCout
    t = GemmArgs.from_buffer_copy(a)
    keep = []
    for i in range(g):
        sa = scratch(a_elems, torch.float16)
        keep.append(sa)
        t.A[i] = sa.data_ptr()
        if a.C[i]:
            sc = scratch(c_elems, torch.float16 if a.c_f16 else torch.float32)
            keep.append(sc)
            t.C[i] = sc.data_ptr()
        if a.tail_n:
            so = scratch((a.M - 1) * a.ld_tail + a.tail_n, torch.float32)
            keep.append(so)
            t.tail_out[i] = so.data_ptr()
        if a.R1[i]:
            r = scratch((a.M - 1) * a.ldr1 + a.N, torch.float16 if a.r1_f16 else torch.float32)
            keep.append(r)
            t.R1[i] = r.data_ptr()
        if a.R2[i]:
            r = scratch((a.M - 1) * a.ldr2 + a.N, torch.float16 if a.r2_f16 else torch.float32)
            keep.append(r)
            t.R2[i] = r.data_ptr()
        if a.C2[i]:
            r = scratch((a.M - 1) * a.ldc2 + a.N, torch.float16)
            keep.append(r)
            t.C2[i] = r.data_ptr()
        if a.rope_pos[i]:
            # (y, x) token positions: zeros are in range for any M (the
            # class_batch shape has more rows than the plan's own pos)
            r = torch.zeros(int(a.M) * 2, device=dev, dtype=torch.int64)
            keep.append(r)
            t.rope_pos[i] = r.data_ptr()
    L = _lib.lib()
    st = _lib.stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best, best_ms = (a.tile, a.split_k), None
    for tile, sk in _tune_candidates(a, split_ok, like):
        t.tile, t.split_k = tile, sk
        ws = None
        if sk > 1:
            ws = torch.empty(L.s3n_gemm_workspace_bytes(ctypes.byref(t)) // 4 + 1,
                             dtype=torch.float32, device=dev)
            t.workspace = ws.data_ptr()
        ref = ctypes.byref(t)
        if L.s3n_gemm(ref, st) != 0:
            continue
        if TUNE_COLD:
            # in the frame graph each GEMM reads its weights cold: evict L2 and
            # MALL before every timed launch and time the launches one by one
            ms = 0.0
            for _ in range(6):
                _flush_buffer(dev).add_(1)
                ev[0].record()
                L.s3n_gemm(ref, st)
                ev[1].record()
                ev[1].synchronize()
                ms += ev[0].elapsed_time(ev[1])
        else:
            torch.cuda._sleep(2_000_000)     # queue the timed launches behind a GPU sleep
            ev[0].record()
            for _ in range(6):
                L.s3n_gemm(ref, st)
            ev[1].record()
            ev[1].synchronize()
            ms = ev[0].elapsed_time(ev[1])
        if best_ms is None or ms < best_ms:
            best, best_ms = (tile, sk), ms
        del ws
    _TUNE_CACHE[key] = best
    if TUNE_LOG:
        print(f"[gemm-tune] {a.M}x{a.N}x{a.K} g{a.groups} mode{a.a_mode} st{a.store_mode} "
              f"-> tile {best[0]} split {best[1]} ({best_ms / 6 * 1e3:.1f} us; static "
              f"tile {a.tile} split {a.split_k})", flush=True)
    return best


def packed_b(B) -> torch.Tensor | None:
    """The fragment-packed copy of a weight matrix B [N, K] (fp16, rows
    contiguous) that the B-direct tiles read (s3n.h s3n_gemm_args.Bp):
    [ceil(N/16)][K/32][4][16][8], one v_mfma_f32_16x16x32_f16 B fragment per
    KiB, N padded with zero rows.  Built once per weight and kept on the
    tensor that owns the storage (a stacked group weight for its group
    views), so it lives exactly as long as the weights.  None when B is not
    such a tensor (raw pointer, other dtype / layout, K % 32 != 0).

    The copy is written on the stream current at plan-build time while the
    plan may launch on any other (the decode-ahead pair replay is built on
    one frame-loop stream and replayed on another), so the build waits for
    its stream once: the packed weights are then complete before any
    launch, whatever stream it is on.  Never built during graph capture
    (the copy would become a graph node over the graph pool): None then."""
    if not isinstance(B, torch.Tensor) or B.dtype != torch.float16 or B.dim() != 2 or not B.is_cuda:
        return None
    N, K = B.shape
    if K % 32 or B.stride() != (K, 1):
        return None
    owner = B._base if B._base is not None else B
    cache = owner.__dict__.setdefault("_s3_packed", {})
    key = (B.storage_offset(), N, K, B._version)
    P_ = cache.get(key)
    if P_ is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        Np = -(-N // 16) * 16
        Bz = B if Np == N else torch.cat([B, B.new_zeros(Np - N, K)])
        P_ = Bz.reshape(Np // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
        torch.cuda.current_stream(B.device).synchronize()
        cache[key] = P_
    return P_


def gemm(A, B, C, M, N, K, *, lda, ldb=None, ldc=None, bias=None, act="none", R1=None,
         ldr1=0, R2=None, ldr2=0, C2=None, ldc2=0, conv=None, store=None, split_k=None,
         tile=0, rope=None, rope_pos=None, rope_ncols=0, tail=None, batch=1,
         class_batch=None) -> Call:
    """Grouped GEMM: A, B, C, bias, R1, R2, C2 are lists (one entry per group)
    of tensors / raw pointers.  conv = dict(H, W, C, k, stride, pad, oH, oW,
    relu_in) switches A to implicit im2col of an NHWC image.  store =
    ("convt"|"pixshuf", sH, sW, s, Cout).  tail = (W [tail_n, N] fp16, bias fp32,
    out fp32 [M, ld], tail_n, ld) lists per group: the fused 1x1 tail (s3n.h);
    C entries may then be None.  batch = b: the M rows are b items of
    M / b rows (a pair plan's Bp pairs).  With class_batch = h (batch-
    invariant plans) the launch is tuned among the configurations of one
    reduction_class, the class of the unconstrained choice for h items (the
    batch the frame loop mostly replays), so every plan of the same one-item
    shape -- whatever its b -- computes each item's rows bit for bit alike.
    With class_batch None and b > 1 the class is the one-item shape's
    choice."""
    a = GemmArgs()
    groups = len(A)
    a.M, a.N, a.K, a.groups = int(M), int(N), int(K), groups
    a.A = _parr(A)
    a.B = _parr(B)
    a.C = _parr(C)
    a.lda = int(lda)
    a.ldb = int(ldb if ldb is not None else K)
    # packed weights for the B-direct tiles (dense A only; every group or none)
    bpk = None
    if conv is None and tail is None and a.ldb == K and _SCOPE[0] not in _BD_OFF:
        bpk = [packed_b(b) for b in B]
        if any(x is None for x in bpk):
            bpk = None
        else:
            a.Bp = _parr(bpk)
    a.ldc = int(ldc if ldc is not None else N)
    a.bias = _parr(bias or [])
    a.act = ACT[act]

    def dtype_f16(x):
        return isinstance(x, torch.Tensor) and x.dtype == torch.float16

    if R1 is not None:
        a.R1 = _parr(R1)
        a.ldr1 = int(ldr1)
        a.r1_f16 = int(dtype_f16(R1[0]))
    if R2 is not None:
        a.R2 = _parr(R2)
        a.ldr2 = int(ldr2)
        a.r2_f16 = int(dtype_f16(R2[0]))
    a.c_f16 = int(dtype_f16(C[0])) if C[0] is not None else 0
    if tail is not None:
        tw, tb, to, tn, tld = tail
        a.tail_w, a.tail_b, a.tail_out = _parr(tw), _parr(tb), _parr(to)
        a.tail_n, a.ld_tail = int(tn), int(tld)
        split_k = 1
    if C2 is not None:
        a.C2 = _parr(C2)
        a.ldc2 = int(ldc2)
    if conv is not None:
        a.a_mode = 1
        a.cH, a.cW, a.cC = conv["H"], conv["W"], conv["C"]
        a.ksize, a.stride, a.pad = conv["k"], conv["stride"], conv["pad"]
        a.oH, a.oW = conv["oH"], conv["oW"]
        a.relu_in = int(conv.get("relu_in", False))
    if store is not None:
        mode, sH, sW, s, cout = store
        a.store_mode = {"convt": 1, "pixshuf": 2}[mode]
        a.sH, a.sW, a.sS, a.sCout = sH, sW, s, cout
    if rope_pos is not None:   # fused RoPE2D epilogue on the first rope_ncols columns
        a.rope_cos, a.rope_sin = rope[0].data_ptr(), rope[1].data_ptr()
        a.rope_maxpos = rope[0].shape[0]
        a.rope_ncols = int(rope_ncols)
        a.rope_pos = _parr(rope_pos)
        split_k = 1
    # the static policy of a batch-invariant plan splits K as for its class
    # shape (class_batch items): the split is the only class-defining choice
    # of the static tile (net_gemm_t1.hip tile 0: 32x32x16, one K-group)
    M_split = M
    if M % max(1, batch) == 0 and (batch > 1 or (class_batch or 1) > 1):
        M_split = M // max(1, batch) * (class_batch or 1)
    a.split_k = int(auto_split_k(M_split, N, K, groups) if split_k is None else split_k)
    a.tile = int(tile) or TILE_OVERRIDE
    if TUNE and not tile and not TILE_OVERRIDE and torch.cuda.is_available():
        split_ok = split_k is None and rope_pos is None
        like = None
        if a.M % max(1, batch) == 0 and (batch > 1 or (class_batch or 1) > 1):
            a1 = GemmArgs.from_buffer_copy(a)
            a1.M = a.M // max(1, batch) * (class_batch or 1)
            like = _tuned(a1, A, B, bias, rope, rope_pos, split_ok)
        if like is not None and a1.M == a.M:
            a.tile, a.split_k = like
        else:
            a.tile, a.split_k = _tuned(a, A, B, bias, rope, rope_pos, split_ok, like)
            if like is not None and (reduction_class(a.K, a.tile, a.split_k)
                                     != reduction_class(a.K, *like)):
                raise RuntimeError(f"s3n_gemm {a.M}x{a.N}x{a.K}: no launch in the reduction "
                                   f"class of tile {like[0]} split {like[1]}")
    ws = None
    if a.split_k > 1:
        nbytes = _lib.lib().s3n_gemm_workspace_bytes(ctypes.byref(a))
        dev = next(t.device for t in (*A, *C) if isinstance(t, torch.Tensor))
        ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        a.workspace = ws.data_ptr()
    # algorithmic bytes: every operand read once, every output written once
    # (fp16 A / B, the residuals, bias, the outputs; split-K partials are not
    # algorithmic)
    M_, N_, K_ = int(M), int(N), int(K)
    a_elems = M_ * K_ if conv is None else M_ // (conv["oH"] * conv["oW"]) * \
        conv["H"] * conv["W"] * conv["C"]
    per = 2 * a_elems + 2 * N_ * K_
    if C[0] is not None:
        per += M_ * N_ * (2 if a.c_f16 else 4)
    if C2 is not None:
        per += 2 * M_ * N_
    for R, f16 in ((R1, a.r1_f16), (R2, a.r2_f16)):
        if R is not None:
            per += M_ * N_ * (2 if f16 else 4)
    if bias:
        per += 4 * N_
    if tail is not None:
        per += 4 * M_ * int(tail[3]) + 2 * int(tail[3]) * N_
    return Call("s3n_gemm", ctypes.byref(a), keep=(a, A, B, C, bias, R1, R2, C2, ws, rope,
                                                    rope_pos, tail, bpk),
                kind="gemm.conv" if conv is not None else "gemm.dense",
                flops=2 * int(M) * int(N) * int(K) * groups, nbytes=per * groups,
                desc=f"gemm{'.conv' if conv is not None else ''} {M}x{N}x{K} g{groups}"
                     + (f" k{conv['k']}s{conv['stride']}" if conv is not None else "")
                     + (f" {act}" if act != "none" else "") + (" R1" if R1 else "")
                     + (f" st={store[0]}" if store else "")
                     + (f" t{a.tile}" if a.tile else "") + (f" sk{a.split_k}" if a.split_k > 1 else "")
                     + (" rope" if rope_pos is not None else ""))


def attention(Q, K, V, O, *, B, Nq, Nk, H, q_stride, k_stride, v_stride, o_stride, qpos=None,
              kpos=None, rope=None, scale=0.125) -> Call:
    if ATTN_VARIANT is not None:
        _lib.lib().s3n_attention_set_variant(ATTN_VARIANT)
    a = AttnArgs()
    a.B, a.Nq, a.Nk, a.H, a.groups = B, Nq, Nk, H, len(Q)
    a.Q, a.K, a.V, a.O = _parr(Q), _parr(K), _parr(V), _parr(O)
    a.q_stride, a.k_stride, a.v_stride, a.o_stride = q_stride, k_stride, v_stride, o_stride
    if qpos is not None:
        a.qpos = _parr(qpos)
    if kpos is not None:
        a.kpos = _parr(kpos)
    if rope is not None:
        a.rope_cos, a.rope_sin = rope[0].data_ptr(), rope[1].data_ptr()
        a.rope_maxpos = rope[0].shape[0]
    a.scale = scale
    return Call("s3n_attention", ctypes.byref(a), keep=(a, Q, K, V, O, qpos, kpos, rope),
                flops=4 * B * H * Nq * Nk * 64 * len(Q),
                desc=f"attn B{B} H{H} {Nq}x{Nk} g{len(Q)}")


def layernorm(x, gamma, beta, *, rows, C, ldx, eps=1e-6, out16=None, ld16=0, out32=None,
              ld32=0) -> Call:
    xs, gs, bs = _parr(x), _parr(gamma), _parr(beta)
    o16 = _parr(out16) if out16 is not None else None
    o32 = _parr(out32) if out32 is not None else None
    return Call("s3n_layernorm", rows, C, len(x), ctypes.cast(xs, _PP), ldx,
                ctypes.cast(gs, _PP), ctypes.cast(bs, _PP), ctypes.c_float(eps),
                ctypes.cast(o16, _PP) if o16 is not None else None, ld16,
                ctypes.cast(o32, _PP) if o32 is not None else None, ld32,
                keep=(xs, gs, bs, o16, o32, x, gamma, beta, out16, out32))


def upsample2x(inp, out, *, B, H, W, C, oh=None, ow=None) -> Call:
    i, o = _parr(inp), _parr(out)
    return Call("s3n_upsample2x", len(inp), ctypes.cast(i, _PP), ctypes.cast(o, _PP), B, H, W, C,
                oh or 2 * H, ow or 2 * W, keep=(i, o, inp, out))


def patch_im2col(img, A, *, B, H, W, p) -> Call:
    return Call("s3n_patch_im2col", _ptr(img), B, H, W, p, _ptr(A), keep=(img, A))


def gaussian_postprocess(n, pts, ld_pts, feat, gauss, ld_g, use_offsets, out: dict,
                         desc16=None) -> Call:
    return Call("s3n_gaussian_postprocess", n, _ptr(pts), ld_pts, _ptr(feat), _ptr(gauss), ld_g,
                int(use_offsets), _ptr(out["pts3d"]), _ptr(out["conf"]), _ptr(out["desc"]),
                _ptr(desc16), _ptr(out["desc_conf"]), _ptr(out["scales"]),
                _ptr(out["rotations"]), _ptr(out["sh"]), _ptr(out["opacities"]),
                _ptr(out["means"]), keep=(pts, feat, gauss, out, desc16))


def prng_fill(out: torch.Tensor, seed: int, a: float, c: float) -> None:
    _lib.call("s3n_prng_fill", out.data_ptr(), out.numel(), ctypes.c_uint64(seed & (2**64 - 1)),
              ctypes.c_float(a), ctypes.c_float(c), _lib.stream(out.device))


def cast_f16(x, out, *, rows, cols, ld_in, ld_out) -> Call:
    """fp32 [rows, cols] (row stride ld_in) -> fp16 (row stride ld_out)."""
    return Call("s3n_cast_f16", _ptr(x), ld_in, _ptr(out), ld_out, rows, cols, keep=(x, out))


class Plan:
    """An ordered list of prebuilt calls over static buffers."""

    def __init__(self):
        self.calls: list[Call] = []
        self.graph = None

    def add(self, c: Call):
        self.calls.append(c)
        return c

    def extend(self, other: "Plan"):
        self.calls.extend(other.calls)

    def run(self, stream=None):
        st = stream if stream is not None else _lib.stream()
        if DEBUG_SYNC:
            for i, c in enumerate(self.calls):
                print(f"[plan] op {i}/{len(self.calls)} {getattr(c, 'name', type(c).__name__)}",
                      flush=True)
                c(st)
                torch.cuda.synchronize()
            return
        for c in self.calls:
            c(st)

    def run_timed(self, stream=None):
        """Eager run with a HIP event pair around every call on the launch
        stream; returns [(kind, flops, start_event, end_event)]."""
        st = stream if stream is not None else _lib.stream()
        ts = torch.cuda.current_stream()
        out = []
        for c in self.calls:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(ts)
            c(st)
            e1.record(ts)
            out.append((getattr(c, "kind", type(c).__name__), getattr(c, "flops", 0), e0, e1,
                        getattr(c, "desc", "")))
        return out

    def capture(self):
        """Capture the plan into a HIP graph (torch.cuda.CUDAGraph)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.run()  # warm-up outside capture (module load, lazy init)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread-local capture: a plan built lazily inside the frame loop is
        # captured while loader / PNG-writer threads wait on their own
        # events, which would invalidate a global-mode capture
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.run()
        self.graph = g
        return g

    def replay(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self.run()
