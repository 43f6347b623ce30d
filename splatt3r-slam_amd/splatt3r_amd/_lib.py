"""ctypes binding of libsplatt3r_hip.so (the C ABI declared in include/*.h).

The product path always goes through this library; there is no Python or
torch fallback for any kernel.  If the library is missing, `lib()` raises.
torch is imported first so that the library binds to the HIP runtime torch
already loaded (same SONAME libamdhip64.so.7): torch's streams and device
pointers are then valid inside the library.
"""
from __future__ import annotations

import ctypes
import os
import time
import threading

import torch  # noqa: F401  (must be loaded before the HIP library, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_native", "libsplatt3r_hip.so")
# S3_LIB_VARIANT=_pk: the library built with S3_PACKED_FP32=1 (packed-FP32
# instructions allowed; A/B runs only, see csrc/build.py)
if os.environ.get("S3_LIB_VARIANT"):
    LIB_PATH = LIB_PATH.replace(".so", os.environ["S3_LIB_VARIANT"] + ".so")

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float
SZ = ctypes.c_size_t

# name -> (restype, argtypes).  Kept in the order of include/*.h.
SIGNATURES: dict[str, tuple] = {
    # s3_common.h
    "s3_last_error": (ctypes.c_char_p, []),
    "s3_abi_version": (I32, []),
    "s3_arch": (ctypes.c_char_p, []),
    "s3_stream_create": (I32, [I32, I32, ctypes.POINTER(P)]),
    "s3_stream_destroy": (I32, [P]),
    # s3lie.h
    "s3lie_sim3_mul": (I32, [P, I64, P, I64, P, I64, P]),
    "s3lie_sim3_inv": (I32, [P, P, I64, P]),
    "s3lie_sim3_act": (I32, [P, I64, P, P, I64, P]),
    "s3lie_sim3_exp": (I32, [P, P, I64, P]),
    "s3lie_sim3_log": (I32, [P, P, I64, P]),
    "s3lie_sim3_retr": (I32, [P, I64, P, I64, P, I64, P]),
    "s3lie_sim3_matrix": (I32, [P, P, I64, P]),
    "s3lie_se3_matrix": (I32, [P, P, I64, P]),
    "s3lie_pose_retr": (I32, [P, P, I64, I64, P]),
    "s3lie_sim3_retr_host": (None, [P, P, P]),
    "s3lie_sim3_mul_host": (None, [P, P, P]),
    "s3lie_sim3_inv_host": (None, [P, P]),
    # s3m.h
    "s3m_iter_proj": (I32, [P, P, P, P, P, I32, I32, I32, I32, I32, F32, F32, P]),
    "s3m_refine_matches": (I32, [P, P, P, P, I32, I32, I32, I32, I32, I32, I32, P]),
    "s3m_refine_set_lanes": (None, [I32]),
    "s3m_refine_set_prefetch": (None, [I32]),
    "s3m_refine_set_sort": (None, [I32]),
    "s3m_prep_iter_proj": (I32, [P, P, P, P, P, P, I32, I32, I32, P]),
    "s3m_occlusion": (I32, [P, P, P, P, P, P, I32, I32, I32, F32, P]),
    "s3m_pixel_to_lin": (I32, [P, P, I64, I32, P]),
}

_lock = threading.Lock()
_lib = None


def register(sigs: dict) -> None:
    """Add signatures (used by modules that own a header)."""
    SIGNATURES.update(sigs)
    if _lib is not None:
        _bind(_lib, sigs)


def _bind(l, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(l, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load (once) and return the bound library; raises if it is missing."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(
                        f"splatt3r-slam_amd native library not built: {LIB_PATH} "
                        "(run __graft_entry__.build() or "
                        "python splatt3r-slam_amd/csrc/build.py)")
                l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
                _bind(l, SIGNATURES)
                _lib = l
    return _lib


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().s3_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def call(name: str, *args) -> None:
    """Call an s3_status-returning entry point and raise on failure."""
    check(getattr(lib(), name)(*args), name)


# S3_SPIN_SYNC=0: blocking stream synchronize in wait_stream (A/B)
_SPIN_SYNC = os.environ.get("S3_SPIN_SYNC", "1") != "0"


def wait_stream(device: torch.device | None = None) -> None:
    """Host wait for the work queued so far on the current stream.  Polls an
    event (yielding the GIL between polls) instead of a blocking
    synchronize: the blocking wait's wake-up latency is device idle time in
    the frame loop, since the next launches are issued only after it
    returns."""
    s = torch.cuda.current_stream(device)
    if not _SPIN_SYNC:
        s.synchronize()
        return
    ev = torch.cuda.Event()
    ev.record(s)
    wait_event(ev)


# S3_SPIN_YIELD=0: poll without yielding the CPU between polls (A/B)
_SPIN_YIELD = os.environ.get("S3_SPIN_YIELD", "1") != "0"
# Longest a host wait polls before it falls back to a blocking synchronize
# (S3_SPIN_US, microseconds): the frame loop's waits (a GN chunk, the render
# flags) end within a few hundred us, where polling saves the blocking wait's
# wake-up latency; a longer wait stops spinning, so a core and the GIL are
# not held by the poll loop while the backend worker, the loader and the PNG
# writer threads need them.
_SPIN_BUDGET_S = float(os.environ.get("S3_SPIN_US", "1000")) * 1e-6


def wait_event(ev) -> None:
    """Host wait for a recorded event (polled up to the spin budget, then a
    blocking synchronize; see wait_stream)."""
    if not _SPIN_SYNC:
        ev.synchronize()
        return
    deadline = time.perf_counter() + _SPIN_BUDGET_S
    while not ev.query():
        if time.perf_counter() > deadline:
            ev.synchronize()
            return
        if _SPIN_YIELD:
            time.sleep(0)


# The frame loop's streams.  HIP gives every new stream
# a hardware queue when it is created -- its own while fewer than
# GPU_MAX_HW_QUEUES (4 on the box) queues of that priority exist, a shared
# one after -- and a queue runs the work of the streams on it in one order.
# torch's pooled streams (torch.cuda.Stream) are created 32 at a time on
# first use and handed out round-robin, so which frame-loop stream shared a
# queue with which (the encoder's 13-ms batch replays with the aux stream or
# the default stream behind the main chain's per-step wait) depended on how
# many streams the process had taken before.  Every role therefore takes
# one stream per (device, role, priority), once, in this fixed order, when
# reserve_frame_streams() runs first (bench.py does).  The streams come from
# torch's pool by default; S3_FRAME_STREAMS=1 creates dedicated library
# streams instead (then the default stream, the encoder, the aux stream and
# the backend worker hold the 4 normal-priority queues and the main chain
# the high-priority one) -- measured slower, see below.
FRAME_STREAM_ROLES = (("encoder", 0), ("aux", 0), ("backend", 0), ("main", -1))
_FRAME_STREAMS: dict = {}
_FRAME_ORDER: list = []        # (device index, role, priority) in creation order
# guards the stream table (not _lock: creating a stream may load the library,
# which takes _lock)
_STREAM_LOCK = threading.Lock()


# S3_FRAME_STREAMS=1: dedicated library streams (s3_stream_create) instead
# of torch's pooled streams.  Measured against each other in driver-command
# benches on one box (profiles/r06y_frame_streams_ab.log): pooled 203.4 /
# 202.6 frames/s, no main-queue gap; dedicated 191.5 (one 5.5 ms gap at
# frame 16) / 197.7, and both r06x runs on the dedicated streams had a
# 6-7 ms gap at frame 16.  The pooled streams are the default.
FRAME_STREAMS_DEDICATED = os.environ.get("S3_FRAME_STREAMS", "0") == "1"


def _make_stream(dev: torch.device, priority: int):
    """A stream of torch's pool, or with S3_FRAME_STREAMS=1 a dedicated
    non-blocking HIP stream (s3_stream_create) wrapped as a torch stream."""
    if not FRAME_STREAMS_DEDICATED:
        return torch.cuda.Stream(device=dev, priority=int(priority))
    h = P()
    check(lib().s3_stream_create(int(dev.index), int(priority), ctypes.byref(h)),
          "s3_stream_create")
    return torch.cuda.ExternalStream(h.value, device=dev)


def _dev(device) -> torch.device:
    dev = torch.device(device if device is not None else "cuda")
    return dev if dev.index is not None else torch.device("cuda", torch.cuda.current_device())


def reserve_frame_streams(device=None) -> None:
    """Create the frame loop's streams of `device` (FRAME_STREAM_ROLES order)
    if they do not exist yet."""
    dev = _dev(device)
    for role, prio in FRAME_STREAM_ROLES:
        frame_stream(dev, role, prio, _reserve=False)


def frame_stream(device, role: str, priority: int = 0, _reserve: bool = True):
    """The process's dedicated stream for (device, role, priority); the
    standard set is created first (reserve_frame_streams) so its creation
    order never depends on the caller's."""
    dev = _dev(device)
    if _reserve and not any(k[0] == dev.index for k in _FRAME_STREAMS):
        reserve_frame_streams(dev)
    key = (dev.index, role, int(priority))
    s = _FRAME_STREAMS.get(key)
    if s is None:
        with _STREAM_LOCK:
            s = _FRAME_STREAMS.get(key)
            if s is None:
                s = _FRAME_STREAMS[key] = _make_stream(dev, int(priority))
                _FRAME_ORDER.append(key)
    return s


def stream(device: torch.device | None = None) -> int:
    """Raw hipStream_t of torch's current stream (as int for ctypes)."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def require_cuda(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "splatt3r-slam_amd kernels run on the GPU only; got a CPU tensor "
                f"of shape {tuple(t.shape)} (there is no CPU fallback)")


def require_contig(name: str, *tensors: torch.Tensor) -> None:
    # reference: CHECK_CONTIGUOUS in splatt3r_slam/backend/src/gn.cpp
    for t in tensors:
        if t is not None and not t.is_contiguous():
            raise RuntimeError(f"{name}: input must be contiguous")
