"""ctypes binding of the C ABI in include/dips_hip.h (libdips_hip.so).

The product path always runs through this library: if the shared object is
missing or fails to load, every entry point raises ``DipsLibraryError`` --
there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading
from typing import List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libdips_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "dips_hip.h")

ABI_VERSION = 3  # DIPS_ABI_VERSION of include/dips_hip.h

DIPS_OK = 0
DIPS_ERR_INVALID = -1
DIPS_ERR_HIP = -2
DIPS_ERR_STATE = -3
DIPS_ERR_NOMEM = -4
DIPS_ERR_CAPACITY = -5
DIPS_ERR_NODEVICE = -6
DIPS_ERR_INTERNAL = -7
DIPS_ERR_COMM = -8

FLAG_DEVICE_PTRS = 0x1
FLAG_TIME_KERNEL = 0x2
FLAG_FORCE_GENERIC = 0x4
FLAG_CROSSCHECK = 0x8
FLAG_GRAY_BAND_TABLE = 0x10
FLAG_GRAY_PAIR_TABLE = 0x20

FMT_GRAY8 = 1
FMT_RGB8 = 3
FMT_RGBA8 = 4
MODE_OVERALL = 0
MODE_PER_FRAME = 1

COMM_ID_BYTES = 128
COMM_RCCL = 1
COMM_LOOPBACK = 2
COMM_HOST = 3
SHARD_REF_RESIDENT = 0x1


class DipsLibraryError(RuntimeError):
    """libdips_hip.so is missing or unusable."""


class DipsError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"dips status {status}: {message}")
        self.status = status


class DipsParams(ctypes.Structure):
    _fields_ = [
        ("colorize", ctypes.c_uint8),
        ("spatial_window_size", ctypes.c_int32),
        ("sensitivity", ctypes.c_float),
        ("filter_type", ctypes.c_uint32),
        ("chroma_filter", ctypes.c_uint32),
        ("mode", ctypes.c_uint32),
        ("format", ctypes.c_uint32),
        ("tau", ctypes.c_float),
        ("flags", ctypes.c_uint32),
    ]


class DipsAltParams(ctypes.Structure):
    _fields_ = [
        ("colorize", ctypes.c_uint8),
        ("window_size", ctypes.c_int32),
        ("sigmoid_horizontal_scalar", ctypes.c_float),
        ("filter_type", ctypes.c_uint32),
        ("chroma_filter", ctypes.c_uint32),
        ("num_textures", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
    ]


class SeriesEntry(ctypes.Structure):
    _fields_ = [
        ("sad", ctypes.c_uint64),
        ("sj", ctypes.c_uint64),
        ("count", ctypes.c_uint64),
        ("si_fixed", ctypes.c_uint64),
    ]


# dips_comm_ops: the caller's transport of DIPS_COMM_HOST (host buffers)
COMM_BROADCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)
COMM_SENDRECV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_size_t)
COMM_GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_int)


class DipsCommOps(ctypes.Structure):
    _fields_ = [
        ("broadcast", COMM_BROADCAST_FN),
        ("sendrecv", COMM_SENDRECV_FN),
        ("gather", COMM_GATHER_FN),
    ]


_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

_vp = ctypes.c_void_p
_u8p = ctypes.c_void_p  # raw pointers (host or device) are passed as integers


def header_functions() -> List[str]:
    """Names of every function declared in include/dips_hip.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dips_[a-z_0-9]+)\s*\(", text, flags=re.M)


def _share_torch_hip_runtime() -> None:
    """Make the process use ONE HIP runtime.

    torch ships its own libamdhip64 (soname libamdhip64.so.7, NEEDED by torch
    as "libamdhip64.so").  Loaded after libdips_hip.so, torch would map a
    second HIP runtime next to /opt/rocm's and fail to initialise; loaded
    first, its runtime satisfies libdips_hip.so's NEEDED entry by soname and
    device pointers / streams are shared.  So: import torch and initialise
    its HIP context before loading the library (no-op without torch/GPU)."""
    try:
        import torch  # noqa: F401
    except Exception:
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def load() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        _share_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise DipsLibraryError(
                f"{LIB_PATH} not found: build it with `make -C dips_amd/csrc` "
                "or __graft_entry__.build() (the HIP path has no fallback)")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise DipsLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        P = ctypes.POINTER
        i32, u32, u64, f32 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float
        st = ctypes.c_int
        sig = {
            "dips_abi_version": ([], st),
            "dips_params_default": ([P(DipsParams)], st),
            "dips_create": ([P(DipsParams), st, P(_vp)], st),
            "dips_destroy": ([_vp], None),
            "dips_last_error": ([_vp], ctypes.c_char_p),
            "dips_set_stream": ([_vp, _vp], st),
            "dips_synchronize": ([_vp], st),
            "dips_add_texture": ([_vp, u32, u32, _u8p, ctypes.c_size_t], st),
            "dips_dispatch": ([_vp, _u8p, ctypes.c_size_t], st),
            "dips_frame_callback": ([_vp, u32, u32, _u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t], st),
            "dips_callback_phases": ([_vp, P(ctypes.c_double), u32, P(u32)], st),
            "dips_start_texture": ([_vp, _u8p, ctypes.c_size_t], st),
            "dips_compat_resume": ([_vp, u32, u32, _u8p, _u8p, u64], st),
            "dips_frame_callback_batch": ([_vp, u32, u32, _u8p, u32, _u8p], st),
            "dips_diff_series": ([_vp, u32, u32, _u8p, u32, _u8p, _vp, _u8p], st),
            "dips_series_si": ([P(SeriesEntry)], ctypes.c_double),
            "dips_diff_series_streamed": ([_vp, u32, u32, _u8p, u32, _u8p, _vp, u32], st),
            "dips_synth_frames": ([_vp, u32, u32, u64, u64, u32, _u8p], st),
            "dips_kernel_time": ([_vp, P(ctypes.c_double), P(u64)], st),
            "dips_kernel_time_reset": ([_vp], st),
            "dips_kernel_time_each": ([_vp, P(ctypes.c_double), u64, P(u64)], st),
            "dips_read_ceiling": ([_vp, _u8p, u64, P(ctypes.c_double)], st),
            "dips_read_ceiling_walk": ([_vp, _u8p, u32, u32, u32, P(ctypes.c_double)], st),
            "dips_series_geometry": ([_vp, u32, u32, u32, P(u64), P(u64), P(u64)], st),
            "dips_comm_unique_id": ([_vp], st),
            "dips_comm_create": ([_vp, st, st, st, P(_vp)], st),
            "dips_comm_create_all": ([st, _vp, _vp], st),
            "dips_comm_create_loopback": ([st, st, _vp], st),
            "dips_comm_create_host": ([P(DipsCommOps), _vp, st, st, st, P(_vp)], st),
            "dips_comm_destroy": ([_vp], None),
            "dips_comm_last_error": ([_vp], ctypes.c_char_p),
            "dips_comm_info": ([_vp, P(st), P(st), P(st)], st),
            "dips_shard_range": ([u64, st, st, P(u64), P(u32)], st),
            "dips_shard_broadcast": ([_vp, _vp, u32, u32, _u8p, _u8p], st),
            "dips_diff_series_sharded": ([_vp, _vp, u32, u32, _u8p, u32, u64, _u8p, u32, _vp, _vp], st),
            "dips_frame_callback_batch_sharded": ([_vp, _vp, u32, u32, _u8p, u32, u64, _u8p], st),
            "dips_shard_plan": ([_vp, _vp, u32, u32, u64, P(u64), P(u32), P(u64), P(u64)], st),
            "dips_shard_reference": ([_vp, _u8p, ctypes.c_size_t], st),
            "dips_alt_params_default": ([P(DipsAltParams)], st),
            "dips_alt_create": ([P(DipsAltParams), u32, u32, st, P(_vp)], st),
            "dips_alt_destroy": ([_vp], None),
            "dips_alt_last_error": ([_vp], ctypes.c_char_p),
            "dips_alt_set_stream": ([_vp, _vp], st),
            "dips_alt_synchronize": ([_vp], st),
            "dips_alt_send_frame": ([_vp, _u8p, ctypes.c_size_t, st, _u8p, ctypes.c_size_t], st),
            "dips_alt_send_frames": ([_vp, _u8p, u32, _u8p, _u8p], st),
            "dips_alt_run": ([_vp, _u8p, u32, _vp, u32, _u8p], st),
            "dips_alt_run_sharded": ([_vp, _vp, _u8p, u32, u64, _vp, u32, _u8p], st),
            "dips_alt_snapshot_texture": ([_vp, _u8p, ctypes.c_size_t], st),
            "dips_alt_kernel_time": ([_vp, P(ctypes.c_double), P(u64)], st),
            "dips_alt_kernel_time_reset": ([_vp], st),
            "dips_alt_lut_selfcheck": ([_vp, P(u64)], st),
            "dips_alt_lut_index": ([_vp, u32, _vp, _vp, u32, P(u32), P(u32)], st),
        }
        del i32, f32
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.dips_abi_version() != ABI_VERSION:
            raise DipsLibraryError(f"{LIB_PATH} has ABI {lib.dips_abi_version()}, the bindings expect {ABI_VERSION}: "
                                   "rebuild it (`make -C dips_amd/csrc`)")
        _lib = lib
        return lib


def check(status: int, handle=None) -> int:
    if status < 0:
        lib = load()
        msg = lib.dips_last_error(handle)
        raise DipsError(status, msg.decode() if msg else "")
    return status


def check_comm(status: int, comm=None) -> int:
    """A communicator call's status (message from dips_comm_last_error)."""
    if status < 0:
        lib = load()
        msg = lib.dips_comm_last_error(comm)
        raise DipsError(status, msg.decode() if msg else "")
    return status


def check_alt(status: int, handle=None) -> int:
    if status < 0:
        lib = load()
        msg = lib.dips_alt_last_error(handle)
        raise DipsError(status, msg.decode() if msg else "")
    return status


class on_stream:
    """Bind a handle to the caller's HIP stream for one call, then back to
    the handle's own stream (``setter(ptr, NULL)``): the switch records an
    event on the stream the handle was bound to, so a handle must never stay
    bound to an external stream that may be destroyed before its next call.
    ``setter`` is dips_set_stream or dips_alt_set_stream."""

    def __init__(self, setter, ptr, check_fn, stream):
        self.setter, self.ptr, self.check_fn, self.stream = setter, ptr, check_fn, stream

    def __enter__(self):
        self.check_fn(self.setter(self.ptr, ctypes.c_void_p(int(self.stream))))
        return self

    def __exit__(self, exc_type, exc, tb):
        st = self.setter(self.ptr, None)
        if exc_type is None:
            self.check_fn(st)
        return False
