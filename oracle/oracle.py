"""ctypes wrapper for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module.  It loads ``oracle/libdips_oracle.so`` (built by
``oracle/Makefile``), a plain-C restatement of the DiPs reference semantics
(see dips_oracle.h for the citations and the parity status: pinned to the
reference's shader text by executing it, oracle/wgsl_exec.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB: Optional[ctypes.CDLL] = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_f64p = ctypes.POINTER(ctypes.c_double)


def build(native: bool = False) -> str:
    """Build the oracle library with make; returns its path."""
    target = "native" if native else "all"
    subprocess.run(["make", "-s", "-C", _HERE, target], check=True)
    return os.path.join(_HERE, "libdips_oracle_native.so" if native else "libdips_oracle.so")


def load(path: Optional[str] = None) -> ctypes.CDLL:
    global _LIB
    if path is None and _LIB is not None:
        return _LIB
    if path is None:
        path = os.path.join(_HERE, "libdips_oracle.so")
        if not os.path.exists(path):
            build()
    lib = ctypes.CDLL(path)
    lib.dips_oracle_u.argtypes = [ctypes.c_uint8]
    lib.dips_oracle_u.restype = ctypes.c_float
    lib.dips_oracle_q.argtypes = [ctypes.c_float]
    lib.dips_oracle_q.restype = ctypes.c_uint8
    lib.dips_oracle_expf.argtypes = [ctypes.c_float]
    lib.dips_oracle_expf.restype = ctypes.c_float
    lib.dips_oracle_logf.argtypes = [ctypes.c_float]
    lib.dips_oracle_logf.restype = ctypes.c_float
    lib.dips_oracle_upper_median4.argtypes = [ctypes.POINTER(ctypes.c_float)]
    lib.dips_oracle_upper_median4.restype = ctypes.c_float
    sargs = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
             ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p,
             _u64p, _f64p, _u8p]
    lib.dips_oracle_series.argtypes = sargs
    lib.dips_oracle_series.restype = ctypes.c_int
    lib.dips_oracle_series_mt.argtypes = sargs + [ctypes.c_int]
    lib.dips_oracle_series_mt.restype = ctypes.c_int
    lib.dips_oracle_synth.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _u8p]
    lib.dips_oracle_synth.restype = None
    lib.dips_oracle_cs_new.argtypes = [ctypes.c_uint8, ctypes.c_int32, ctypes.c_float,
                                       ctypes.c_uint32, ctypes.c_uint32]
    lib.dips_oracle_cs_new.restype = ctypes.c_void_p
    lib.dips_oracle_cs_add_texture.argtypes = [ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_uint32, _u8p]
    lib.dips_oracle_cs_add_texture.restype = ctypes.c_int
    lib.dips_oracle_cs_resume.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint64]
    lib.dips_oracle_cs_resume.restype = ctypes.c_int
    lib.dips_oracle_cs_dispatch.argtypes = [ctypes.c_void_p, _u8p]
    lib.dips_oracle_cs_dispatch.restype = ctypes.c_int
    lib.dips_oracle_cs_start_texture.argtypes = [ctypes.c_void_p, _u8p]
    lib.dips_oracle_cs_start_texture.restype = ctypes.c_int
    lib.dips_oracle_cs_free.argtypes = [ctypes.c_void_p]
    lib.dips_oracle_cs_free.restype = None
    lib.dips_oracle_alt_new.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint8, ctypes.c_int32, ctypes.c_float,
                                        ctypes.c_uint32, ctypes.c_uint32]
    lib.dips_oracle_alt_new.restype = ctypes.c_void_p
    lib.dips_oracle_alt_temporal.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_uint32]
    lib.dips_oracle_alt_temporal.restype = ctypes.c_float
    lib.dips_oracle_alt_send_frame.argtypes = [ctypes.c_void_p, _u8p, ctypes.c_int, _u8p]
    lib.dips_oracle_alt_send_frame.restype = ctypes.c_int
    lib.dips_oracle_alt_run.argtypes = [ctypes.c_void_p, _u8p, ctypes.c_uint32, _u64p,
                                        ctypes.c_uint32, _u8p]
    lib.dips_oracle_alt_run.restype = ctypes.c_int
    lib.dips_oracle_alt_free.argtypes = [ctypes.c_void_p]
    lib.dips_oracle_alt_free.restype = None
    if path == os.path.join(_HERE, "libdips_oracle.so"):
        _LIB = lib
    return lib


def _p(a: Optional[np.ndarray], t=_u8p):
    if a is None:
        return ctypes.cast(None, t)
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


def series(frames: np.ndarray, *, mode: int = 0, chroma: int = 0, tau: float = 0.0,
           ref: Optional[np.ndarray] = None, want_map: bool = False,
           nthreads: int = 1, lib: Optional[ctypes.CDLL] = None):
    """frames: uint8 [N, H, W] (gray) or [N, H, W, C].  Returns
    (out4 uint64 [N,4] = SAD, SJ, count, SI_fixed; si_f64 [N]; dmap or None)."""
    lib = lib or load()
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    n = frames.shape[0]
    h, w = frames.shape[1], frames.shape[2]
    c = 1 if frames.ndim == 3 else frames.shape[3]
    out4 = np.zeros((n, 4), dtype=np.uint64)
    si = np.zeros(n, dtype=np.float64)
    dmap = np.zeros_like(frames) if want_map else None
    if ref is not None:
        ref = np.ascontiguousarray(ref, dtype=np.uint8)
        assert ref.size == h * w * c
    args = (c, chroma, mode, ctypes.c_float(tau), w, h, _p(frames), n, _p(ref),
            _p(out4, _u64p), _p(si, _f64p), _p(dmap))
    if nthreads > 1:
        rc = lib.dips_oracle_series_mt(*args, nthreads)
    else:
        rc = lib.dips_oracle_series(*args)
    if rc != 0:
        raise ValueError(f"dips_oracle_series rc={rc}")
    return out4, si, dmap


def synth(channels: int, width: int, height: int, seed: int, t0: int, n: int,
          lib: Optional[ctypes.CDLL] = None) -> np.ndarray:
    lib = lib or load()
    shape = (n, height, width) if channels == 1 else (n, height, width, channels)
    out = np.zeros(shape, dtype=np.uint8)
    lib.dips_oracle_synth(channels, width, height, seed, t0, n, _p(out))
    return out


class ComputeState:
    """Oracle twin of dips/src/gpu/mod.rs ComputeState (new/add_texture/dispatch)."""

    def __init__(self, colorize: bool, spatial_window_size: int, sensitivity: float,
                 filter_type: int, chroma_filter: int):
        self._lib = load()
        self._h = self._lib.dips_oracle_cs_new(1 if colorize else 0, spatial_window_size,
                                               ctypes.c_float(sensitivity), filter_type,
                                               chroma_filter)
        if not self._h:
            raise ValueError("invalid ComputeState parameters")
        self._w = self._hgt = 0

    def add_texture(self, width: int, height: int, frame: np.ndarray) -> None:
        frame = np.ascontiguousarray(frame, dtype=np.uint8)
        assert frame.size == width * height * 4
        rc = self._lib.dips_oracle_cs_add_texture(self._h, width, height, _p(frame))
        if rc != 0:
            raise ValueError(f"add_texture rc={rc}")
        self._w, self._hgt = width, height

    def dispatch(self) -> Optional[np.ndarray]:
        out = np.zeros((self._hgt, self._w, 4), dtype=np.uint8)
        rc = self._lib.dips_oracle_cs_dispatch(self._h, _p(out))
        return out if rc == 1 else None

    def start_texture(self) -> Optional[np.ndarray]:
        out = np.zeros((self._hgt, self._w, 4), dtype=np.uint8)
        rc = self._lib.dips_oracle_cs_start_texture(self._h, _p(out))
        return out if rc == 1 else None

    def resume(self, width: int, height: int, start: np.ndarray, halo: np.ndarray, t0: int) -> None:
        """State after frame_callback of frames 0..t0-1 (t0 >= 7) from the
        start texture and the raw frames t0-3..t0-1 (halo [3, H, W, 4])."""
        start = np.ascontiguousarray(start, dtype=np.uint8)
        halo = np.ascontiguousarray(halo, dtype=np.uint8)
        assert start.size == width * height * 4 and halo.size == 3 * width * height * 4
        rc = self._lib.dips_oracle_cs_resume(self._h, width, height, _p(start), _p(halo), int(t0))
        if rc != 0:
            raise ValueError(f"resume rc={rc}")
        self._w, self._hgt = width, height

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.dips_oracle_cs_free(h)
            self._h = None


def frame_callback(width: int, height: int, frame: np.ndarray, compute: ComputeState) -> np.ndarray:
    """dips/src/lib.rs:233-246: add_texture, then dispatch or pass the input through."""
    compute.add_texture(width, height, frame)
    out = compute.dispatch()
    return out if out is not None else np.array(frame, dtype=np.uint8, copy=True).reshape(height, width, 4)


class AltCompute:
    """Oracle twin of dips_alt's DiPsCompute (dips_alt/src/dips_compute/mod.rs:243-647).
    width = frame columns, height = rows (natural order; the reference's
    constructor takes (rows, cols), lib.rs:596-603)."""

    def __init__(self, num_textures: int, width: int, height: int, colorize: bool = True,
                 window: int = 1, scalar: float = 5.0, filter_type: int = 0, chroma: int = 0):
        self._lib = load()
        self._h = self._lib.dips_oracle_alt_new(num_textures, width, height, 1 if colorize else 0,
                                                window, ctypes.c_float(scalar), filter_type, chroma)
        if not self._h:
            raise ValueError("invalid DiPsCompute parameters")
        self.width, self.height = width, height

    def send_frame(self, frame: np.ndarray, snapshot: bool = False) -> np.ndarray:
        frame = np.ascontiguousarray(frame, dtype=np.uint8)
        assert frame.size == self.width * self.height * 4
        out = np.zeros((self.height, self.width, 4), dtype=np.uint8)
        rc = self._lib.dips_oracle_alt_send_frame(self._h, _p(frame), 1 if snapshot else 0, _p(out))
        if rc != 0:
            raise ValueError(f"send_frame rc={rc}")
        return out

    def run(self, frames: np.ndarray, markers=()) -> np.ndarray:
        """run_dips_on_file's frame loop (dips_alt/src/lib.rs:588-683)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        n = frames.shape[0]
        out = np.zeros_like(frames)
        mk = np.ascontiguousarray(np.asarray(list(markers), dtype=np.uint64))
        rc = self._lib.dips_oracle_alt_run(self._h, _p(frames), n, _p(mk, _u64p), mk.size, _p(out))
        if rc != 0:
            raise ValueError(f"alt run rc={rc}")
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.dips_oracle_alt_free(h)
            self._h = None


def alt_temporal(values, lib: Optional[ctypes.CDLL] = None) -> float:
    lib = lib or load()
    v = np.ascontiguousarray(np.asarray(values, dtype=np.float32))
    return float(lib.dips_oracle_alt_temporal(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), v.size))
