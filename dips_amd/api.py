"""Host-side mirror of the reference operator surface, over the C ABI.

Reference surface (RubenMovsesyan/DiPs, crate ``dips``):
  DiPsFilter / ChromaFilter        dips/src/lib.rs:25-61
  DiPsProperties (builder)         dips/src/lib.rs:63-170
  ComputeState::new/add_texture/dispatch   dips/src/gpu/mod.rs:59, :170, :306
  frame_callback                   dips/src/lib.rs:233-246
plus the north-star batch path (per-frame difference series), which has no
reference counterpart beyond the per-pixel math of dips_shader.wgsl:64-82.
Every call goes to libdips_hip.so; there is no Python compute path.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass
from typing import Callable, Iterable, Iterator, List, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import DipsError, DipsParams, check


class DiPsFilter(enum.IntEnum):
    """dips/src/lib.rs:25-41; the value is the WGSL override id 3 code."""
    Unfiltered = 255
    Sigmoid = 0
    InverseSigmoid = 1


class ChromaFilter(enum.IntEnum):
    """dips/src/lib.rs:43-61; the value is the WGSL override id 4 code."""
    None_ = 0
    Red = 1
    Green = 2
    Blue = 3


class PixelFormat(enum.IntEnum):
    Gray8 = _lib.FMT_GRAY8
    RGB8 = _lib.FMT_RGB8
    RGBA8 = _lib.FMT_RGBA8


class Mode(enum.IntEnum):
    Overall = _lib.MODE_OVERALL     # against frame 0 (README.md:7)
    PerFrame = _lib.MODE_PER_FRAME  # against the previous frame (README.md:8-10)


class VideoPathNotSpecifiedError(Exception):
    """dips/src/lib.rs:173-186"""


class FrameCallbackNotSpecifiedError(Exception):
    """dips/src/lib.rs:188-201"""


class DiPsProperties:
    """Builder mirroring dips/src/lib.rs:63-170 (defaults :74-86)."""

    def __init__(self) -> None:
        self._video_path: Optional[str] = None
        self._frame_callback: Optional[Callable] = None
        self._output_path: Optional[str] = None
        self.colorize_: bool = False
        self.spatial_window_size_: int = 1
        self.sensitivity_: float = 5.0
        self.filter_type_: DiPsFilter = DiPsFilter.Unfiltered
        self.chroma_filter_: ChromaFilter = ChromaFilter.None_

    @classmethod
    def new(cls) -> "DiPsProperties":
        return cls()

    def video_path(self, p: str) -> "DiPsProperties":
        self._video_path = str(p)
        return self

    def frame_callback(self, cb: Callable) -> "DiPsProperties":
        self._frame_callback = cb
        return self

    def output_path(self, p: str) -> "DiPsProperties":
        self._output_path = str(p)
        return self

    def colorize(self, v: bool) -> "DiPsProperties":
        self.colorize_ = bool(v)
        return self

    def spatial_window_size(self, v: int) -> "DiPsProperties":
        self.spatial_window_size_ = int(v)
        return self

    def sensitivity(self, v: float) -> "DiPsProperties":
        self.sensitivity_ = float(v)
        return self

    def filter_type(self, v: DiPsFilter) -> "DiPsProperties":
        self.filter_type_ = DiPsFilter(v)
        return self

    def chroma_filter(self, v: ChromaFilter) -> "DiPsProperties":
        self.chroma_filter_ = ChromaFilter(v)
        return self

    def get_video_path(self) -> Optional[str]:
        return self._video_path

    def get_output_path(self) -> Optional[str]:
        return self._output_path

    def get_frame_callback(self) -> Optional[Callable]:
        return self._frame_callback

    def build(self) -> "DiPsProperties":
        out = DiPsProperties()
        out.__dict__.update(self.__dict__)
        return out


def _params(colorize=False, spatial_window_size=1, sensitivity=5.0,
            filter_type=DiPsFilter.Unfiltered, chroma_filter=ChromaFilter.None_,
            mode=Mode.Overall, fmt=PixelFormat.RGB8, tau=0.0, flags=0) -> DipsParams:
    p = DipsParams()
    check(_lib.load().dips_params_default(ctypes.byref(p)))
    p.colorize = 1 if colorize else 0
    p.spatial_window_size = int(spatial_window_size)
    p.sensitivity = float(sensitivity)
    p.filter_type = int(filter_type)
    p.chroma_filter = int(chroma_filter)
    p.mode = int(mode)
    p.format = int(fmt)
    p.tau = float(tau)
    p.flags = int(flags)
    return p


class _Handle:
    def __init__(self, params: DipsParams, device: int = 0):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        st = self._lib.dips_create(ctypes.byref(params), int(device), ctypes.byref(h))
        check(st, None)
        self._h = h
        self.params = params
        self.device = device

    @property
    def ptr(self) -> ctypes.c_void_p:
        if self._h is None:
            raise DipsError(_lib.DIPS_ERR_STATE, "handle destroyed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            self._lib.dips_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, st: int) -> int:
        return check(st, self._h)


def _stream_of(hd: "_Handle", tensor, stream=None) -> "_lib.on_stream":
    """`hd` bound to `stream` (default: the tensor's current stream) for one
    call, then back to its own stream (see _lib.on_stream)."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(tensor.device).cuda_stream
    return _lib.on_stream(hd._lib.dips_set_stream, hd.ptr, hd.check, stream)


def _as_u8(frame) -> np.ndarray:
    a = np.ascontiguousarray(frame)
    if a.dtype != np.uint8:
        a = a.astype(np.uint8)
    return a


class ComputeState:
    """Drop-in for dips/src/gpu/mod.rs ComputeState on a HIP device."""

    def __init__(self, colorize: bool, spatial_window_size: int, sensitivity: float,
                 filter_type: DiPsFilter, chroma_filter: ChromaFilter, device: int = 0,
                 time_kernel: bool = False, crosscheck: bool = False):
        """crosscheck: the plain kernels and transfers (DIPS_FLAG_CROSSCHECK):
        same outputs, for tests."""
        flags = (_lib.FLAG_TIME_KERNEL if time_kernel else 0) | (_lib.FLAG_CROSSCHECK if crosscheck else 0)
        self._hd = _Handle(_params(colorize, spatial_window_size, sensitivity, filter_type,
                                   chroma_filter, fmt=PixelFormat.RGBA8, flags=flags), device)
        self._dev: Optional[_Handle] = None
        self._w = 0
        self._h = 0

    @classmethod
    def new(cls, colorize, spatial_window_size, sensitivity, filter_type, chroma_filter,
            device: int = 0) -> "ComputeState":
        return cls(colorize, spatial_window_size, sensitivity, filter_type, chroma_filter, device)

    def add_texture(self, width: int, height: int, frame_data) -> None:
        a = _as_u8(frame_data)
        self._hd.check(self._hd._lib.dips_add_texture(self._hd.ptr, width, height,
                                                      a.ctypes.data, a.nbytes))
        self._w, self._h = width, height

    def dispatch(self) -> Optional[np.ndarray]:
        """gpu/mod.rs:306-397: None only while the ring warms up (frames
        0..2); a device or argument error raises DipsError (the reference's
        wgpu path panics), so None never hides a failure."""
        out = np.empty((self._h, self._w, 4), dtype=np.uint8)
        r = self._hd.check(self._hd._lib.dips_dispatch(self._hd.ptr, out.ctypes.data, out.nbytes))
        return out if r == 1 else None

    def frame_callback_batch(self, width: int, height: int, frames) -> np.ndarray:
        """len(frames) consecutive frame_callback calls (dips/src/lib.rs:233-246)
        in one pass over HBM (dips_frame_callback_batch); frames [N, H, W, 4]."""
        a = _as_u8(frames)
        if a.size % (width * height * 4) != 0:
            raise ValueError("frames must be [N, height, width, 4] RGBA8")
        n = a.size // (width * height * 4)
        out = np.empty((n, height, width, 4), dtype=np.uint8)
        self._hd.check(self._hd._lib.dips_frame_callback_batch(self._hd.ptr, width, height, a.ctypes.data, n,
                                                               out.ctypes.data))
        self._w, self._h = width, height
        return out

    def frame_callback_batch_device(self, frames, out, stream=None) -> None:
        """Device form: uint8 HIP tensors [N, H, W, 4], asynchronous on the
        tensor's current stream.  Keeps its own ComputeState, separate from
        the host-pointer calls of this object."""
        n, h, w = int(frames.shape[0]), int(frames.shape[1]), int(frames.shape[2])
        if tuple(frames.shape) != (n, h, w, 4) or tuple(out.shape) != tuple(frames.shape):
            raise ValueError("frames/out must be [N, H, W, 4] uint8 tensors")
        for t in (frames, out):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("device path needs contiguous HIP tensors")
        dv = self._device_handle()
        with _stream_of(dv, frames, stream):
            dv.check(dv._lib.dips_frame_callback_batch(dv.ptr, w, h, frames.data_ptr(), n, out.data_ptr()))

    def _device_handle(self) -> "_Handle":
        """The device-pointer twin handle (own ComputeState)."""
        if self._dev is None:
            p = DipsParams()
            ctypes.memmove(ctypes.byref(p), ctypes.byref(self._hd.params), ctypes.sizeof(p))
            p.flags |= _lib.FLAG_DEVICE_PTRS
            self._dev = _Handle(p, self._hd.device)
        return self._dev

    # -- frame-range sharding (3-frame halo + start texture) --
    def frame_callback_batch_sharded(self, comm, width: int, height: int, frames, n_total: int) -> np.ndarray:
        """dips_frame_callback_batch_sharded on host arrays: this rank's
        frames [n_local, H, W, 4] (its shard_range of n_total) through a
        fresh ComputeState, the outputs one ComputeState over all frames
        gives them; the library exchanges the 3-frame halo and broadcasts the
        start texture."""
        a = _as_u8(frames)
        if a.size % (width * height * 4) != 0:
            raise ValueError("frames must be [N, height, width, 4] RGBA8")
        n = a.size // (width * height * 4)
        out = np.empty((n, height, width, 4), dtype=np.uint8)
        self._hd.check(self._hd._lib.dips_frame_callback_batch_sharded(
            self._hd.ptr, comm.ptr, width, height, a.ctypes.data, n, int(n_total), out.ctypes.data))
        self._w, self._h = width, height
        return out

    def frame_callback_batch_sharded_device(self, comm, frames, out, n_total: int, stream=None) -> None:
        """The same on uint8 HIP tensors [n_local, H, W, 4] (the device
        handle, asynchronous on the tensor's current stream)."""
        n, h, w = int(frames.shape[0]), int(frames.shape[1]), int(frames.shape[2])
        if tuple(frames.shape) != (n, h, w, 4) or tuple(out.shape) != tuple(frames.shape):
            raise ValueError("frames/out must be [N, H, W, 4] uint8 tensors")
        for t in (frames, out):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("device path needs contiguous HIP tensors")
        dv = self._device_handle()
        with _stream_of(dv, frames, stream):
            dv.check(dv._lib.dips_frame_callback_batch_sharded(dv.ptr, comm.ptr, w, h, frames.data_ptr(), n,
                                                               int(n_total), out.data_ptr()))

    def resume(self, width: int, height: int, start, halo, t0: int) -> None:
        """Continue as if frame_callback had seen global frames 0..t0-1
        (t0 >= 7, any window): `start` is the start texture of the handle that
        saw frames 0..3, `halo` the raw RGBA8 frames t0-3..t0-1 ([3, H, W, 4])."""
        s, hl = _as_u8(start), _as_u8(halo)
        if s.size != width * height * 4 or hl.size != 3 * width * height * 4:
            raise ValueError("start must be [H, W, 4] and halo [3, H, W, 4] RGBA8")
        self._hd.check(self._hd._lib.dips_compat_resume(self._hd.ptr, width, height, s.ctypes.data,
                                                        hl.ctypes.data, int(t0)))
        self._w, self._h = width, height

    def resume_device(self, start, halo, t0: int, stream=None) -> None:
        """Device form of resume (uint8 HIP tensors), for the device handle
        that frame_callback_batch_device drives."""
        h, w = int(start.shape[0]), int(start.shape[1])
        if tuple(start.shape) != (h, w, 4) or tuple(halo.shape) != (3, h, w, 4):
            raise ValueError("start must be [H, W, 4] and halo [3, H, W, 4] uint8 tensors")
        for t in (start, halo):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("device path needs contiguous HIP tensors")
        dv = self._device_handle()
        with _stream_of(dv, start, stream):
            dv.check(dv._lib.dips_compat_resume(dv.ptr, w, h, start.data_ptr(), halo.data_ptr(), int(t0)))

    def start_texture_device(self, out, stream=None) -> bool:
        """The device handle's start texture into a uint8 HIP tensor [H, W, 4]
        (asynchronous); False while it is not built yet."""
        dv = self._device_handle()
        with _stream_of(dv, out, stream):
            return dv.check(dv._lib.dips_start_texture(dv.ptr, out.data_ptr(), out.numel())) == 1

    def kernel_time(self, reset: bool = False) -> Tuple[float, int]:
        """hipEvent time of the batch kernel on the device handle (time_kernel=True)."""
        ms, cnt = ctypes.c_double(), ctypes.c_uint64()
        hd = self._dev
        if hd is None:
            return 0.0, 0
        hd.check(hd._lib.dips_kernel_time(hd.ptr, ctypes.byref(ms), ctypes.byref(cnt)))
        if reset:
            hd.check(hd._lib.dips_kernel_time_reset(hd.ptr))
        return ms.value, cnt.value

    CALLBACK_PHASES = ("sync_us", "staged_us", "launched_us", "kernels_us", "wall_us", "pack_cpu_us",
                       "expand_cpu_us", "wait_cpu_us", "threads", "stripes", "expand_start_us")

    def callback_phases(self) -> Optional[dict]:
        """Where the last zero-copy frame_callback spent its time
        (dips_callback_phases; None before the first such call)."""
        v = (ctypes.c_double * len(self.CALLBACK_PHASES))()
        n = ctypes.c_uint32()
        st = self._hd._lib.dips_callback_phases(self._hd.ptr, v, len(v), ctypes.byref(n))
        if st == _lib.DIPS_ERR_STATE:
            return None
        self._hd.check(st)
        return dict(zip(self.CALLBACK_PHASES, list(v)[: n.value]))

    def start_texture(self) -> Optional[np.ndarray]:
        out = np.empty((self._h, self._w, 4), dtype=np.uint8)
        r = self._hd.check(self._hd._lib.dips_start_texture(self._hd.ptr, out.ctypes.data, out.nbytes))
        return out if r == 1 else None

    def close(self) -> None:
        self._hd.close()
        if self._dev is not None:
            self._dev.close()


def frame_callback(width: int, height: int, frame_data, compute: ComputeState) -> np.ndarray:
    """dips/src/lib.rs:233-246 through the C ABI's dips_frame_callback: the
    visualisation, or the input passed through while the ring warms up; an
    error raises DipsError instead of passing the input through."""
    a = _as_u8(frame_data)
    out = np.empty((height, width, 4), dtype=np.uint8)
    compute._hd.check(compute._hd._lib.dips_frame_callback(
        compute._hd.ptr, width, height, a.ctypes.data, a.nbytes, out.ctypes.data, out.nbytes))
    compute._w, compute._h = width, height
    return out


def perform_dips_frames(properties: DiPsProperties, frames: Iterable, width: int, height: int,
                        device: int = 0, batch: int = 0) -> Iterator[np.ndarray]:
    """perform_dips (dips/src/lib.rs:252-257) minus the GStreamer decode
    front-end (out of scope): runs the frame callback over an iterable of
    RGBA8 frames and yields the callback's outputs in order.  With the
    default callback and batch > 0, frames are grouped `batch` at a time
    through dips_frame_callback_batch (same outputs, one device pass each)."""
    cs = ComputeState(properties.colorize_, properties.spatial_window_size_,
                      properties.sensitivity_, properties.filter_type_,
                      properties.chroma_filter_, device)
    cb = properties.get_frame_callback()
    try:
        if cb is None and batch > 0:
            pending = []
            for f in frames:
                pending.append(np.asarray(f, dtype=np.uint8).reshape(height, width, 4))
                if len(pending) == batch:
                    yield from cs.frame_callback_batch(width, height, np.stack(pending))
                    pending = []
            if pending:
                yield from cs.frame_callback_batch(width, height, np.stack(pending))
            return
        cb = cb or frame_callback
        for f in frames:
            yield cb(width, height, f, cs)
    finally:
        cs.close()


# ---------------------------------------------------------------------------
# Batch difference series (north-star path)
# ---------------------------------------------------------------------------

@dataclass
class Series:
    """Per-frame difference series (see dips_series_entry in dips_hip.h)."""
    sad: np.ndarray       # uint64 [N]
    sj: np.ndarray        # uint64 [N]
    count: np.ndarray     # uint64 [N]
    si_fixed: np.ndarray  # uint64 [N]

    @property
    def si(self) -> np.ndarray:
        return np.ldexp(self.si_fixed.astype(np.float64), -32)

    @property
    def sj_norm(self) -> np.ndarray:
        return self.sj.astype(np.float64) / 510.0

    def as_array(self) -> np.ndarray:
        return np.stack([self.sad, self.sj, self.count, self.si_fixed], axis=1)

    @classmethod
    def from_array(cls, a: np.ndarray) -> "Series":
        a = np.asarray(a, dtype=np.uint64).reshape(-1, 4)
        return cls(a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy(), a[:, 3].copy())


def _frame_geometry(frames, fmt: PixelFormat) -> Tuple[int, int, int]:
    shape = tuple(frames.shape)
    c = int(fmt)
    if c == 1:
        if len(shape) == 4 and shape[3] == 1:
            shape = shape[:3]
        if len(shape) != 3:
            raise ValueError("gray8 frames must be [N, H, W]")
        return shape[0], shape[1], shape[2]
    if len(shape) != 4 or shape[3] != c:
        raise ValueError(f"frames must be [N, H, W, {c}]")
    return shape[0], shape[1], shape[2]


class DiffSeriesOperator:
    """The batch operator: per-frame difference series of a frame stack.

    Inputs are numpy arrays (host; the call stages them through HBM) or
    torch tensors on a HIP device (zero-copy, asynchronous on the tensor's
    current stream)."""

    def __init__(self, fmt: PixelFormat = PixelFormat.RGB8, mode: Mode = Mode.Overall,
                 tau: float = 0.0, chroma_filter: ChromaFilter = ChromaFilter.None_,
                 device: int = 0, time_kernel: bool = False, force_generic: bool = False,
                 crosscheck: bool = False, gray_table: str = "auto"):
        """force_generic: the any-shape kernel; crosscheck: the plain kernels
        (DIPS_FLAG_CROSSCHECK; GRAY8 f32 kernel, f64 intensity sums);
        gray_table: "auto" (the GRAY8 table kernel picks its layout per
        workgroup from the content), "band" or "pair" (pinned,
        DIPS_FLAG_GRAY_BAND_TABLE / _PAIR_TABLE).  All give the same series."""
        tables = {"auto": 0, "band": _lib.FLAG_GRAY_BAND_TABLE, "pair": _lib.FLAG_GRAY_PAIR_TABLE}
        if gray_table not in tables:
            raise ValueError("gray_table must be 'auto', 'band' or 'pair'")
        flags = ((_lib.FLAG_TIME_KERNEL if time_kernel else 0) | (_lib.FLAG_FORCE_GENERIC if force_generic else 0)
                 | (_lib.FLAG_CROSSCHECK if crosscheck else 0) | tables[gray_table])
        self.fmt = PixelFormat(fmt)
        self.mode = Mode(mode)
        self.tau = float(tau)
        self._host = _Handle(_params(fmt=self.fmt, mode=self.mode, tau=tau,
                                     chroma_filter=chroma_filter, flags=flags), device)
        self._dev = _Handle(_params(fmt=self.fmt, mode=self.mode, tau=tau,
                                    chroma_filter=chroma_filter,
                                    flags=flags | _lib.FLAG_DEVICE_PTRS), device)

    def close(self) -> None:
        self._host.close()
        self._dev.close()

    # -- host arrays -------------------------------------------------------
    def __call__(self, frames: np.ndarray, ref: Optional[np.ndarray] = None,
                 want_map: bool = False) -> Tuple[Series, Optional[np.ndarray]]:
        frames = _as_u8(frames)
        n, h, w = _frame_geometry(frames, self.fmt)
        out = np.zeros((n, 4), dtype=np.uint64)
        dmap = np.empty_like(frames) if want_map else None
        rp = None
        if ref is not None:
            ref = _as_u8(ref)
            if ref.size != h * w * int(self.fmt):
                raise ValueError("ref must have the shape of one frame")
            rp = ref.ctypes.data
        self._host.check(self._host._lib.dips_diff_series(
            self._host.ptr, w, h, frames.ctypes.data, n, rp, out.ctypes.data,
            dmap.ctypes.data if dmap is not None else None))
        return Series.from_array(out), dmap

    def streamed(self, frames: np.ndarray, ref: Optional[np.ndarray] = None,
                 chunk_frames: int = 0) -> Series:
        """Pinned-staging + side-stream DMA feed (dips_diff_series_streamed)."""
        frames = _as_u8(frames)
        n, h, w = _frame_geometry(frames, self.fmt)
        out = np.zeros((n, 4), dtype=np.uint64)
        rp = None
        if ref is not None:
            ref = _as_u8(ref)
            if ref.size != h * w * int(self.fmt):
                raise ValueError("ref must have the shape of one frame")
            rp = ref.ctypes.data
        self._host.check(self._host._lib.dips_diff_series_streamed(
            self._host.ptr, w, h, frames.ctypes.data, n, rp, out.ctypes.data, int(chunk_frames)))
        return Series.from_array(out)

    # -- device tensors (torch, HIP) ----------------------------------------
    def run_device(self, frames, series_out, ref=None, map_out=None, stream=None) -> None:
        """Asynchronous: frames / ref / map_out uint8 device tensors,
        series_out an int64 device tensor of shape [N, 4]."""
        n, h, w = _frame_geometry(frames, self.fmt)
        if tuple(series_out.shape) != (n, 4) or series_out.element_size() != 8:
            raise ValueError("series_out must be an 8-byte tensor of shape [N, 4]")
        for t in (frames, series_out, ref, map_out):
            if t is not None and (not t.is_cuda or not t.is_contiguous()):
                raise ValueError("device path needs contiguous HIP tensors")
        import torch
        for t in (frames, ref, map_out):
            if t is not None and t.dtype != torch.uint8:
                raise ValueError("frames, ref and map_out must be uint8 tensors")
        if ref is not None and ref.numel() != h * w * int(self.fmt):
            raise ValueError("ref must have the size of one frame")
        if map_out is not None and tuple(map_out.shape) != tuple(frames.shape):
            raise ValueError("map_out must have the shape of frames")
        lib = self._dev._lib
        with _stream_of(self._dev, frames, stream):
            self._dev.check(lib.dips_diff_series(
                self._dev.ptr, w, h, frames.data_ptr(), n,
                ref.data_ptr() if ref is not None else None, series_out.data_ptr(),
                map_out.data_ptr() if map_out is not None else None))

    # -- frame-range sharding (native: shard_abi.hip) -------------------------
    def run_sharded(self, comm, frames, n_total: int, series_local, series_all=None, ref=None,
                    ref_resident: bool = False, stream=None) -> None:
        """dips_diff_series_sharded on device tensors, asynchronous on the
        tensor's current stream: this rank's frames [n_local, H, W(, C)]
        (its dips_shard_range of n_total), series_local int64 [n_local, 4],
        series_all int64 [n_total, 4] on rank 0 (ignored elsewhere); `ref`:
        'overall' rank 0's reference (None = its first frame) or, with
        ref_resident, every rank's copy; 'per-frame' rank 0's predecessor of
        global frame 0 (None = frame 0)."""
        n, h, w = _frame_geometry(frames, self.fmt)
        if tuple(series_local.shape) != (n, 4) or series_local.element_size() != 8:
            raise ValueError("series_local must be an 8-byte tensor of shape [n_local, 4]")
        if comm.rank == 0 and (series_all is None or tuple(series_all.shape) != (int(n_total), 4)
                               or series_all.element_size() != 8):
            raise ValueError("rank 0 needs series_all, an 8-byte tensor of shape [n_total, 4]")
        for t in (frames, series_local, series_all, ref):
            if t is not None and (not t.is_cuda or not t.is_contiguous()):
                raise ValueError("device path needs contiguous HIP tensors")
        if ref is not None and ref.numel() != h * w * int(self.fmt):
            raise ValueError("ref must have the size of one frame")
        lib = self._dev._lib
        with _stream_of(self._dev, frames, stream):
            self._dev.check(lib.dips_diff_series_sharded(
                self._dev.ptr, comm.ptr, w, h, frames.data_ptr(), n, int(n_total),
                ref.data_ptr() if ref is not None else None,
                _lib.SHARD_REF_RESIDENT if ref_resident else 0, series_local.data_ptr(),
                series_all.data_ptr() if (series_all is not None and comm.rank == 0) else None))

    def sharded(self, comm, frames: np.ndarray, n_total: int, ref: Optional[np.ndarray] = None,
                ref_resident: bool = False) -> Tuple[Series, Optional[Series]]:
        """The same on host arrays (staged through HBM, synchronous):
        returns (this rank's series, the gathered series on rank 0 / None)."""
        frames = _as_u8(frames)
        n, h, w = _frame_geometry(frames, self.fmt)
        local = np.zeros((n, 4), dtype=np.uint64)
        full = np.zeros((int(n_total), 4), dtype=np.uint64) if comm.rank == 0 else None
        rp = None
        if ref is not None:
            ref = _as_u8(ref)
            if ref.size != h * w * int(self.fmt):
                raise ValueError("ref must have the shape of one frame")
            rp = ref.ctypes.data
        self._host.check(self._host._lib.dips_diff_series_sharded(
            self._host.ptr, comm.ptr, w, h, frames.ctypes.data, n, int(n_total), rp,
            _lib.SHARD_REF_RESIDENT if ref_resident else 0, local.ctypes.data,
            full.ctypes.data if full is not None else None))
        return Series.from_array(local), (Series.from_array(full) if full is not None else None)

    def shard_broadcast_device(self, comm, frame, out, stream=None) -> None:
        """Rank 0's `frame` into `out` on every rank (dips_shard_broadcast)."""
        h, w = int(out.shape[0]), int(out.shape[1])
        lib = self._dev._lib
        with _stream_of(self._dev, out, stream):
            self._dev.check(lib.dips_shard_broadcast(self._dev.ptr, comm.ptr, w, h,
                                                     frame.data_ptr() if frame is not None else None,
                                                     out.data_ptr()))

    def shard_plan(self, comm, width: int, height: int, n_total: int) -> dict:
        """dips_shard_plan: this rank's frame range and the waves of its
        series launch beside the halo transfer (and uncapped)."""
        first, count = ctypes.c_uint64(), ctypes.c_uint32()
        waves, unc = ctypes.c_uint64(), ctypes.c_uint64()
        self._dev.check(self._dev._lib.dips_shard_plan(self._dev.ptr, comm.ptr, width, height, int(n_total),
                                                       ctypes.byref(first), ctypes.byref(count),
                                                       ctypes.byref(waves), ctypes.byref(unc)))
        return {"first": first.value, "count": count.value, "waves": waves.value, "waves_uncapped": unc.value}

    def shard_reference_device(self, out, stream=None) -> bool:
        """The reference the last run_sharded used for this rank's first
        frame, into a uint8 device tensor; False before any sharded call."""
        with _stream_of(self._dev, out, stream):
            return self._dev.check(self._dev._lib.dips_shard_reference(self._dev.ptr, out.data_ptr(),
                                                                       out.numel())) == 1

    def synth_device(self, dst, width: int, height: int, seed: int, t0: int, stream=None) -> None:
        """Fill a uint8 device tensor [N, H, W(, C)] with synthetic frames t0..t0+N-1."""
        n = dst.shape[0]
        lib = self._dev._lib
        with _stream_of(self._dev, dst, stream):
            self._dev.check(lib.dips_synth_frames(self._dev.ptr, width, height, int(seed), int(t0), n,
                                                  dst.data_ptr()))

    def read_ceiling_ms(self, tensor) -> float:
        """hipEvent time of one read-only stream over a device tensor's bytes."""
        ms = ctypes.c_double()
        self._dev.check(self._dev._lib.dips_read_ceiling(self._dev.ptr, tensor.data_ptr(),
                                                         tensor.numel() * tensor.element_size(),
                                                         ctypes.byref(ms)))
        return ms.value

    def read_ceiling_walk_ms(self, frames) -> float:
        """hipEvent time of one read-only walk over device frames [N, H, W, C]
        in the series kernel's own access shape (RGB8 / RGBA8)."""
        n, h, w = _frame_geometry(frames, self.fmt)
        ms = ctypes.c_double()
        self._dev.check(self._dev._lib.dips_read_ceiling_walk(self._dev.ptr, frames.data_ptr(), w, h, n,
                                                              ctypes.byref(ms)))
        return ms.value

    def kernel_times(self) -> List[float]:
        """Per-launch hipEvent times (ms) of the series kernel since the last reset."""
        lib, ptr = self._dev._lib, self._dev.ptr
        n = ctypes.c_uint64()
        self._dev.check(lib.dips_kernel_time_each(ptr, None, 0, ctypes.byref(n)))
        buf = (ctypes.c_double * max(1, n.value))()
        self._dev.check(lib.dips_kernel_time_each(ptr, buf, n.value, ctypes.byref(n)))
        return list(buf[: n.value])

    def kernel_time(self, reset: bool = False) -> Tuple[float, int]:
        ms = ctypes.c_double()
        cnt = ctypes.c_uint64()
        self._dev.check(self._dev._lib.dips_kernel_time(self._dev.ptr, ctypes.byref(ms), ctypes.byref(cnt)))
        out = (ms.value, cnt.value)
        if reset:
            self._dev.check(self._dev._lib.dips_kernel_time_reset(self._dev.ptr))
        return out

    def geometry(self, width: int, height: int, n_frames: int) -> Tuple[int, int, int]:
        waves, tiles, pbytes = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._dev.check(self._dev._lib.dips_series_geometry(
            self._dev.ptr, width, height, n_frames, ctypes.byref(waves), ctypes.byref(tiles),
            ctypes.byref(pbytes)))
        return waves.value, tiles.value, pbytes.value


def diff_series(frames: np.ndarray, *, fmt: Optional[PixelFormat] = None, mode: Mode = Mode.Overall,
                tau: float = 0.0, chroma_filter: ChromaFilter = ChromaFilter.None_,
                ref: Optional[np.ndarray] = None, want_map: bool = False, device: int = 0,
                force_generic: bool = False, crosscheck: bool = False) -> Tuple[Series, Optional[np.ndarray]]:
    """One-shot helper over DiffSeriesOperator for host arrays."""
    if fmt is None:
        fmt = PixelFormat.Gray8 if frames.ndim == 3 else PixelFormat(frames.shape[-1])
    op = DiffSeriesOperator(fmt, mode, tau, chroma_filter, device, force_generic=force_generic,
                            crosscheck=crosscheck)
    try:
        return op(frames, ref=ref, want_map=want_map)
    finally:
        op.close()


def si_from_fixed(si_fixed) -> np.ndarray:
    return np.ldexp(np.asarray(si_fixed, dtype=np.float64), -32)


__all__ = [
    "DiPsFilter", "ChromaFilter", "PixelFormat", "Mode", "DiPsProperties", "ComputeState",
    "frame_callback", "perform_dips_frames", "Series", "DiffSeriesOperator", "diff_series",
    "si_from_fixed", "VideoPathNotSpecifiedError", "FrameCallbackNotSpecifiedError", "DipsError",
]
