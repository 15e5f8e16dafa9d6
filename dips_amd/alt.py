"""Host-side mirror of the dips_alt crate's operator surface, over the C ABI.

Reference surface (RubenMovsesyan/DiPs, crate ``dips_alt``):
  Filter / ChromaFilter / DiPsProperties (+ setters)  dips_alt/src/dips_compute/mod.rs:151-234
  DiPsCompute::new / send_frame                      dips_alt/src/dips_compute/mod.rs:270-646
  Encoding                                           dips_alt/src/lib.rs:38-55
  FRAME_COUNT, run_dips_on_file's frame loop         dips_alt/src/lib.rs:36, :554-690
  command line                                       dips_alt/src/main.rs:4-107, help.txt
The OpenCV decode / encode, highgui window, live camera app and egui panel are
out of scope; frames come in and go out as RGBA8 arrays.  Every
frame is computed by libdips_hip.so (alt_kernels.hip); there is no Python
compute path.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import DipsAltParams, DipsError, check_alt

FRAME_COUNT = 2  # dips_alt/src/lib.rs:36


class Filter(enum.IntEnum):
    """dips_alt/src/dips_compute/mod.rs:151-156 (FILTER_TYPE override)."""
    Sigmoid = 0
    InverseSigmoid = 1


class ChromaFilter(enum.IntEnum):
    """dips_alt/src/dips_compute/mod.rs:158-165 (CHROMA_FILTER override)."""
    All = 0
    Red = 1
    Green = 2
    Blue = 3


class Encoding(enum.Enum):
    """dips_alt/src/lib.rs:38-55 (the fourcc of the OpenCV writer)."""
    Uncompressed = "RGBA"
    Huffman = "HFYU"
    H264 = "H264"

    def as_fourcc(self) -> int:
        a, b, c, d = self.value
        return ord(a) | (ord(b) << 8) | (ord(c) << 16) | (ord(d) << 24)


@dataclass
class DiPsProperties:
    """dips_alt/src/dips_compute/mod.rs:167-234 (defaults :176-186)."""
    colorize: bool = True
    window_size: int = 1
    sigmoid_horizontal_scalar: float = 5.0
    filter_type: Filter = Filter.Sigmoid
    chroma_filter: ChromaFilter = ChromaFilter.All

    def set_filter(self, f: Filter) -> None:
        self.filter_type = Filter(f)

    def set_chroma_filter(self, c: ChromaFilter) -> None:
        self.chroma_filter = ChromaFilter(c)

    def set_sigmoid_horizontal_scalar(self, scalar: float) -> None:
        # scalar.clamp(1.0, 10.0) (:218-221); f32::clamp keeps NaN
        s = float(np.float32(scalar))
        self.sigmoid_horizontal_scalar = s if s != s else min(max(s, 1.0), 10.0)

    def set_window_size(self, size: int) -> None:
        # size.clamp(1, 7), even sizes minus one (:223-229); u8 argument
        if not 0 <= int(size) <= 255:
            raise ValueError("window size is a u8")
        w = min(max(int(size), 1), 7)
        self.window_size = w - 1 if w % 2 == 0 else w

    def set_colorize(self, colorize: bool) -> None:
        self.colorize = bool(colorize)


def _params(props: DiPsProperties, num_textures: int, flags: int = 0) -> DipsAltParams:
    p = DipsAltParams()
    check_alt(_lib.load().dips_alt_params_default(ctypes.byref(p)))
    p.colorize = 1 if props.colorize else 0
    p.window_size = int(props.window_size)
    p.sigmoid_horizontal_scalar = float(props.sigmoid_horizontal_scalar)
    p.filter_type = int(props.filter_type)
    p.chroma_filter = int(props.chroma_filter)
    p.num_textures = int(num_textures)
    p.flags = int(flags)
    return p


class _AltHandle:
    def __init__(self, params: DipsAltParams, width: int, height: int, device: int):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        check_alt(self._lib.dips_alt_create(ctypes.byref(params), int(width), int(height), int(device),
                                            ctypes.byref(h)))
        self._h = h

    @property
    def ptr(self) -> ctypes.c_void_p:
        if self._h is None:
            raise DipsError(_lib.DIPS_ERR_STATE, "handle destroyed")
        return self._h

    def check(self, st: int) -> int:
        return check_alt(st, self._h)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            self._lib.dips_alt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _frames_u8(frames, height: int, width: int) -> np.ndarray:
    a = np.ascontiguousarray(frames)
    if a.dtype != np.uint8:
        a = a.astype(np.uint8)
    if a.size % (height * width * 4) != 0:
        raise ValueError(f"frames must be [N, {height}, {width}, 4] RGBA8")
    return a.reshape(-1, height, width, 4)


class DiPsCompute:
    """Drop-in for dips_alt's DiPsCompute on a HIP device.

    ``DiPsCompute(num_textures, textures_width, textures_height, props)``
    keeps the reference's argument order: its callers pass the frame's ROWS
    as textures_width and its COLUMNS as textures_height (lib.rs:596-603),
    and the texture extent is (cols, rows) (mod.rs:283-287)."""

    def __init__(self, num_textures: int, textures_width: int, textures_height: int,
                 dips_properties: Optional[DiPsProperties] = None, device: int = 0,
                 time_kernel: bool = False, force_generic: bool = False, crosscheck: bool = False):
        self.rows, self.cols = int(textures_width), int(textures_height)
        self.num_textures = int(num_textures)
        self.properties = dips_properties or DiPsProperties()
        flags = ((_lib.FLAG_TIME_KERNEL if time_kernel else 0) | (_lib.FLAG_FORCE_GENERIC if force_generic else 0)
                 | (_lib.FLAG_CROSSCHECK if crosscheck else 0))
        p = _params(self.properties, num_textures, flags)
        self._host = _AltHandle(p, self.cols, self.rows, device)
        self._dev_flags = flags | _lib.FLAG_DEVICE_PTRS
        self._device = device
        self._dev: Optional[_AltHandle] = None

    @classmethod
    def new(cls, num_textures, textures_width, textures_height, dips_properties=None, device=0):
        return cls(num_textures, textures_width, textures_height, dips_properties, device)

    # -- reference surface ------------------------------------------------------
    def send_frame(self, frame, snapshot=None) -> np.ndarray:
        """mod.rs:498-646; ``snapshot`` is the reference's Option<()>: any
        value other than None/False takes the snapshot."""
        a = _frames_u8(frame, self.rows, self.cols)
        if a.shape[0] != 1:
            raise ValueError("send_frame takes one frame")
        out = np.empty((self.rows, self.cols, 4), dtype=np.uint8)
        snap = 0 if snapshot is None or snapshot is False else 1
        self._host.check(self._host._lib.dips_alt_send_frame(self._host.ptr, a.ctypes.data, a.nbytes, snap,
                                                             out.ctypes.data, out.nbytes))
        return out

    # -- batch forms -------------------------------------------------------------
    def send_frames(self, frames, snapshots: Optional[Sequence[bool]] = None) -> np.ndarray:
        """len(frames) consecutive send_frame calls in one device pass."""
        a = _frames_u8(frames, self.rows, self.cols)
        n = a.shape[0]
        out = np.empty_like(a)
        flags = None
        if snapshots is not None:
            if len(snapshots) != n:
                raise ValueError("one snapshot flag per frame")
            flags = np.ascontiguousarray(np.asarray(snapshots, dtype=bool).astype(np.uint8))
        self._host.check(self._host._lib.dips_alt_send_frames(
            self._host.ptr, a.ctypes.data, n, flags.ctypes.data if flags is not None else None, out.ctypes.data))
        return out

    def _device_handle(self) -> _AltHandle:
        if self._dev is None:
            self._dev = _AltHandle(_params(self.properties, self.num_textures, self._dev_flags),
                                   self.cols, self.rows, self._device)
        return self._dev

    def send_frames_device(self, frames, out, snapshots: Optional[Sequence[bool]] = None, stream=None) -> None:
        """HBM-resident form (torch uint8 tensors [N, rows, cols, 4]),
        asynchronous on the tensor's current stream.  It keeps its own
        texture/snapshot state, separate from the host-pointer calls."""
        n = int(frames.shape[0])
        if tuple(frames.shape) != (n, self.rows, self.cols, 4) or tuple(out.shape) != tuple(frames.shape):
            raise ValueError("frames/out must be [N, rows, cols, 4] uint8 tensors")
        for t in (frames, out):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("device path needs contiguous HIP tensors")
        hd = self._device_handle()
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        flags = None
        if snapshots is not None:
            flags = np.ascontiguousarray(np.asarray(snapshots, dtype=bool).astype(np.uint8))
        # bound to the caller's stream for this call only (_lib.on_stream)
        with _lib.on_stream(hd._lib.dips_alt_set_stream, hd.ptr, hd.check, stream):
            hd.check(hd._lib.dips_alt_send_frames(hd.ptr, frames.data_ptr(), n,
                                                  flags.ctypes.data if flags is not None else None,
                                                  out.data_ptr()))

    def kernel_time(self, reset: bool = False):
        hd = self._device_handle()
        ms, cnt = ctypes.c_double(), ctypes.c_uint64()
        hd.check(hd._lib.dips_alt_kernel_time(hd.ptr, ctypes.byref(ms), ctypes.byref(cnt)))
        if reset:
            hd.check(hd._lib.dips_alt_kernel_time_reset(hd.ptr))
        return ms.value, cnt.value

    def lut_selfcheck(self) -> int:
        """Mismatches of the batch kernel's epilogue table against the
        specification over every (snapshot byte, max, min) -- 0 expected."""
        n = ctypes.c_uint64()
        self._host.check(self._host._lib.dips_alt_lut_selfcheck(self._host.ptr, ctypes.byref(n)))
        return n.value

    def snapshot_texture(self) -> np.ndarray:
        out = np.empty((self.rows, self.cols), dtype=np.uint8)
        self._host.check(self._host._lib.dips_alt_snapshot_texture(self._host.ptr, out.ctypes.data, out.nbytes))
        return out

    def close(self) -> None:
        self._host.close()
        if self._dev is not None:
            self._dev.close()


class DiPsRunner:
    """run_dips_on_file (dips_alt/src/lib.rs:554-690) minus the OpenCV
    front/back end: one DiPsCompute with FRAME_COUNT textures driven by the
    snapshot / refresh-marker loop, fed frames in pieces of any size."""

    def __init__(self, rows: int, cols: int, properties: Optional[DiPsProperties] = None,
                 refresh_markers: Iterable[int] = (), device: int = 0, num_textures: int = FRAME_COUNT,
                 crosscheck: bool = False):
        self.compute = DiPsCompute(num_textures, rows, cols, properties, device, crosscheck=crosscheck)
        self.markers = np.ascontiguousarray(np.asarray(list(refresh_markers), dtype=np.uint64))

    def __call__(self, frames) -> np.ndarray:
        c = self.compute
        a = _frames_u8(frames, c.rows, c.cols)
        out = np.empty_like(a)
        h = c._host
        h.check(h._lib.dips_alt_run(h.ptr, a.ctypes.data, a.shape[0],
                                    self.markers.ctypes.data if self.markers.size else None,
                                    int(self.markers.size), out.ctypes.data))
        return out

    def run_sharded(self, comm, frames, n_total: int) -> np.ndarray:
        """This rank's part of one loop over an `n_total`-frame video split
        by frame range over `comm` (a dips_amd.comm.Comm; dips_alt_run_sharded):
        `frames` are the rank's frames [first, first + count) of
        comm.shard_range, the result is what the single loop gives them.  The
        runner must be fresh (no frame sent yet) on every rank."""
        c = self.compute
        a = _frames_u8(frames, c.rows, c.cols)
        out = np.empty_like(a)
        h = c._host
        h.check(h._lib.dips_alt_run_sharded(h.ptr, comm.ptr, a.ctypes.data, a.shape[0], int(n_total),
                                            self.markers.ctypes.data if self.markers.size else None,
                                            int(self.markers.size), out.ctypes.data))
        return out

    def run_sharded_device(self, comm, frames, out, n_total: int, stream=None) -> None:
        """run_sharded on HBM-resident frames (torch uint8 [count, rows,
        cols, 4] on the communicator's device), on the tensor's current
        stream; returns once `out` is written."""
        c = self.compute
        n = int(frames.shape[0])
        if tuple(frames.shape) != (n, c.rows, c.cols, 4) or tuple(out.shape) != tuple(frames.shape):
            raise ValueError("frames/out must be [N, rows, cols, 4] uint8 tensors")
        for t in (frames, out):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("device path needs contiguous HIP tensors")
        hd = c._device_handle()
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        with _lib.on_stream(hd._lib.dips_alt_set_stream, hd.ptr, hd.check, stream):
            hd.check(hd._lib.dips_alt_run_sharded(hd.ptr, comm.ptr, frames.data_ptr(), n, int(n_total),
                                                  self.markers.ctypes.data if self.markers.size else None,
                                                  int(self.markers.size), out.data_ptr()))

    def close(self) -> None:
        self.compute.close()


def run_loop_flags(n_frames: int, refresh_markers: Iterable[int] = ()) -> np.ndarray:
    """The snapshot flag run_dips_on_file gives each of frames 0..n-1
    (dips_alt/src/lib.rs:636-670, the same loop as dips_alt_run): a snapshot
    when `index` reaches FRAME_COUNT; index counts up to FRAME_COUNT + 1 and
    restarts at 0 after the frame whose 1-based position is a refresh marker."""
    markers = set(int(m) for m in refresh_markers)
    flags = np.zeros(n_frames, dtype=bool)
    index = overall = 0
    for t in range(n_frames):
        flags[t] = index == FRAME_COUNT
        if index <= FRAME_COUNT:
            index += 1
        overall += 1
        if overall in markers:
            index = 0
    return flags


def run_dips_on_frames(frames, properties: Optional[DiPsProperties] = None,
                       refresh_markers: Iterable[int] = (), device: int = 0) -> np.ndarray:
    """All of a clip's frames ([N, rows, cols, 4] RGBA8) through the
    run_dips_on_file loop; returns the N RGBA8 output frames."""
    a = np.asarray(frames)
    r = DiPsRunner(a.shape[1], a.shape[2], properties, refresh_markers, device)
    try:
        return r(a)
    finally:
        r.close()


# ---------------------------------------------------------------------------
# Command line (dips_alt/src/main.rs:4-107)
# ---------------------------------------------------------------------------

class CliError(ValueError):
    """anyhow! errors of main.rs."""


@dataclass
class CliArgs:
    input_path: str = ""
    output_path: str = ""
    encoding: Encoding = Encoding.Uncompressed
    properties: DiPsProperties = field(default_factory=DiPsProperties)
    refresh_markers: List[int] = field(default_factory=list)
    help: bool = False
    live: bool = False


def parse_args(argv: Sequence[str]) -> CliArgs:
    """main.rs:14-89: `--key=value` options, bare integers are refresh
    markers; the same errors for a bad filter/chroma/number and a missing
    input or output path.  `--help` stops parsing; `--live` (the camera app,
    out of scope) is recorded."""
    a = CliArgs()
    for arg in argv:
        if arg in ("--help", "-h"):
            a.help = True
            return a
        if arg == "--live":
            a.live = True
        split = arg.split("=")
        key = split[0]

        def value() -> str:
            if len(split) < 2:  # split[1] panics in the reference
                raise CliError(f"missing value for {key}")
            return split[1]

        if key == "--input":
            a.input_path = value()
        elif key == "--output":
            a.output_path = value()
        elif key == "--encoding":
            a.encoding = {"RGBA": Encoding.Uncompressed, "HFYU": Encoding.Huffman,
                          "H264": Encoding.H264}.get(value(), Encoding.Uncompressed)
        elif key == "--filter":
            v = value()
            if v not in ("sigmoid", "inv_sig"):
                raise CliError("Invalide Filter Type")
            a.properties.set_filter(Filter.Sigmoid if v == "sigmoid" else Filter.InverseSigmoid)
        elif key == "--chroma":
            v = value()
            if v not in ("r", "g", "b"):
                raise CliError("Invalid Chroma Type")
            a.properties.set_chroma_filter({"r": ChromaFilter.Red, "g": ChromaFilter.Green,
                                            "b": ChromaFilter.Blue}[v])
        elif key == "--sig_scalar":
            try:
                a.properties.set_sigmoid_horizontal_scalar(float(value()))
            except ValueError as e:
                raise CliError(str(e)) from None
        elif key == "--win_size":
            v = value()
            if not v.isdigit() or int(v) > 255:
                raise CliError(f"invalid u8 {v!r}")
            a.properties.set_window_size(int(v))
        elif key == "--colorize":
            a.properties.set_colorize(value() != "false")
        else:
            if not key.isdigit():  # usize parse
                raise CliError(f"invalid digit found in string: {key!r}")
            a.refresh_markers.append(int(key))
    if not a.help:
        if not a.input_path:
            raise CliError("Input file not specified")
        if not a.output_path:
            raise CliError("Output file not specified")
    return a


__all__ = ["FRAME_COUNT", "run_loop_flags", "Filter", "ChromaFilter", "Encoding", "DiPsProperties", "DiPsCompute",
           "DiPsRunner", "run_dips_on_frames", "CliArgs", "CliError", "parse_args"]
