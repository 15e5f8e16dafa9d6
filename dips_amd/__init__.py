"""dips_amd -- MI355X-native (gfx950) DiPs per-pixel frame-difference path.

The compute lives in hand-written HIP kernels behind the C ABI of
include/dips_hip.h (dips_amd/lib/libdips_hip.so); this package is the host
mirror of the reference crate's operator surface (dips/src/lib.rs,
dips/src/gpu/mod.rs) plus the batch difference-series operator and the
frame-range sharding over RCCL (dips_amd.shard).
"""
from . import alt  # dips_alt crate surface (DiPsCompute, run_dips_on_file loop)
from ._lib import DipsError, DipsLibraryError, LIB_PATH, load as load_library
from .api import (ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, DiPsProperties,
                  FrameCallbackNotSpecifiedError, Mode, PixelFormat, Series,
                  VideoPathNotSpecifiedError, diff_series, frame_callback, perform_dips_frames,
                  si_from_fixed)

__all__ = [
    "ChromaFilter", "ComputeState", "DiffSeriesOperator", "DiPsFilter", "DiPsProperties",
    "DipsError", "DipsLibraryError", "FrameCallbackNotSpecifiedError", "LIB_PATH", "Mode",
    "PixelFormat", "Series", "VideoPathNotSpecifiedError", "diff_series", "frame_callback",
    "load_library", "perform_dips_frames", "si_from_fixed",
]
