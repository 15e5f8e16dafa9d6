"""Failures are visible at the boundary: a call the
library cannot serve returns a negative dips_status and a message
(dips_last_error), never the warm-up's 0 / None or a passthrough copy, and
the Python binding raises DipsError for it (the Rust crate's try_dispatch /
dispatch / frame_callback are checked as source in tests/test_rust_shim.py).
Reference: dips/src/gpu/mod.rs:306-397 (dispatch), dips/src/lib.rs:233-246
(frame_callback), whose wgpu errors panic."""
import ctypes

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def test_dispatch_error_is_negative_with_a_message():
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, _lib
    w, h = 64, 32
    frames = np.random.default_rng(3).integers(0, 256, (6, h, w, 4), dtype=np.uint8)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    try:
        small = np.empty(w * h * 4 - 1, dtype=np.uint8)
        # warm-up: None (0) even with a small buffer -- nothing to write yet
        cs.add_texture(w, h, frames[0])
        assert lib.dips_dispatch(hd.ptr, small.ctypes.data, small.nbytes) == 0
        for f in frames[1:4]:
            cs.add_texture(w, h, f)
        # steady state: a buffer one byte short is an error, not None
        st = lib.dips_dispatch(hd.ptr, small.ctypes.data, small.nbytes)
        assert st == _lib.DIPS_ERR_CAPACITY, st
        assert b"smaller than width*height*4" in lib.dips_last_error(hd.ptr)
        # a null output as well
        assert lib.dips_dispatch(hd.ptr, None, w * h * 4) == _lib.DIPS_ERR_INVALID
        # the handle still works, and equals the oracle
        ref = oracle.ComputeState(False, 1, 5.0, 255, 0)
        for f in frames[:4]:
            ref.add_texture(w, h, f)
        assert np.array_equal(cs.dispatch(), ref.dispatch())
    finally:
        cs.close()


def test_frame_callback_error_raises_not_passthrough():
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, DipsError, _lib, frame_callback
    w, h = 64, 32
    frames = np.random.default_rng(4).integers(0, 256, (6, h, w, 4), dtype=np.uint8)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    try:
        for f in frames[:5]:
            frame_callback(w, h, f, cs)
        out = np.zeros(w * h * 4, dtype=np.uint8)
        # a frame of another size after the first: an error, the output untouched
        st = lib.dips_frame_callback(hd.ptr, w, h - 1, frames[5].ctypes.data, w * (h - 1) * 4, out.ctypes.data,
                                     out.nbytes)
        assert st < 0 and lib.dips_last_error(hd.ptr), st
        assert not out.any()
        with pytest.raises(DipsError):
            frame_callback(w, h - 1, frames[5][: h - 1], cs)
        with pytest.raises(DipsError):
            cs.add_texture(w, h, frames[5][:, :-1])  # wrong length
        # an output buffer too small: capacity error
        st = lib.dips_frame_callback(hd.ptr, w, h, frames[5].ctypes.data, frames[5].nbytes, out.ctypes.data, 16)
        assert st == _lib.DIPS_ERR_CAPACITY
    finally:
        cs.close()


def test_series_errors_are_statuses():
    from dips_amd import DiffSeriesOperator, DipsError, Mode, PixelFormat, _lib
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255)
    try:
        lib, hd = op._host._lib, op._host
        ser = (ctypes.c_uint64 * 4)()
        st = lib.dips_diff_series(hd.ptr, 0, 4, None, 1, None, ctypes.byref(ser), None)
        assert st == _lib.DIPS_ERR_INVALID and b"null or empty" in lib.dips_last_error(hd.ptr)
        import torch
        tiny = torch.zeros((1, 1, 1, 3), dtype=torch.uint8, device="cuda")
        with pytest.raises(DipsError):
            op.read_ceiling_walk_ms(tiny)  # one pixel: no whole vec, not eligible for the walk
    finally:
        op.close()
