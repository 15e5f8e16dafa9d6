"""Edge cases of the C ABI against the oracle: empty batches (every batch
entry point returns OK, writes nothing and leaves the operator's state as it
was), a 1x1 frame and 1-pixel-wide / -high frames in every format and mode,
a batch of one frame, and arguments the library must refuse (zero width or
height with frames, a frame size change inside a ComputeState, a dips_alt
frame of the wrong size) with DIPS_ERR_INVALID and a message."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

TAU = 8 / 255


def _fmt(c):
    from dips_amd import PixelFormat
    return {1: PixelFormat.Gray8, 3: PixelFormat.RGB8, 4: PixelFormat.RGBA8}[c]


def _frames(n, h, w, c, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (n, h, w) if c == 1 else (n, h, w, c), dtype=np.uint8)


@pytest.mark.parametrize("c", [1, 3, 4])
def test_empty_series_batches(c):
    import torch
    from dips_amd import DiffSeriesOperator, Mode
    shape = (0, 8, 16) if c == 1 else (0, 8, 16, c)
    empty = np.zeros(shape, np.uint8)
    for mode in (Mode.Overall, Mode.PerFrame):
        op = DiffSeriesOperator(_fmt(c), mode, TAU)
        try:
            got, dmap = op(empty, want_map=True)
            assert got.as_array().shape == (0, 4) and dmap.shape == shape
            assert op.streamed(empty).as_array().shape == (0, 4)
            ref = np.zeros(shape[1:], np.uint8)
            assert op(empty, ref=ref)[0].as_array().shape == (0, 4)
            dev = torch.empty(shape, dtype=torch.uint8, device="cuda")
            ser = torch.full((0, 4), 7, dtype=torch.int64, device="cuda")
            op.run_device(dev, ser)
            torch.cuda.synchronize()
            # the operator still works after the empty calls
            fr = _frames(3, 8, 16, c, 5)
            got, _ = op(fr)
            assert np.array_equal(got.as_array(), oracle.series(fr, mode=int(mode), tau=TAU)[0])
        finally:
            op.close()


@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("hw", [(1, 1), (1, 37), (29, 1), (2, 3)])
def test_tiny_frames_and_single_frame_batches(c, hw):
    from dips_amd import DiffSeriesOperator, Mode
    h, w = hw
    fr = _frames(5, h, w, c, 11 + h + w + c)
    for mode in (Mode.Overall, Mode.PerFrame):
        op = DiffSeriesOperator(_fmt(c), mode, TAU)
        try:
            for batch in (fr, fr[:1]):
                got, dmap = op(batch, want_map=True)
                want, _, want_map = oracle.series(batch, mode=int(mode), tau=TAU, want_map=True)
                assert np.array_equal(got.as_array(), want), (hw, mode, len(batch))
                assert np.array_equal(dmap, want_map)
        finally:
            op.close()


def test_empty_visual_batches_keep_state():
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    from dips_amd.alt import DiPsCompute, DiPsProperties
    rng = np.random.default_rng(3)
    w, h = 24, 10
    fr = rng.integers(0, 256, (9, h, w, 4), dtype=np.uint8)
    cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    ref = oracle.ComputeState(True, 1, 5.0, 0, 0)
    try:
        a = cs.frame_callback_batch(w, h, fr[:5])
        assert cs.frame_callback_batch(w, h, fr[:0]).shape == (0, h, w, 4)
        b = cs.frame_callback_batch(w, h, fr[5:])
        want = np.stack([oracle.frame_callback(w, h, f, ref) for f in fr])
        assert np.array_equal(np.concatenate([a, b]), want)
    finally:
        cs.close()
    alt = DiPsCompute(2, h, w, DiPsProperties())
    aref = oracle.AltCompute(2, w, h)
    try:
        x = alt.send_frames(fr[:4], [False, False, True, False])
        assert alt.send_frames(fr[:0], []).shape == (0, h, w, 4)
        y = alt.send_frames(fr[4:], [False] * 5)
        want = np.stack([aref.send_frame(f, snapshot=(k == 2)) for k, f in enumerate(fr)])
        assert np.array_equal(np.concatenate([x, y]), want)
    finally:
        alt.close()


def test_invalid_arguments_are_refused_with_a_message():
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, DipsError, Mode
    from dips_amd import _lib
    from dips_amd.alt import DiPsCompute, DiPsProperties
    op = DiffSeriesOperator(_fmt(3), Mode.Overall, TAU)
    try:
        ser = np.zeros((2, 4), np.uint64)
        fr = _frames(2, 4, 4, 3, 1)
        lib = op._host._lib
        st = lib.dips_diff_series(op._host.ptr, 0, 4, fr.ctypes.data, 2, None, ser.ctypes.data, None)
        assert st == _lib.DIPS_ERR_INVALID
        assert lib.dips_last_error(op._host.ptr)
    finally:
        op.close()
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    try:
        f = np.zeros((6, 8, 4), np.uint8)
        cs.add_texture(8, 6, f)
        with pytest.raises(DipsError) as e:
            cs.add_texture(8, 5, np.zeros((5, 8, 4), np.uint8))  # size change after the first frame
        assert e.value.status == _lib.DIPS_ERR_INVALID and "size" in str(e.value)
    finally:
        cs.close()
    alt = DiPsCompute(2, 6, 8, DiPsProperties())
    try:
        with pytest.raises((DipsError, ValueError)):
            alt.send_frame(np.zeros((6, 7, 4), np.uint8))
    finally:
        alt.close()
