"""The largest frames, on both sides of the vectorised kernels' limit: a
frame of 2^31 bytes or more (the kernels' 32-bit frame offsets) goes to the
generic kernel with 64-bit offsets, one just under it to the vectorised
kernel (series_abi.hip fast_geometry / gray_lut_geometry)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

TAU = 8 / 255
LIMIT = 1 << 31
# (channels, width, height): the first of each pair just under 2^31 bytes,
# the second just over
SHAPES = [(3, 32768, 21845), (3, 32768, 21846), (4, 32768, 16383), (4, 32768, 16385),
          (1, 65536, 32767), (1, 65536, 32769)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("c,w,h", SHAPES, ids=lambda v: str(v))
def test_frames_at_the_2gib_limit(c, w, h):
    """Two synthesised frames, 'per-frame' mode: frame 1 against frame 0
    (its bytes 2^31 or more past the batch start on the far side) checked
    against the oracle, frame 0 against itself all zero.  ('overall' runs
    the same kernels with the reference pointer set.)"""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fb = w * h * c
    assert (fb < LIMIT) == (h in (21845, 16383, 32767))
    fmt = {1: PixelFormat.Gray8, 3: PixelFormat.RGB8, 4: PixelFormat.RGBA8}[c]
    shape = (2, h, w) if c == 1 else (2, h, w, c)
    op = DiffSeriesOperator(fmt, Mode.PerFrame, TAU)
    try:
        frames = torch.empty(shape, dtype=torch.uint8, device="cuda")
        op.synth_device(frames, w, h, 0xD1B5, 11)
        ser = torch.zeros((2, 4), dtype=torch.int64, device="cuda")
        op.run_device(frames, ser)
        torch.cuda.synchronize()
        got = ser.cpu().numpy().view(np.uint64)
        host = frames.cpu().numpy()
        del frames
        torch.cuda.empty_cache()
    finally:
        op.close()
    assert not got[0].any()
    assert got[1, 0] > 0 and np.array_equal(got[1], _oracle_frame(host[1], host[0], c)), (c, w, h, got[1])


def _oracle_frame(cur, ref, c, parts=16):
    """The oracle's series entry of one frame against a reference, in 16
    pixel slices on 16 threads (every field is a per-pixel sum, SI as an exact
    fixed-point integer, so the slices' entries add up to the frame's)."""
    from concurrent.futures import ThreadPoolExecutor
    npx = cur.size // c
    assert npx % parts == 0
    a = cur.reshape(parts, 1, npx // parts, c) if c > 1 else cur.reshape(parts, 1, npx // parts)
    b = ref.reshape(a.shape)
    with ThreadPoolExecutor(parts) as ex:
        rows = list(ex.map(lambda k: oracle.series(a[k:k + 1], mode=0, tau=TAU, ref=b[k])[0][0], range(parts)))
    return np.sum(np.stack(rows), axis=0, dtype=np.uint64)
