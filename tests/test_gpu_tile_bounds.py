"""Frame sizes around the series kernels' tile boundaries, against the
oracle.  A tile is one wave's slice of a frame: 64 lanes x U vecs of 4 px --
1,280 px for RGB8 (U = 5), 1,024 px for RGBA8 (U = 4), 64 x 16 x 4 = 4,096 px
for the GRAY8 table kernel -- and the pixels past the last whole vec go to
the generic kernel.  Each size runs in both modes, with the u8 map, in
batches of 7 and 260 frames (frames this small keep one contiguous range
per wave); the part-major schedule (series_abi.hip part_geometry) with a
partial last tile is the second test."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

TAU = 8 / 255
TILE_PX = {3: 64 * 5 * 4, 4: 64 * 4 * 4, 1: 64 * 16 * 4}


def _fmt(c):
    from dips_amd import PixelFormat
    return {1: PixelFormat.Gray8, 3: PixelFormat.RGB8, 4: PixelFormat.RGBA8}[c]


def _sizes(c):
    t = TILE_PX[c]
    return [t - 4, t - 1, t, t + 1, t + 4, 2 * t + 3, 3 * t - 5]


@pytest.mark.parametrize("c", [3, 4, 1])
def test_tile_boundary_sizes(c):
    from dips_amd import DiffSeriesOperator, Mode
    rng = np.random.default_rng(20261018 + c)
    for npx in _sizes(c):
        # two frame shapes of the same pixel count where it factors
        shapes = [(1, npx)] + ([(2, npx // 2)] if npx % 2 == 0 else [])
        for h, w in shapes:
            for n in (7, 260):
                fr = rng.integers(0, 256, (n, h, w) if c == 1 else (n, h, w, c), dtype=np.uint8)
                # a little temporal coherence so that some pixels stay under tau
                fr[1::2] = fr[0::2][: len(fr[1::2])] ^ np.uint8(3)
                for mode in (Mode.Overall, Mode.PerFrame):
                    op = DiffSeriesOperator(_fmt(c), mode, TAU)
                    try:
                        got, dmap = op(fr, want_map=True)
                        want, _, want_map = oracle.series(fr, mode=int(mode), tau=TAU, want_map=True)
                        assert np.array_equal(got.as_array(), want), (c, npx, (h, w), n, mode)
                        assert np.array_equal(dmap, want_map), (c, npx, (h, w), n, mode)
                    finally:
                        op.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("c", [3, 4])
def test_part_major_with_partial_last_tile(c):
    """Frames of 1,030 tiles minus 3 pixels (a partial last tile and 3
    trailing pixels for the generic kernel) in a 1,024-frame per-frame batch:
    the part-major schedule (parts of >= 128 frames), asserted through
    the library's wave count (tests/_sched.py), every frame against the
    oracle."""
    import torch
    from _sched import library_schedule
    from dips_amd import DiffSeriesOperator, Mode
    npx = 1030 * TILE_PX[c] - 3
    n = 1024
    rng = np.random.default_rng(77 + c)
    fr = rng.integers(0, 256, (n, 1, npx, c), dtype=np.uint8)
    fr[1::2] = fr[0::2] ^ np.uint8(3)
    op = DiffSeriesOperator(_fmt(c), Mode.PerFrame, TAU)
    try:
        sch = library_schedule(op, npx, 1, n)
        assert sch is not None and sch[1] >= 2, sch  # part-major
        dev = torch.from_numpy(fr).cuda()
        ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        op.run_device(dev, ser)
        torch.cuda.synchronize()
        got = ser.cpu().numpy().view(np.uint64)
    finally:
        op.close()
    want, _, _ = oracle.series(fr, mode=1, tau=TAU, nthreads=16)
    bad = np.nonzero(~np.all(got == want, axis=1))[0]
    assert bad.size == 0, f"frames differing from the oracle: {bad[:10]}"
