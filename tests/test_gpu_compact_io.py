"""The per-frame zero-copy path's I/O forms against the oracle:
the packed input ((max, min) of R, G, B per pixel, or the chroma channel,
packed by the copy pool) and the keyed output (1-B gray / 2-B colour keys
expanded by the copy pool), against the cross-check form
(DIPS_FLAG_CROSSCHECK: whole RGBA8 frames by DMA through add_texture +
dispatch), on an odd width whose row stripes start at odd pixel offsets
(host_stream.h piece_bytes: stripes of 15 rows from row 3, so 3 * 997 and
33 * 997 cut the packed kernel's pixel groups), for colour on and off,
every filter and every chroma filter.  ComputeState.frame_callback and
add_texture + dispatch (the deferred form) must equal the oracle's
ComputeState (dips/src/gpu/mod.rs:170-397, dips/src/lib.rs:233-246) byte for
byte."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

W, H = 997, 61

PROPS = [(False, 5.0, 255, 0), (True, 5.0, 0, 0), (False, 0.7, 1, 1), (True, 2.5, 255, 2), (True, 5.0, 1, 3)]


def _frames(n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, H, W, 4), dtype=np.uint8)
    # tie-heavy rows: equal channels (gray pixels) and odd max + min
    f[:, ::5, :, :3] = f[:, ::5, :, :1]
    f[5] = f[4]
    return f


@pytest.mark.parametrize("crosscheck", [False, True])
@pytest.mark.parametrize("props", PROPS)
def test_zero_copy_io_forms_match_oracle(props, crosscheck):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    colorize, sens, filt, chroma = props
    frames = _frames(14, 31 + filt + 7 * chroma)
    cs = ComputeState(colorize, 1, sens, DiPsFilter(filt), ChromaFilter(chroma), crosscheck=crosscheck)
    ref = oracle.ComputeState(colorize, 1, sens, filt, chroma)
    try:
        for k in range(10):
            got = frame_callback(W, H, frames[k], cs)
            want = oracle.frame_callback(W, H, frames[k], ref)
            assert np.array_equal(got, want), (k, np.argwhere(got != want)[:4])
            if not crosscheck and k >= 4:
                ph = cs.callback_phases()  # the zero-copy path ran (and left its record)
                assert ph is not None and ph["stripes"] == 5, ph
        # the deferred add_texture + dispatch form on the same handle
        for k in range(10, 14):
            cs.add_texture(W, H, frames[k])
            ref.add_texture(W, H, frames[k])
            a, b = cs.dispatch(), ref.dispatch()
            assert np.array_equal(a, b), (k, np.argwhere(a != b)[:4])
    finally:
        cs.close()
