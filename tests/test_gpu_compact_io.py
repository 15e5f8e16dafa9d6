"""The per-frame zero-copy path's I/O forms against the oracle:
the packed input (DIPS_COMPACT_IN: (max, min) of R, G, B per pixel, or the
chroma channel), the keyed output (DIPS_COMPACT_OUT: 1-B gray / 2-B colour
keys expanded by the copy pool), the two-pixels-per-thread kernel
(DIPS_HOST_PX=2, compat_main_host2_kernel) and the plain RGBA8 forms, on an
odd width whose row stripes start at odd pixel offsets (y0 * width odd cuts
pixel pairs), for colour on and off, every filter and every chroma filter.
ComputeState.frame_callback and add_texture + dispatch (the deferred form)
must equal the oracle's ComputeState (dips/src/gpu/mod.rs:170-397,
dips/src/lib.rs:233-246) byte for byte.  One case also runs on pinned
buffers built from huge pages (DIPS_PIN_HUGE=1, hipHostRegister)."""
import itertools

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

W, H = 997, 61  # odd width: stripes of 13 rows start at rows 3, 16, 29, ... (3 * 997, 29 * 997 odd)

PROPS = [(False, 5.0, 255, 0), (True, 5.0, 0, 0), (False, 0.7, 1, 1), (True, 2.5, 255, 2), (True, 5.0, 1, 3)]
FORMS = list(itertools.product(["0", "1"], ["0", "1"], ["1", "2"]))  # COMPACT_OUT, COMPACT_IN, HOST_PX


def _frames(n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, H, W, 4), dtype=np.uint8)
    # tie-heavy rows: equal channels (gray pixels) and odd max + min
    f[:, ::5, :, :3] = f[:, ::5, :, :1]
    f[5] = f[4]
    return f


def _run(monkeypatch, props, out_form, in_form, px, huge=False, direct="1"):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    colorize, sens, filt, chroma = props
    monkeypatch.setenv("DIPS_CALLBACK_DIRECT", direct)
    monkeypatch.setenv("DIPS_COMPACT_OUT", out_form)
    monkeypatch.setenv("DIPS_COMPACT_IN", in_form)
    monkeypatch.setenv("DIPS_HOST_PX", px)
    monkeypatch.setenv("DIPS_PIECE_BYTES", str(13 * W * 4))
    monkeypatch.setenv("DIPS_PIN_HUGE", "1" if huge else "0")
    frames = _frames(14, 31 + filt + 7 * chroma)
    cs = ComputeState(colorize, 1, sens, DiPsFilter(filt), ChromaFilter(chroma))
    ref = oracle.ComputeState(colorize, 1, sens, filt, chroma)
    try:
        for k in range(10):
            got = frame_callback(W, H, frames[k], cs)
            want = oracle.frame_callback(W, H, frames[k], ref)
            assert np.array_equal(got, want), (k, np.argwhere(got != want)[:4])
        # the deferred add_texture + dispatch form on the same handle
        for k in range(10, 14):
            cs.add_texture(W, H, frames[k])
            ref.add_texture(W, H, frames[k])
            a, b = cs.dispatch(), ref.dispatch()
            assert np.array_equal(a, b), (k, np.argwhere(a != b)[:4])
    finally:
        cs.close()


@pytest.mark.parametrize("out_form,in_form,px", FORMS)
@pytest.mark.parametrize("props", PROPS)
def test_zero_copy_io_forms_match_oracle(monkeypatch, props, out_form, in_form, px):
    _run(monkeypatch, props, out_form, in_form, px)


def test_zero_copy_on_huge_page_pinned_buffers(monkeypatch):
    _run(monkeypatch, (True, 5.0, 0, 0), "1", "1", "1", huge=True)
    _run(monkeypatch, (False, 5.0, 255, 2), "0", "0", "2", huge=True)


@pytest.mark.parametrize("props", PROPS)
def test_copy_engine_keys_path_matches_oracle(monkeypatch, props):
    """DIPS_CALLBACK_DIRECT=2: the packed input and the keys travel by the
    copy engines (host_stream.h run_striped_frame_dma_keys), the kernel runs
    on HBM copies -- same outputs as the oracle."""
    _run(monkeypatch, props, "1", "1", "1", direct="2")


@pytest.mark.parametrize("direct", ["1", "2"])
def test_sleeping_waits_match_oracle(monkeypatch, direct):
    """DIPS_CB_BLOCKING=1 (blocking-sync stripe events, condition-variable
    waits) on both per-frame pipelines: same outputs."""
    monkeypatch.setenv("DIPS_CB_BLOCKING", "1")
    _run(monkeypatch, (True, 5.0, 0, 0), "1", "1", "1", direct=direct)
    _run(monkeypatch, (False, 5.0, 255, 3), "1", "1", "1", direct=direct)
