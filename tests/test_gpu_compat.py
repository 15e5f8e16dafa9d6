"""GPU parity tests of the dips-compat ComputeState (add_texture / dispatch /
frame_callback, dips/src/gpu/mod.rs:170-397, dips/src/lib.rs:233-246)
against the CPU oracle's ComputeState twin: bit-exact RGBA8 output for every
parameter combination (the sigmoid/inverse filters use the deterministic
f32 exp/log shared by spec with the oracle)."""
import itertools

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _frames(w, h, n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    f[4] = f[3]
    return f


PARAMS = list(itertools.product([False, True], [1, 2, 3, 5, 11], [5.0, 0.7],
                                [255, 0, 1], [0, 1, 3]))


@pytest.mark.parametrize("colorize,window,sens,filt,chroma", PARAMS)
def test_compute_state_matches_oracle(colorize, window, sens, filt, chroma):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    w, h = (37, 21) if window > 1 else (64, 33)
    frames = _frames(w, h, 10, 7 + window)
    gpu = ComputeState(colorize, window, sens, DiPsFilter(filt), ChromaFilter(chroma))
    ref = oracle.ComputeState(colorize, window, sens, filt, chroma)
    try:
        for k in range(10):
            gpu.add_texture(w, h, frames[k])
            ref.add_texture(w, h, frames[k])
            a, b = gpu.dispatch(), ref.dispatch()
            if k < 3:
                assert a is None and b is None
                continue
            assert a is not None and b is not None
            assert np.array_equal(a, b), (k, np.argwhere(a != b)[:5])
            if k == 3:
                assert np.array_equal(gpu.start_texture(), ref.start_texture())
    finally:
        gpu.close()


def _tie_frames(w, h, n, seed):
    """Frames drawn from five byte values: many equal intensities per window."""
    rng = np.random.default_rng(seed)
    return np.array([0, 1, 2, 128, 255], dtype=np.uint8)[rng.integers(0, 5, (n, h, w, 4))]


@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("chroma", [0, 2])
@pytest.mark.parametrize("window", list(range(2, 12)))
def test_every_window_matches_oracle(window, chroma, ties):
    """Spatial median (dips_shader.wgsl:120-170) for every window 2..11: each
    side 2h = 2..10 and each rank the quirky index maps to (window_net.h
    sorting networks), on a ragged 53x29 frame (partial 16x16 tiles)."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    w, h = 53, 29
    frames = (_tie_frames if ties else _frames)(w, h, 6, 100 + window)
    gpu = ComputeState(True, window, 5.0, DiPsFilter.Unfiltered, ChromaFilter(chroma))
    ref = oracle.ComputeState(True, window, 5.0, 255, chroma)
    try:
        for k in range(6):
            gpu.add_texture(w, h, frames[k])
            ref.add_texture(w, h, frames[k])
            a, b = gpu.dispatch(), ref.dispatch()
            if k < 3:
                continue
            assert np.array_equal(a, b), (k, np.argwhere(a != b)[:5])
            if k == 3:
                assert np.array_equal(gpu.start_texture(), ref.start_texture())
    finally:
        gpu.close()


def test_frame_callback_passthrough_then_visual():
    """lib.rs:241-245: frames 0..2 come back unchanged; from frame 3 on the
    callback returns the visualisation."""
    from dips_amd import ComputeState, DiPsFilter, ChromaFilter, frame_callback
    w, h = 48, 16
    frames = _frames(w, h, 8, 3)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    ref = oracle.ComputeState(False, 1, 5.0, 255, 0)
    try:
        for k in range(8):
            out = frame_callback(w, h, frames[k], cs)
            want = oracle.frame_callback(w, h, frames[k], ref)
            assert np.array_equal(out, want)
            if k < 3:
                assert np.array_equal(out, frames[k])
    finally:
        cs.close()


def test_identical_frames_known_answer():
    """identical frames give 128 for gray pixels at once; a
    pixel with odd max+min such as (10,20,31) gives 129 while the unquantised
    F1..F3 still decide the temporal upper median (t = 3..5; the survey's
    "from frame 7" is one frame late: at t = 6 three of four slots are
    quantised and element [2] is a quantised one), 128 from t = 6 on."""
    from dips_amd import ComputeState, DiPsFilter, ChromaFilter
    w, h = 16, 16
    f = np.zeros((h, w, 4), dtype=np.uint8)
    f[..., 3] = 255
    f[0, 0, :3] = (10, 20, 31)
    f[0, 1, :3] = (100, 101, 102)
    f[0, 2, :3] = (77, 77, 77)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    try:
        for t in range(9):
            cs.add_texture(w, h, f)
            out = cs.dispatch()
            if t < 3:
                assert out is None
                continue
            assert out[0, 2, 0] == 128 and out[0, 1, 0] == 128
            assert out[0, 0, 0] == (129 if t <= 5 else 128)
            assert (out[..., 3] == 255).all()
    finally:
        cs.close()


def test_rejects_bad_input():
    from dips_amd import ComputeState, DiPsFilter, ChromaFilter, DipsError
    with pytest.raises(DipsError):
        ComputeState(False, 12, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    try:
        cs.add_texture(8, 8, np.zeros((8, 8, 4), np.uint8))
        with pytest.raises(DipsError):
            cs.add_texture(8, 4, np.zeros((4, 8, 4), np.uint8))
        with pytest.raises(DipsError):
            cs.add_texture(8, 8, np.zeros((8, 7, 4), np.uint8))
    finally:
        cs.close()


# ---------------------------------------------------------------------------
# dips_frame_callback_batch: the steady-state batch kernel (compat_batch.hip)
# ---------------------------------------------------------------------------

def _oracle_callbacks(frames, params):
    ref = oracle.ComputeState(*params)
    h, w = frames.shape[1], frames.shape[2]
    return np.stack([oracle.frame_callback(w, h, f, ref) for f in frames])


BATCH_PARAMS = list(itertools.product([False, True], [1, 3], [5.0, 0.7, 200.0], [255, 0, 1], [0, 2]))


@pytest.mark.parametrize("colorize,window,sens,filt,chroma", BATCH_PARAMS)
def test_frame_callback_batch_matches_oracle(colorize, window, sens, filt, chroma):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    params = (colorize, window, sens, filt, chroma)
    for (w, h), pieces in [((64, 48), [40]), ((64, 48), [3, 5, 32]), ((37, 21), [10, 30])]:
        frames = _frames(w, h, 40, 21 + window + filt)
        frames[20] = frames[19]
        want = _oracle_callbacks(frames, params)
        cs = ComputeState(colorize, window, sens, DiPsFilter(filt), ChromaFilter(chroma))
        try:
            outs, s = [], 0
            for k in pieces:
                outs.append(cs.frame_callback_batch(w, h, frames[s:s + k]))
                s += k
        finally:
            cs.close()
        got = np.concatenate(outs)
        assert np.array_equal(got, want), ((w, h), pieces, np.argwhere(got != want)[:4])


@pytest.mark.parametrize("scratch_frames", [None, 5])
@pytest.mark.parametrize("chroma", [0, 2])
@pytest.mark.parametrize("window", list(range(2, 12)))
def test_frame_callback_batch_window_matches_oracle(window, chroma, scratch_frames, monkeypatch):
    """W > 1 in steady state: compat_filter_frames writes the filtered ring
    texels of a chunk of frames, then the batch kernel runs on them.  Every
    window 2..11, split calls (the ring carries over), a scratch of 5 frames
    (several filter + batch rounds per call, each round's first frames read
    the ring the previous round left) and a 20-frame hold (ties)."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    if scratch_frames is not None:
        monkeypatch.setenv("DIPS_WINDOW_BATCH_FRAMES", str(scratch_frames))
    params = (True, window, 5.0, 0, chroma)
    for (w, h), pieces in [((40, 21), [30]), ((64, 48), [9, 4, 17])]:
        frames = (_tie_frames if window % 2 else _frames)(w, h, 30, 300 + window)
        frames[20] = frames[19]
        want = _oracle_callbacks(frames, params)
        cs = ComputeState(True, window, 5.0, DiPsFilter.Sigmoid, ChromaFilter(chroma))
        try:
            outs, s = [], 0
            for k in pieces:
                outs.append(cs.frame_callback_batch(w, h, frames[s:s + k]))
                s += k
        finally:
            cs.close()
        got = np.concatenate(outs)
        assert np.array_equal(got, want), ((w, h), pieces, np.argwhere(got != want)[:4])


def test_frame_callback_batch_multi_chunk_and_mixed_calls():
    """A small frame (4 tiles) over 150 frames runs as ~10 frame chunks (the
    second ring set and the chunk-start rebuild from HBM); per-frame calls
    before and after a batch see the same ComputeState."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h = 64, 32
    frames = _frames(w, h, 180, 77)
    params = (True, 1, 5.0, 0, 0)
    want = _oracle_callbacks(frames, params)
    cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    try:
        got = [frame_callback(w, h, frames[t], cs) for t in range(9)]
        got += list(cs.frame_callback_batch(w, h, frames[9:159]))
        got += [frame_callback(w, h, frames[t], cs) for t in range(159, 165)]
        got += list(cs.frame_callback_batch(w, h, frames[165:]))
    finally:
        cs.close()
    assert np.array_equal(np.stack(got), want)


def test_frame_callback_batch_device_4k():
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    w, h, n = 3840, 2160, 24
    dev = torch.empty((n, h, w, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    try:
        op.synth_device(dev, w, h, 0xD1B5, 0)
    finally:
        op.close()
    out = torch.empty_like(dev)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    try:
        cs.frame_callback_batch_device(dev, out)
        torch.cuda.synchronize()
        host = dev.cpu().numpy()
        got = out.cpu().numpy()
    finally:
        cs.close()
    ref = oracle.ComputeState(False, 1, 5.0, 255, 0)
    for t in range(10):
        assert np.array_equal(oracle.frame_callback(w, h, host[t], ref), got[t]), t
    cs2 = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    try:
        assert np.array_equal(cs2.frame_callback_batch(w, h, host), got)
    finally:
        cs2.close()


@pytest.mark.parametrize("pieces", [[5, 56], [1, 2, 58], [61], [9, 9, 9, 34]])
def test_frame_callback_batch_host_feed_chunks(pieces):
    """The host-pointer batch is fed through the pipelined upload / kernel /
    download in chunks of at most a quarter of the call's batch (two in
    flight; host_stream.h feed_chunk_frames); calls of 1 to 61 frames (ragged
    last chunks, the warm-up frames split over calls) give the oracle's
    outputs."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    w, h = 64, 48
    frames = _frames(w, h, 61, 5 + len(pieces))
    params = (True, 1, 5.0, 0, 0)
    want = _oracle_callbacks(frames, params)
    cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    try:
        bounds = np.cumsum([0] + pieces)
        got = np.concatenate([cs.frame_callback_batch(w, h, frames[a:b]) for a, b in zip(bounds[:-1], bounds[1:])])
    finally:
        cs.close()
    assert np.array_equal(got, want), np.argwhere(got != want)[:4]


# frame shapes of the per-frame pipeline (host_stream.h piece_bytes /
# DirectGeom): 40 x 200 -- 5 row stripes of 50 (the first 12); 41 x 157 (odd
# row bytes) -- 5 stripes, the last ragged; 16 x 8 -- one stripe
STRIPE_SHAPES = [(40, 200), (41, 157), (16, 8)]


@pytest.mark.parametrize("colorize,sens,filt,chroma", [(False, 5.0, 255, 0), (True, 5.0, 0, 0), (True, 0.7, 1, 2)])
@pytest.mark.parametrize("shape", STRIPE_SHAPES)
@pytest.mark.parametrize("crosscheck", [False, True])
def test_frame_callback_striped_matches_oracle(colorize, sens, filt, chroma, shape, crosscheck):
    """Steady-state frame_callback goes through the zero-copy striped path
    (the copy pool packs each row stripe into pinned memory, the kernel reads
    it over PCIe and writes the output keys back, stripes alternating over
    two streams) or, with DIPS_FLAG_CROSSCHECK, through add_texture +
    dispatch with whole-frame DMA transfers; with several ragged stripes or
    one, every output and the ring state equal the oracle's add_texture +
    dispatch."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h = shape
    frames = _frames(w, h, 16, 90 + filt)
    cs = ComputeState(colorize, 1, sens, DiPsFilter(filt), ChromaFilter(chroma), crosscheck=crosscheck)
    ref = oracle.ComputeState(colorize, 1, sens, filt, chroma)
    try:
        for k in range(16):
            got = frame_callback(w, h, frames[k], cs)
            want = oracle.frame_callback(w, h, frames[k], ref)
            assert np.array_equal(got, want), (k, np.argwhere(got != want)[:4])
        # per-call add_texture / dispatch after striped calls see the same ring
        cs.add_texture(w, h, frames[3])
        ref.add_texture(w, h, frames[3])
        assert np.array_equal(cs.dispatch(), ref.dispatch())
    finally:
        cs.close()


@pytest.mark.parametrize("colorize,sens,filt,chroma", [(False, 5.0, 255, 0), (True, 5.0, 0, 1), (True, 0.7, 1, 3)])
def test_resume_matches_continuous_run(colorize, sens, filt, chroma):
    """dips_compat_resume (frame-range sharding): a ComputeState resumed at
    global frame t0 from the start texture and the raw frames t0-3..t0-1
    gives the outputs of one ComputeState that saw every frame -- host and
    device pointers, batch and per-frame calls, several t0."""
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h, n = 64, 36, 60
    frames = _frames(w, h, n, 300 + filt)
    params = (colorize, 1, sens, DiPsFilter(filt), ChromaFilter(chroma))
    want = _oracle_callbacks(frames, (colorize, 1, sens, filt, chroma))
    a = ComputeState(*params)
    try:
        assert np.array_equal(a.frame_callback_batch(w, h, frames), want)
        start = a.start_texture()
    finally:
        a.close()
    for t0 in (7, 8, 33):
        b = ComputeState(*params)
        try:
            b.resume(w, h, start, frames[t0 - 3:t0], t0)
            got = np.concatenate([b.frame_callback_batch(w, h, frames[t0:t0 + 20]),
                                  np.stack([frame_callback(w, h, f, b) for f in frames[t0 + 20:]])])
            assert np.array_equal(got, want[t0:]), (t0, np.argwhere(got != want[t0:])[:4])
            # device twin
            dev = torch.from_numpy(frames).cuda()
            out = torch.empty_like(dev[t0:])
            b.resume_device(torch.from_numpy(start).cuda(), dev[t0 - 3:t0].contiguous(), t0)
            b.frame_callback_batch_device(dev[t0:].contiguous(), out)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), want[t0:]), t0
        finally:
            b.close()


@pytest.mark.parametrize("window", [2, 3, 5, 8, 11])
def test_resume_window_matches_continuous_run(window):
    """dips_compat_resume with a spatial window: the halo frames are filtered
    into the ring (compat_filter_frames), then batch and per-frame calls
    continue exactly like one ComputeState that saw every frame."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h, n = 48, 36, 40
    frames = _frames(w, h, n, 700 + window)
    params = (True, window, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    want = _oracle_callbacks(frames, (True, window, 5.0, 0, 0))
    a = ComputeState(*params)
    try:
        assert np.array_equal(a.frame_callback_batch(w, h, frames), want)
        start = a.start_texture()
    finally:
        a.close()
    for t0 in (7, 22):
        b = ComputeState(*params)
        try:
            b.resume(w, h, start, frames[t0 - 3:t0], t0)
            got = np.concatenate([b.frame_callback_batch(w, h, frames[t0:t0 + 12]),
                                  np.stack([frame_callback(w, h, f, b) for f in frames[t0 + 12:]])])
            assert np.array_equal(got, want[t0:]), (t0, np.argwhere(got != want[t0:])[:4])
        finally:
            b.close()


@pytest.mark.parametrize("window", [1, 3])
def test_resume_after_deferred_add_texture(window):
    """dips_compat_resume on a handle whose last call was a deferred
    add_texture (W = 1: its speculative stripes -- 5 of them at 96 x 64 --
    still in flight on two streams): resume waits for them before rewriting
    the ring, so the resumed handle gives the outputs of a fresh resumed one
    (ADVICE r2)."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h, n = 96, 64, 30
    frames = _frames(w, h, n, 900 + window)
    params = (True, window, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    want = _oracle_callbacks(frames, (True, window, 5.0, 0, 0))
    a = ComputeState(*params)
    try:
        assert np.array_equal(a.frame_callback_batch(w, h, frames[:12]), want[:12])
        start = a.start_texture()
        a.add_texture(w, h, frames[12])  # deferred: no dispatch follows
        t0 = 17
        a.resume(w, h, start, frames[t0 - 3:t0], t0)
        got = np.stack([frame_callback(w, h, f, a) for f in frames[t0:]])
        assert np.array_equal(got, want[t0:]), np.argwhere(got != want[t0:])[:4]
    finally:
        a.close()


def test_resume_rejects_bad_arguments():
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    from dips_amd._lib import DipsError
    w, h = 16, 8
    f = _frames(w, h, 8, 1)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    try:
        with pytest.raises(DipsError):
            cs.resume(w, h, f[0], f[:3], 6)  # t0 < 7: the ring is not in steady state
        with pytest.raises(ValueError):
            cs.resume(w, h, f[0], f[:2], 9)  # halo must be 3 frames
    finally:
        cs.close()


def test_handles_on_concurrent_threads():
    """The ABI's threading contract: a handle is not internally synchronised,
    but distinct handles may be driven from different threads at the same
    time (ctypes drops the GIL during the calls; the staging copies share
    one process-wide pool).  Four threads, each with its own ComputeState /
    DiPsCompute, per-frame and batch calls, outputs equal to the oracle."""
    import threading
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    from dips_amd.alt import DiPsCompute
    w, h, n = 256, 192, 14  # 5 stripes per frame: the copy pool runs
    clips = [_frames(w, h, n, 500 + k) for k in range(4)]
    results, errors = {}, []

    def compat_worker(k):
        try:
            cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
            try:
                got = [frame_callback(w, h, f, cs) for f in clips[k][:9]]
                got += list(cs.frame_callback_batch(w, h, clips[k][9:]))
            finally:
                cs.close()
            results[k] = np.stack(got)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    def alt_worker(k):
        try:
            c = DiPsCompute(2, h, w)
            try:
                got = [c.send_frame(f, True if t == 2 else None) for t, f in enumerate(clips[k][:6])]
                got += list(c.send_frames(clips[k][6:]))
            finally:
                c.close()
            results[k] = np.stack(got)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    threads = [threading.Thread(target=compat_worker if k % 2 == 0 else alt_worker, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    for k in (0, 2):
        assert np.array_equal(results[k], _oracle_callbacks(clips[k], (True, 1, 5.0, 0, 0))), k
    for k in (1, 3):
        ref = oracle.AltCompute(2, w, h)
        want = np.stack([ref.send_frame(f, t == 2) for t, f in enumerate(clips[k])])
        assert np.array_equal(results[k], want), k


@pytest.mark.parametrize("colorize", [False, True])
@pytest.mark.parametrize("filt", [0, 1, 255])
@pytest.mark.parametrize("sens", [5.0, -3.0, 0.0, 200.0, 1e-30])
def test_batch_epilogue_table_equals_arithmetic_and_oracle(colorize, filt, sens):
    """compat_batch_lut_kernel (the epilogue as a 65536-entry (S, m) table in
    LDS, the default) against compat_batch_kernel (the per-pixel arithmetic,
    DIPS_FLAG_CROSSCHECK) and the oracle, on random frames that reach many (S, m)
    pairs, for every filter, negative / zero / huge / tiny sensitivities (the
    inverse sigmoid's inf and NaN texels included) and both colour modes."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    w, h, n = 96, 64, 30
    frames = _frames(w, h, n, 1234 + filt)
    frames[15] = frames[14]
    params = (colorize, 1, sens, filt, 0)
    want = _oracle_callbacks(frames, params)
    outs = {}
    for xc in (False, True):
        cs = ComputeState(colorize, 1, sens, DiPsFilter(filt), ChromaFilter.None_, crosscheck=xc)
        try:
            outs[xc] = cs.frame_callback_batch(w, h, frames)
        finally:
            cs.close()
    assert np.array_equal(outs[False], outs[True]), np.argwhere(outs[False] != outs[True])[:4]
    assert np.array_equal(outs[False], want), np.argwhere(outs[False] != want)[:4]


@pytest.mark.parametrize("crosscheck", [False, True])
@pytest.mark.parametrize("colorize,sens,filt,chroma,window", [(False, 5.0, 255, 0, 1), (True, 0.7, 0, 3, 1),
                                                             (False, 5.0, 255, 0, 4), (True, 5.0, 1, 2, 7)])
def test_deferred_add_texture_sequences_match_oracle(crosscheck, colorize, sens, filt, chroma, window):
    """add_texture in steady state (host frame) stages the frame and starts
    the dispatch that normally follows on it (zero-copy; W > 1: upload,
    spatial filter, then the main kernel); that dispatch collects it, every
    other call first lets it finish and keeps the slot raw.  Mixed call sequences -- add + dispatch,
    two adds without a dispatch, dispatch twice, add then start_texture, add
    then a striped frame_callback, add then a host batch -- give the oracle's
    outputs and ring state, with the deferral on and off (DIPS_FLAG_CROSSCHECK:
    no deferral, no zero-copy stripes).  44 x 61 frames: 4 ragged stripes."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h = 44, 61
    frames = _frames(w, h, 40, 140 + filt)
    cs = ComputeState(colorize, window, sens, DiPsFilter(filt), ChromaFilter(chroma), crosscheck=crosscheck)
    ref = oracle.ComputeState(colorize, window, sens, filt, chroma)
    t = 0

    def add():
        nonlocal t
        cs.add_texture(w, h, frames[t])
        ref.add_texture(w, h, frames[t])
        t += 1

    def disp(tag):
        got, want = cs.dispatch(), ref.dispatch()
        assert (got is None) == (want is None), tag
        if want is not None:
            assert np.array_equal(got, want), (tag, t, np.argwhere(got != want)[:4])

    try:
        for _ in range(6):  # warm-up phase and first steady frames
            add()
            disp("warm")
        for _ in range(3):
            add()
            disp("add+dispatch")
        add()
        add()  # two adds: the first deferred frame is flushed into its slot
        disp("add,add,dispatch")
        add()
        disp("dispatch 1")
        disp("dispatch twice")
        add()
        assert np.array_equal(cs.start_texture(), ref.start_texture())
        disp("after start_texture")
        add()
        got = frame_callback(w, h, frames[t], cs)  # striped call right after a deferred add
        want = oracle.frame_callback(w, h, frames[t], ref)
        t += 1
        assert np.array_equal(got, want), ("frame_callback after add", t)
        disp("dispatch after callback")
        add()
        got = cs.frame_callback_batch(w, h, frames[t:t + 5])
        want = np.stack([oracle.frame_callback(w, h, frames[t + k], ref) for k in range(5)])
        t += 5
        assert np.array_equal(got, want), ("batch after add", np.argwhere(got != want)[:4])
        add()
        add()  # two raw slots in the ring the batch reads: its first frames go one by one
        got = cs.frame_callback_batch(w, h, frames[t:t + 6])
        want = np.stack([oracle.frame_callback(w, h, frames[t + k], ref) for k in range(6)])
        t += 6
        assert np.array_equal(got, want), ("batch after two adds", np.argwhere(got != want)[:4])
        for _ in range(4):
            add()
            disp("tail")
    finally:
        cs.close()


@pytest.mark.parametrize("window", [1, 3])
def test_deferred_add_texture_across_stream_switches(window):
    """dips_set_stream between calls: before an add_texture (the speculative
    dispatch runs on the new stream) and between an add_texture and its
    dispatch (the switch first lets the speculative kernels finish; the
    dispatch then computes from the raw slot) -- outputs equal the oracle's."""
    import ctypes
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    w, h = 52, 37
    frames = _frames(w, h, 18, 400 + window)
    cs = ComputeState(True, window, 2.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    ref = oracle.ComputeState(True, window, 2.0, 0, 0)
    lib, hd = cs._hd._lib, cs._hd
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        for t in range(18):
            if t == 9:
                hd.check(lib.dips_set_stream(hd.ptr, ctypes.c_void_p(int(s1.cuda_stream))))
            cs.add_texture(w, h, frames[t])
            ref.add_texture(w, h, frames[t])
            if t == 12:
                hd.check(lib.dips_set_stream(hd.ptr, ctypes.c_void_p(int(s2.cuda_stream))))
            if t == 15:
                hd.check(lib.dips_set_stream(hd.ptr, None))  # back to the handle's own stream
            got, want = cs.dispatch(), ref.dispatch()
            assert (got is None) == (want is None), t
            if want is not None:
                assert np.array_equal(got, want), (t, np.argwhere(got != want)[:4])
    finally:
        cs.close()
