"""GPU parity tests of the dips_alt operator (DiPsCompute.send_frame and the
run_dips_on_file loop, dips_alt/src/dips_compute/mod.rs:498-646,
dips_alt/src/lib.rs:588-683) against the CPU oracle's twin: bit-exact RGBA8
outputs and snapshot texture for every parameter combination, on the
per-frame kernel (any N, any window) and the batch kernel (N = 2, W = 1)."""
import itertools

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _frames(w, h, n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    if n > 5:
        f[5] = f[4]
    return f


def _props(colorize, window, scalar, filt, chroma):
    from dips_amd.alt import ChromaFilter, DiPsProperties
    return DiPsProperties(colorize=colorize, window_size=window, sigmoid_horizontal_scalar=scalar,
                          filter_type=filt, chroma_filter=ChromaFilter(chroma))


SEND_PARAMS = [(n, w, f, c, ch) for (n, w), f, c, ch in itertools.product(
    [(2, 1), (1, 1), (3, 1), (16, 1), (2, 2), (2, 3), (2, 5), (4, 7), (2, 11)], [0, 1, 255], [False, True], [0, 2])]


@pytest.mark.parametrize("n_tex,window,filt,colorize,chroma", SEND_PARAMS)
def test_send_frame_matches_oracle(n_tex, window, filt, colorize, chroma):
    from dips_amd.alt import DiPsCompute
    w, h = (37, 21) if window > 1 else (40, 17)
    frames = _frames(w, h, 9, 5 + n_tex + window)
    gpu = DiPsCompute(n_tex, h, w, _props(colorize, window, 3.0, filt, chroma))
    ref = oracle.AltCompute(n_tex, w, h, colorize, window, 3.0, filt, chroma)
    try:
        for t in range(9):
            snap = t in (2, 6)
            a = gpu.send_frame(frames[t], () if snap else None)
            b = ref.send_frame(frames[t], snap)
            assert np.array_equal(a, b), (t, np.argwhere(a != b)[:4])
            if t == 6:  # the snapshot frame's output is the stored gray texture
                assert np.array_equal(gpu.snapshot_texture(), b[..., 0])
    finally:
        gpu.close()


@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("window", list(range(2, 12)))
def test_send_frame_every_window_matches_oracle(window, ties):
    """dips_alt spatial filter (W^2 sort, pre_compute_shader.wgsl:141-184) for
    every window 2..11 on a ragged 53x29 frame; `ties` draws the bytes from
    five values so most windows hold equal intensities."""
    from dips_amd.alt import DiPsCompute
    w, h = 53, 29
    rng = np.random.default_rng(200 + window)
    if ties:
        frames = np.array([0, 1, 2, 128, 255], dtype=np.uint8)[rng.integers(0, 5, (5, h, w, 4))]
    else:
        frames = rng.integers(0, 256, (5, h, w, 4), dtype=np.uint8)
    gpu = DiPsCompute(3, h, w, _props(True, window, 3.0, 255, 0))
    ref = oracle.AltCompute(3, w, h, True, window, 3.0, 255, 0)
    try:
        for t in range(5):
            a = gpu.send_frame(frames[t], () if t == 1 else None)
            b = ref.send_frame(frames[t], t == 1)
            assert np.array_equal(a, b), (t, np.argwhere(a != b)[:4])
    finally:
        gpu.close()


BATCH_SHAPES = [(64, 48), (40, 17), (37, 21), (3, 1)]  # npx % 4 == 0 -> batch kernel; else per-frame


@pytest.mark.parametrize("shape", BATCH_SHAPES)
@pytest.mark.parametrize("filt,colorize,chroma", list(itertools.product([0, 1, 255], [False, True], [0, 1, 3])))
def test_run_matches_oracle(shape, filt, colorize, chroma):
    from dips_amd.alt import DiPsRunner
    w, h = shape
    frames = _frames(w, h, 40, 17 + filt + chroma)
    markers = [5, 6, 19, 33]
    r = DiPsRunner(h, w, _props(colorize, 1, 4.0, filt, chroma), markers)
    try:
        got = r(frames)
    finally:
        r.close()
    want = oracle.AltCompute(2, w, h, colorize, 1, 4.0, filt, chroma).run(frames, markers)
    assert np.array_equal(got, want), np.argwhere(got != want)[:4]


@pytest.mark.parametrize("n_tex,window", [(2, 1), (2, 3), (3, 1), (16, 2)])
def test_run_pieces_equal_one_call(n_tex, window):
    """The loop state (texture slots, snapshot, index) carries across calls:
    feeding the clip in pieces gives the outputs of one call and of the
    oracle."""
    from dips_amd.alt import DiPsRunner
    w, h = 32, 24
    frames = _frames(w, h, 60, 3 + n_tex)
    markers = [4, 20, 21, 45]
    want = oracle.AltCompute(n_tex, w, h, True, window, 5.0, 0, 0).run(frames, markers)
    for pieces in ([60], [1, 1, 1, 57], [2, 17, 5, 36], [29, 31]):
        r = DiPsRunner(h, w, _props(True, window, 5.0, 0, 0), markers, num_textures=n_tex)
        try:
            outs, s = [], 0
            for k in pieces:
                outs.append(r(frames[s:s + k]))
                s += k
        finally:
            r.close()
        got = np.concatenate(outs)
        assert np.array_equal(got, want), (pieces, np.argwhere(got != want)[:4])


@pytest.mark.parametrize("scratch_frames", [None, 5])
@pytest.mark.parametrize("window", list(range(2, 12)))
def test_run_window_batch_matches_oracle(window, scratch_frames, monkeypatch):
    """N = 2, W > 1 through the prefiltered batch path (alt_filter_frames_kernel
    + the batch kernel on f32 intensities): every window 2..11, refresh
    markers (a snapshot at a chunk's first frame included), split calls and a
    5-frame scratch (several filter + batch rounds per call)."""
    from dips_amd.alt import ChromaFilter, DiPsRunner
    if scratch_frames is not None:
        monkeypatch.setenv("DIPS_WINDOW_BATCH_FRAMES", str(scratch_frames))
    for (w, h), pieces, chroma in [((40, 17), [30], 0), ((64, 48), [9, 4, 17], 2)]:
        frames = _frames(w, h, 30, 40 + window)
        frames[20] = frames[19]
        markers = [4, 11, 12, 26]
        want = oracle.AltCompute(2, w, h, True, window, 5.0, 0, chroma).run(frames, markers)
        r = DiPsRunner(h, w, _props(True, window, 5.0, 0, chroma), markers)
        try:
            outs, s = [], 0
            for k in pieces:
                outs.append(r(frames[s:s + k]))
                s += k
        finally:
            r.close()
        got = np.concatenate(outs)
        assert np.array_equal(got, want), ((w, h), pieces, np.argwhere(got != want)[:4])


@pytest.mark.parametrize("window", [2, 5, 11])
def test_window_batch_equals_per_frame_kernel(window):
    """W > 1: the prefiltered batch path and the per-frame kernel agree over a
    clip cut into several frame chunks (chunk starts rebuild the previous
    intensities and snapshots from the filtered buffer)."""
    from dips_amd.alt import DiPsCompute
    w, h = 64, 32
    frames = _frames(w, h, 150, 19 + window)
    flags = np.zeros(150, bool)
    flags[[0, 2, 40, 41, 97, 149]] = True
    outs = []
    for generic in (False, True):
        c = DiPsCompute(2, h, w, _props(False, window, 3.0, 1, 0), force_generic=generic)
        try:
            outs.append(c.send_frames(frames[:70], flags[:70]))
            outs.append(c.send_frames(frames[70:], flags[70:]))
            outs.append(c.snapshot_texture())
        finally:
            c.close()
    for a, b in zip(outs[:3], outs[3:]):
        assert np.array_equal(a, b)


def test_batch_kernel_equals_per_frame_kernel():
    """The N = 2 batch kernel and the generic per-frame kernel agree on a
    clip long enough to be cut into several frame chunks (the chunk start
    rebuilds the previous intensities and the snapshot from HBM)."""
    from dips_amd.alt import DiPsCompute
    w, h = 64, 32
    frames = _frames(w, h, 150, 9)
    flags = np.zeros(150, bool)
    flags[[2, 40, 41, 97, 149]] = True
    outs = []
    for generic in (False, True):
        c = DiPsCompute(2, h, w, _props(True, 1, 5.0, 0, 0), force_generic=generic)
        try:
            outs.append(c.send_frames(frames[:70], flags[:70]))
            outs.append(c.send_frames(frames[70:], flags[70:]))
            outs.append(c.snapshot_texture())
        finally:
            c.close()
    for a, b in zip(outs[:3], outs[3:]):
        assert np.array_equal(a, b)
    ref = oracle.AltCompute(2, w, h, True, 1, 5.0, 0, 0)
    want = np.stack([ref.send_frame(frames[t], bool(flags[t])) for t in range(150)])
    assert np.array_equal(np.concatenate(outs[:2]), want)


def test_identical_frames_known_answer():
    from dips_amd.alt import DiPsRunner
    w, h = 16, 8
    f = np.zeros((h, w, 4), np.uint8)
    f[..., 3] = 255
    f[0, 0, :3] = (10, 20, 31)
    f[0, 1, :3] = (77, 77, 77)
    r = DiPsRunner(h, w, _props(False, 1, 5.0, 255, 0))
    try:
        outs = r(np.repeat(f[None], 6, axis=0))
    finally:
        r.close()
    assert outs[2][0, 0, 0] == 20 and outs[2][0, 1, 0] == 77
    for o in outs[3:]:
        assert o[0, 1, 0] == 128 and o[0, 0, 0] == 129 and (o[..., 3] == 255).all()


def test_device_path_4k():
    """4K RGBA8 resident in HBM: the device-pointer batch equals the oracle on
    the first frames and the host-pointer path on all of them."""
    import torch
    from dips_amd import DiffSeriesOperator, PixelFormat
    from dips_amd.alt import DiPsCompute
    w, h, n = 3840, 2160, 24
    dev = torch.empty((n, h, w, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    try:
        op.synth_device(dev, w, h, 0xD1B5, 0)
    finally:
        op.close()
    out = torch.empty_like(dev)
    flags = [t == 2 for t in range(n)]
    c = DiPsCompute(2, h, w)
    try:
        c.send_frames_device(dev, out, flags)
        torch.cuda.synchronize()
        host = dev.cpu().numpy()
        got = out.cpu().numpy()
        assert np.array_equal(c.send_frames(host, flags), got)
    finally:
        c.close()
    ref = oracle.AltCompute(2, w, h, True, 1, 5.0, 0, 0)
    for t in range(5):
        assert np.array_equal(ref.send_frame(host[t], t == 2), got[t]), t


def test_rejects_bad_input():
    from dips_amd import DipsError
    from dips_amd.alt import DiPsCompute
    with pytest.raises(DipsError):
        DiPsCompute(17, 8, 8)
    c = DiPsCompute(2, 8, 8)
    try:
        with pytest.raises(ValueError):
            c.send_frame(np.zeros((8, 7, 4), np.uint8))
    finally:
        c.close()


@pytest.mark.parametrize("pieces", [[13, 37], [1, 4, 45], [50], [7, 7, 7, 29]])
def test_run_host_feed_chunks(pieces):
    """Host frames go through the pipelined feed in chunks of at most a
    quarter of each call's batch (host_stream.h feed_chunk_frames); calls of
    1 to 50 frames (ragged last chunks, refresh markers and snapshots falling
    on chunk and call edges) give the loop's outputs equal to the oracle's."""
    from dips_amd.alt import DiPsRunner
    w, h = 32, 24
    frames = _frames(w, h, 50, 40 + len(pieces))
    markers = [4, 9, 10, 27, 36]
    want = oracle.AltCompute(2, w, h, True, 1, 5.0, 0, 0).run(frames, markers)
    r = DiPsRunner(h, w, _props(True, 1, 5.0, 0, 0), markers)
    try:
        bounds = np.cumsum([0] + pieces)
        got = np.concatenate([r(frames[a:b]) for a, b in zip(bounds[:-1], bounds[1:])])
    finally:
        r.close()
    assert np.array_equal(got, want), np.argwhere(got != want)[:4]


# frame shapes whose per-frame pipeline cuts several row stripes with a
# ragged last one (host_stream.h piece_bytes / DirectGeom): 40 x 200 -- 5
# stripes of 50 rows (the first 12); 41 x 157 (odd row bytes) -- 5 stripes
STRIPE_SHAPES = [(40, 200), (41, 157)]


@pytest.mark.parametrize("n_tex,filt,colorize", [(2, 0, True), (3, 255, False), (1, 1, True), (16, 0, False)])
@pytest.mark.parametrize("shape", STRIPE_SHAPES)
@pytest.mark.parametrize("crosscheck", [False, True])
def test_send_frame_striped_matches_oracle(n_tex, filt, colorize, shape, crosscheck):
    """send_frame with W = 1 goes through the zero-copy striped path (the
    kernel reads the frame from pinned host memory, stores it into its slot
    and writes the output to pinned host memory, stripes alternating over two
    streams) or, with DIPS_FLAG_CROSSCHECK, whole-frame DMA transfers; with
    several ragged stripes, more frames than slots and snapshots on some
    frames (read back by the frames after them), every output equals the
    oracle's."""
    from dips_amd.alt import DiPsCompute
    w, h = shape
    frames = _frames(w, h, 20, 60 + n_tex)
    snaps = [False, True, False, False, True, False, False, False, False, True, False, False] + [False] * 8
    c = DiPsCompute(n_tex, h, w, _props(colorize, 1, 5.0, filt, 0), crosscheck=crosscheck)
    ref = oracle.AltCompute(n_tex, w, h, colorize, 1, 5.0, filt, 0)
    try:
        for t in range(20):
            got = c.send_frame(frames[t], True if snaps[t] else None)
            want = ref.send_frame(frames[t], snaps[t])
            assert np.array_equal(got, want), (t, np.argwhere(got != want)[:4])
    finally:
        c.close()


@pytest.mark.parametrize("n_tex,markers", [(2, [5, 6, 30]), (3, [4, 17, 18])])
def test_replay_resume_matches_one_loop(n_tex, markers):
    """Frame-range sharding of the dips_alt loop (shard.alt_sharded): a fresh
    DiPsCompute that replays the last snapshot's source frames and the
    N-frame halo, then takes frames t0.. with the loop's flags, gives the
    outputs of one loop over every frame -- host and device pointers."""
    import torch
    from dips_amd import shard
    from dips_amd.alt import DiPsCompute, DiPsRunner, run_loop_flags
    w, h, n = 64, 32, 48
    frames = _frames(w, h, n, 70 + n_tex)
    props = _props(True, 1, 5.0, 0, 0)
    r = DiPsRunner(h, w, props, markers, num_textures=n_tex)
    try:
        want = r(frames)
    finally:
        r.close()
    flags = run_loop_flags(n, markers)
    for t0 in (1, 7, 19, 33):
        need, fl = shard.alt_replay_frames(t0, flags, n_tex)
        c = DiPsCompute(n_tex, h, w, props)
        try:
            if need:
                c.send_frames(frames[need], fl)
            got = c.send_frames(frames[t0:], list(flags[t0:]))
            assert np.array_equal(got, want[t0:]), (t0, np.argwhere(got != want[t0:])[:4])
            dev = torch.from_numpy(frames).cuda()
            if need:
                rep = dev[need].contiguous()
                c.send_frames_device(rep, torch.empty_like(rep), fl)
            out = torch.empty_like(dev[t0:])
            c.send_frames_device(dev[t0:].contiguous(), out, list(flags[t0:]))
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), want[t0:]), t0
        finally:
            c.close()


LUT_SCALARS = [5.0, 1.0, 4.0, 10.0, 0.0, -3.0, 200.0, 1e-30, 1e30]


@pytest.mark.parametrize("filt", [0, 1, 255])
@pytest.mark.parametrize("colorize", [False, True])
def test_lut_selfcheck_exhaustive(filt, colorize):
    """The batch kernel's epilogue table (alt_lut.h) against the
    specification's epilogue for EVERY snapshot byte x (max, min) byte pair
    -- all 2,993 distinct diff values of every chroma mode and of the
    prefiltered path -- on the device, for sensitivities inside and far
    outside the setter's [1, 10] clamp (0, negative, huge, tiny)."""
    from dips_amd.alt import DiPsCompute
    for k in LUT_SCALARS:
        c = DiPsCompute(2, 8, 8, _props(colorize, 1, k, filt, 0))
        try:
            assert c.lut_selfcheck() == 0, (filt, colorize, k)
        finally:
            c.close()


@pytest.mark.parametrize("filt,colorize", list(itertools.product([0, 1, 255], [False, True])))
@pytest.mark.parametrize("window,chroma", [(1, 0), (1, 2), (1, 3), (3, 0), (5, 1)])
def test_batch_lut_equals_arithmetic_and_oracle(filt, colorize, window, chroma):
    """alt_batch_kernel with the epilogue table (default) against its
    per-pixel arithmetic form (DIPS_FLAG_CROSSCHECK) and the oracle's run
    loop, on random frames with snapshots, W = 1 (RGBA8 frames) and W > 1
    (prefiltered intensities)."""
    from dips_amd.alt import DiPsRunner
    w, h = 72, 40
    frames = _frames(w, h, 36, 500 + filt + 7 * chroma + window)
    markers = [4, 5, 20]
    outs = {}
    for xc in (False, True):
        r = DiPsRunner(h, w, _props(colorize, window, 4.0, filt, chroma), markers, crosscheck=xc)
        try:
            outs[xc] = r(frames)
        finally:
            r.close()
    assert np.array_equal(outs[False], outs[True]), np.argwhere(outs[False] != outs[True])[:4]
    want = oracle.AltCompute(2, w, h, colorize, window, 4.0, filt, chroma).run(frames, markers)
    assert np.array_equal(outs[False], want), np.argwhere(outs[False] != want)[:4]


@pytest.mark.parametrize("window", [3, 6])
@pytest.mark.parametrize("crosscheck", [False, True])
@pytest.mark.parametrize("shape", STRIPE_SHAPES)
def test_send_frame_window_stripes_match_oracle(window, crosscheck, shape):
    """send_frame with W > 1: the zero-copy form uploads the stripes into the
    slot by copy kernels, runs the frame kernel on the whole frame and brings
    the output back by copy kernels, stripe by stripe (several ragged stripes
    here); the cross-check form (DIPS_FLAG_CROSSCHECK) moves whole frames by
    DMA.  Every output equals the oracle's, snapshots included."""
    from dips_amd.alt import DiPsCompute
    w, h = shape
    frames = _frames(w, h, 10, 300 + window)
    gpu = DiPsCompute(3, h, w, _props(True, window, 3.0, 0, 0), crosscheck=crosscheck)
    ref = oracle.AltCompute(3, w, h, True, window, 3.0, 0, 0)
    try:
        for t in range(10):
            snap = t in (1, 5)
            a = gpu.send_frame(frames[t], () if snap else None)
            b = ref.send_frame(frames[t], snap)
            assert np.array_equal(a, b), (t, np.argwhere(a != b)[:4])
    finally:
        gpu.close()
