"""GPU parity tests of the batch difference series (HIP, through the C ABI)
against the CPU oracle (oracle/dips_oracle.c) on the same seeded inputs.

Bar: bit-exact for SAD, SJ, count, SI_fixed and the |F-R| byte map; the f64
intensity sum within 1e-6 relative of the oracle's sequential f64 sum."""
import itertools

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

SI_RTOL = 1e-6


def _frames(c, w, h, n, seed, kind):
    if kind == "synth":
        return oracle.synth(c, w, h, seed, 0, n)
    rng = np.random.default_rng(seed)
    shape = (n, h, w) if c == 1 else (n, h, w, c)
    f = rng.integers(0, 256, shape, dtype=np.uint8)
    if n > 2:
        f[2] = f[1]  # an exact repeat -> zero row in per-frame mode
    return f


def _check(got, want_out4, want_si, got_map=None, want_map=None):
    arr = got.as_array()
    assert np.array_equal(arr, want_out4), (arr, want_out4)
    np.testing.assert_allclose(got.si, want_si, rtol=SI_RTOL, atol=1e-9)
    if want_map is not None:
        assert np.array_equal(got_map, want_map)


FAST_SHAPES = [(64, 48), (128, 8)]     # pixels % 16 == 0 -> fast kernel
GENERIC_SHAPES = [(37, 23), (1, 1), (5, 3)]


@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("shape", FAST_SHAPES + GENERIC_SHAPES)
def test_series_matches_oracle(c, mode, shape):
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h = shape
    for chroma, tau, kind in itertools.product([0, 2] if c != 1 else [0], [0.0, 8 / 255], ["synth", "random"]):
        frames = _frames(c, w, h, 7, 11 + chroma, kind)
        op = DiffSeriesOperator(PixelFormat(c), Mode(mode), tau, chroma)
        try:
            got, gmap = op(frames, want_map=True)
            got_nomap, _ = op(frames)
        finally:
            op.close()
        out4, si, dmap = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, want_map=True)
        _check(got, out4, si, gmap, dmap)
        _check(got_nomap, out4, si)


@pytest.mark.parametrize("c", [3, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("chroma", [1, 3])
@pytest.mark.parametrize("tau", [0.0, 8 / 255])
def test_series_chroma_red_blue(c, mode, chroma, tau):
    """series_v2_kernel<C, CH=1|3, ...> (chroma Red / Blue, dips_shader.wgsl:
    64-72) with and without a threshold, with and without the byte map, on
    the fast shapes, the ragged generic shapes and the generic kernel forced
    on a fast shape -- every instantiation against the oracle."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    for (w, h), generic in [((64, 48), False), ((128, 8), False), ((37, 23), False), ((64, 48), True)]:
        for kind in ("synth", "random"):
            frames = _frames(c, w, h, 9, 70 + chroma, kind)
            op = DiffSeriesOperator(PixelFormat(c), Mode(mode), tau, chroma, force_generic=generic)
            try:
                got, gmap = op(frames, want_map=True)
                got_nomap, _ = op(frames)
            finally:
                op.close()
            out4, si, dmap = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, want_map=True)
            _check(got, out4, si, gmap, dmap)
            _check(got_nomap, out4, si)


@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
def test_series_explicit_ref(c, mode):
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    frames = _frames(c, 64, 32, 5, 3, "synth")
    ref = _frames(c, 64, 32, 1, 99, "random")[0]
    op = DiffSeriesOperator(PixelFormat(c), Mode(mode), 0.0, 0)
    try:
        got, _ = op(frames, ref=ref)
    finally:
        op.close()
    out4, si, _ = oracle.series(frames, mode=mode, ref=ref)
    _check(got, out4, si)


@pytest.mark.parametrize("c", [1, 3, 4])
def test_fast_equals_generic(c):
    from dips_amd import diff_series, Mode, PixelFormat
    frames = _frames(c, 256, 64, 9, 5, "synth")
    for mode in (Mode.Overall, Mode.PerFrame):
        a, am = diff_series(frames, fmt=PixelFormat(c), mode=mode, tau=3 / 255, want_map=True)
        b, bm = diff_series(frames, fmt=PixelFormat(c), mode=mode, tau=3 / 255, want_map=True,
                            force_generic=True)
        assert np.array_equal(a.as_array(), b.as_array())
        assert np.array_equal(am, bm)


def test_single_pixel_known_answer():
    """one pixel (0,0,0) -> (255,255,255): SJ = 510, SI = 1.0."""
    from dips_amd import diff_series, PixelFormat
    for w, h in [(64, 48), (7, 5)]:
        f = np.zeros((2, h, w, 3), dtype=np.uint8)
        f[1, h // 2, w // 3] = 255
        s, _ = diff_series(f, fmt=PixelFormat.RGB8)
        assert list(s.sj) == [0, 510]
        assert list(s.sad) == [0, 765]
        assert list(s.count) == [0, 1]
        assert s.si[1] == 1.0


def test_identical_frames_zero():
    from dips_amd import diff_series, PixelFormat, Mode
    f = np.repeat(oracle.synth(3, 64, 48, 1, 0, 1), 6, axis=0)
    for mode in (Mode.Overall, Mode.PerFrame):
        s, m = diff_series(f, fmt=PixelFormat.RGB8, mode=mode, want_map=True)
        assert not s.as_array().any()
        assert not m.any()


def test_streamed_equals_batch():
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    frames = _frames(3, 64, 48, 23, 7, "synth")
    ref = _frames(3, 64, 48, 1, 8, "random")[0]
    for mode in (Mode.Overall, Mode.PerFrame):
        op = DiffSeriesOperator(PixelFormat.RGB8, mode, 1 / 255, 0)
        try:
            for chunk in (1, 4, 5, 0):
                for r in (None, ref):
                    a = op.streamed(frames, ref=r, chunk_frames=chunk)
                    out4, _, _ = oracle.series(frames, mode=int(mode), tau=1 / 255, ref=r)
                    assert np.array_equal(a.as_array(), out4), (mode, chunk, r is None)
        finally:
            op.close()


@pytest.mark.parametrize("c", [1, 3, 4])
def test_synth_device_bit_exact(c):
    import torch
    from dips_amd import DiffSeriesOperator, PixelFormat
    w, h, n, t0 = 61, 37, 5, 1234
    shape = (n, h, w) if c == 1 else (n, h, w, c)
    dst = torch.empty(shape, dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat(c))
    try:
        op.synth_device(dst, w, h, 0xD1B5, t0)
        torch.cuda.synchronize()
    finally:
        op.close()
    want = oracle.synth(c, w, h, 0xD1B5, t0, n)
    assert np.array_equal(dst.cpu().numpy(), want)


def test_8k_threshold_config_matches_oracle():
    """BASELINE.json configs[4]: 7680x4320 RGB8, the f32 intensity path with
    a threshold (tau = 8/255), overall and per-frame, against the oracle."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n = 7680, 4320, 4
    dev = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
    for mode in (Mode.Overall, Mode.PerFrame):
        op = DiffSeriesOperator(PixelFormat.RGB8, mode, 8 / 255, 0)
        try:
            op.synth_device(dev, w, h, 0xD1B5, 9996)
            ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            op.run_device(dev, ser)
            torch.cuda.synchronize()
            host = dev.cpu().numpy()
            out4, si, _ = oracle.series(host, mode=int(mode), tau=8 / 255, nthreads=8)
            got = ser.cpu().numpy().view(np.uint64)
            assert np.array_equal(got, out4)
            np.testing.assert_allclose(np.ldexp(got[:, 3].astype(np.float64), -32), si, rtol=SI_RTOL)
        finally:
            op.close()


def test_1080p_overall_full_batch_properties():
    """BASELINE.json configs[1] at full size (1920x1080 RGB8, 1000 frames,
    'overall'): the series of the whole batch equals the concatenation of two
    half batches against the same reference (frame 0) and of a per-frame run
    whose reference is the halo frame; frame 0's entry is zero; the first
    frames equal the oracle."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n = 1920, 1080, 1000
    dev = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.Overall, 8 / 255, 0)
    pf = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, 0)
    try:
        op.synth_device(dev, w, h, 0xD1B5, 0)
        full = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        op.run_device(dev, full)
        a = torch.zeros((500, 4), dtype=torch.int64, device="cuda")
        b = torch.zeros((500, 4), dtype=torch.int64, device="cuda")
        op.run_device(dev[:500], a, ref=dev[0])
        op.run_device(dev[500:], b, ref=dev[0])
        p_full = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        p_half = torch.zeros((500, 4), dtype=torch.int64, device="cuda")
        pf.run_device(dev, p_full)
        pf.run_device(dev[500:], p_half, ref=dev[499])
        torch.cuda.synchronize()
        assert torch.equal(full, torch.cat([a, b]))
        assert torch.equal(p_full[500:], p_half)
        assert not full[0].any() and not p_full[0].any()
        host = dev[:3].cpu().numpy()
        out4, _, _ = oracle.series(host, mode=0, tau=8 / 255, nthreads=8)
        assert np.array_equal(full[:3].cpu().numpy().view(np.uint64), out4)
    finally:
        op.close()
        pf.close()


def test_device_path_matches_host_path():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n = 3840, 2160, 6
    for mode in (Mode.Overall, Mode.PerFrame):
        op = DiffSeriesOperator(PixelFormat.RGB8, mode, 8 / 255, 0)
        try:
            dev = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
            op.synth_device(dev, w, h, 0xD1B5, 100)
            ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            op.run_device(dev, ser)
            torch.cuda.synchronize()
            host = dev.cpu().numpy()
            out4, si, _ = oracle.series(host, mode=int(mode), tau=8 / 255, nthreads=8)
            got = ser.cpu().numpy().view(np.uint64)
            assert np.array_equal(got, out4)
        finally:
            op.close()


@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
def test_long_batch_segments_match_oracle(c, mode):
    """A small frame over thousands of frames: every resident wave walks a
    multi-frame segment (the unrolled 4-frame ring, the tail and segments
    that start mid-tile or cross into the next tile), the last tile is
    ragged.  Every frame's entry and the full byte map equal the oracle."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h = 80, 36  # 2880 px: 2.8 RGB tiles of 1024 px, 1.4 gray tiles of 2048 px
    n = 20011 if c == 1 else 8009
    frames = _frames(c, w, h, n, 40 + c + mode, "random")
    for chroma, tau in ([(0, 8 / 255), (1, 0.0), (3, 8 / 255), (1, 8 / 255)] if c != 1
                        else [(0, 8 / 255), (0, 0.0)]):
        op = DiffSeriesOperator(PixelFormat(c), Mode(mode), tau, chroma)
        try:
            got, gmap = op(frames, want_map=True)
            got_nomap, _ = op(frames)
        finally:
            op.close()
        out4, si, dmap = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, want_map=True, nthreads=8)
        _check(got, out4, si, gmap, dmap)
        _check(got_nomap, out4, si)


def test_wave_cap_same_series(monkeypatch):
    """DIPS_SERIES_WAVES_PER_SIMD (a deployment cap; nothing sets it by
    default) only changes how the (tile, frame) items are split over waves:
    same series, fewer waves."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n = 640, 360, 300
    dev = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
    out = []
    for cap in (None, "3", "1"):
        if cap is None:
            monkeypatch.delenv("DIPS_SERIES_WAVES_PER_SIMD", raising=False)
        else:
            monkeypatch.setenv("DIPS_SERIES_WAVES_PER_SIMD", cap)
        op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, 0)
        try:
            op.synth_device(dev, w, h, 0xD1B5, 0)
            ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            op.run_device(dev, ser)
            torch.cuda.synchronize()
            waves, _, _ = op.geometry(w, h, n)
            out.append((waves, ser.cpu().numpy()))
        finally:
            op.close()
    assert out[0][0] > out[1][0] > out[2][0]
    assert all(np.array_equal(out[0][1], o[1]) for o in out[1:])


def test_config0_gray8_full_clip_matches_oracle():
    """BASELINE.json configs[0] at its full size: 640x480 gray8, the
    300-frame synthetic clip, 'overall' mode (tau 0 and 8/255), through the
    HIP path (host and device pointers) against the oracle, every entry and
    the whole byte map bit-exact."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n = 640, 480, 300
    frames = oracle.synth(1, w, h, 0xD1B5, 0, n)
    dev = torch.from_numpy(frames).cuda()
    for tau in (0.0, 8 / 255):
        out4, si, dmap = oracle.series(frames, mode=0, tau=tau, want_map=True, nthreads=8)
        op = DiffSeriesOperator(PixelFormat.Gray8, Mode.Overall, tau)
        try:
            got, gmap = op(frames, want_map=True)
            ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            op.run_device(dev, ser)
            torch.cuda.synchronize()
        finally:
            op.close()
        _check(got, out4, si, gmap, dmap)
        assert np.array_equal(ser.cpu().numpy().view(np.uint64), out4)


RAGGED_SHAPES = [(37, 23), (5, 3), (1, 1), (641, 3), (17, 1)]


@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("with_map", [True, False])
@pytest.mark.parametrize("offsets", [(0, 0, 0), (1, 2, 3), (3, 1, 2), (2, 3, 1)])
def test_unaligned_device_batches(c, mode, offsets, with_map):
    """The vectorised kernel on frame batches, references and maps at byte
    offsets 1-3 from an aligned address and with ragged pixel counts (frame
    strides that are not a multiple of 4, < pixels_per_vec trailing pixels
    per frame handled by the generic kernel) -- against the oracle.  These
    shapes ran entirely on series_generic_kernel before (4 % of 8 TB/s,
    profiles/r02_fallback_rate_before.jsonl)."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fo, ro, mo = offsets
    # (RGB8 / RGBA8 frames off a 4-byte boundary -- an offset batch, or an
    # RGB8 stride W*H*3 that is not a multiple of 4 such as (62, 33)'s 6138
    # -- run the aligned-load kernel, series_v2.hip ALIGN; the reference at
    # its own offset gets its own funnel shift)
    for (w, h) in [(64, 48), (62, 33)] + RAGGED_SHAPES:
        for tau, chroma in [(0.0, 0), (8 / 255, 0 if c == 1 else 2)]:
            n = 9
            frames = _frames(c, w, h, n, 5 + w, "random" if w % 2 else "synth")
            ref = _frames(c, w, h, 1, 77, "random")[0]
            fb = frames[0].size
            dev = torch.device("cuda")
            fbuf = torch.zeros(n * fb + 8, dtype=torch.uint8, device=dev)
            rbuf = torch.zeros(fb + 8, dtype=torch.uint8, device=dev)
            mbuf = torch.full((n * fb + 8,), 0xA5, dtype=torch.uint8, device=dev)
            fdev = fbuf[fo:fo + n * fb].view(frames.shape)
            fdev.copy_(torch.from_numpy(frames))
            rdev = rbuf[ro:ro + fb].view(ref.shape)
            rdev.copy_(torch.from_numpy(ref))
            mdev = mbuf[mo:mo + n * fb].view(frames.shape)
            series = torch.zeros((n, 4), dtype=torch.int64, device=dev)
            op = DiffSeriesOperator(PixelFormat(c), Mode(mode), tau, chroma)
            try:
                op.run_device(fdev, series, ref=rdev if mode == 0 else None, map_out=mdev if with_map else None)
                torch.cuda.synchronize()
            finally:
                op.close()
            out4, _, dmap = oracle.series(frames, mode=mode, chroma=chroma, tau=tau,
                                          ref=ref if mode == 0 else None, want_map=True)
            got = series.cpu().numpy().view(np.uint64)
            assert np.array_equal(got, out4), ((w, h), tau, got, out4)
            if not with_map:
                continue
            m = mbuf.cpu().numpy()
            assert np.array_equal(m[mo:mo + n * fb].reshape(frames.shape), dmap), (w, h)
            # nothing written outside the map
            assert (m[:mo] == 0xA5).all() and (m[mo + n * fb:] == 0xA5).all()


GRAY_FORMS = [dict(), dict(gray_table="band"), dict(gray_table="pair"), dict(crosscheck=True)]


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("tau", [0.0, 1 / 255, 8 / 255, 0.5, 1.0])
def test_gray_kernels_agree(mode, tau):
    """GRAY8 on the table kernel (layout chosen per workgroup from the content,
    the default), its two tables pinned (DIPS_FLAG_GRAY_BAND_TABLE: keyed by
    (a ^ b, a) with the band clamp; _PAIR_TABLE: keyed by (a, b)) and the f32
    series_fast_kernel (DIPS_FLAG_CROSSCHECK), with and without the map,
    against the oracle -- random and synthetic frames, ragged shape included."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    for (w, h), kind in [((256, 64), "random"), ((640, 48), "synth"), ((37, 23), "random")]:
        frames = _frames(1, w, h, 9, 40 + w, kind)
        out4, si, dmap = oracle.series(frames, mode=mode, tau=tau, want_map=True)
        for form in GRAY_FORMS:
            op = DiffSeriesOperator(PixelFormat.Gray8, Mode(mode), tau, **form)
            try:
                got, gmap = op(frames, want_map=True)
                got_nomap, _ = op(frames)
            finally:
                op.close()
            _check(got, out4, si, gmap, dmap)
            _check(got_nomap, out4, si)


@pytest.mark.parametrize("table", ["band", "pair", "auto"])
@pytest.mark.parametrize("tau", [0.0, 1 / 255, 8 / 255, 0.1, 0.5, 1.0])
def test_gray_table_every_byte_pair(tau, table):
    """Every (frame byte a, reference byte b) through each GRAY8 table (band:
    keyed by (a ^ b, a), indices below the band clamp raised to it; pair:
    keyed by (a, b), swizzled; auto: per workgroup), against the oracle:
    'overall' against a reference with b = x; frame t = 1..256 holds a = t - 1
    everywhere (so each a value is its own series entry), frame 257 holds
    a = y (all 65,536 pairs in one frame); plus a flat low-noise clip (the
    content that piles LDS reads onto few banks without a swizzle, and nearly
    all inside the band) and a clip whose frames alternate between one flat
    frame and random ones (a = const against varying b)."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    x = np.arange(256, dtype=np.uint8)
    frames = np.empty((258, 256, 256), dtype=np.uint8)
    frames[0] = x[None, :]
    frames[1:257] = x[:, None, None]
    frames[257] = x[:, None]
    rng = np.random.default_rng(11)
    flat = np.clip(128 + rng.integers(-3, 4, (12, 64, 512)), 0, 255).astype(np.uint8)
    alt = rng.integers(0, 256, (9, 32, 256), dtype=np.uint8)
    alt[::2] = 77
    bw = np.zeros((7, 64, 256), dtype=np.uint8)
    bw[1::2] = 255  # every pixel dI = 1: the largest per-lane sums
    for fr, mode in ((frames, 0), (frames, 1), (flat, 1), (alt, 1), (alt, 0), (bw, 1)):
        out4, si, _ = oracle.series(fr, mode=mode, tau=tau)
        op = DiffSeriesOperator(PixelFormat.Gray8, Mode(mode), tau, gray_table=table)
        try:
            got, _ = op(fr)
        finally:
            op.close()
        _check(got, out4, si)


@pytest.mark.parametrize("c", [1, 3])
def test_stream_switch_orders_shared_scratch(c):
    """Back-to-back batches on two different streams through one operator,
    no synchronisation in between: the handle's partial records and tables
    are shared, so dips_set_stream orders the second stream after the first
    (both series must equal the oracle's)."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n = 640, 480, 24
    fa = _frames(c, w, h, n, 301, "random")
    fb = _frames(c, w, h, n, 302, "synth")
    want = [oracle.series(f, mode=1, tau=8 / 255)[0] for f in (fa, fb)]
    op = DiffSeriesOperator(PixelFormat(c), Mode.PerFrame, 8 / 255)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        da, db = torch.from_numpy(fa).cuda(), torch.from_numpy(fb).cuda()
        torch.cuda.synchronize()
        outs = []
        for rep in range(3):
            sa = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            sb = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            with torch.cuda.stream(s1):
                op.run_device(da, sa)
            with torch.cuda.stream(s2):
                op.run_device(db, sb)
            outs.append((sa, sb))
        torch.cuda.synchronize()
        for sa, sb in outs:
            assert np.array_equal(sa.cpu().numpy().view(np.uint64), want[0])
            assert np.array_equal(sb.cpu().numpy().view(np.uint64), want[1])
    finally:
        op.close()


def test_device_calls_ordered_with_torch_default_stream():
    """torch's default stream is stream 0 (cuda_stream 0), which the wrappers
    pass as NULL = the handle's own stream; that stream is a blocking one, so
    library work and torch work on the default stream are ordered both ways
    with no synchronisation in between (round 3: with a non-blocking own
    stream a torch read right after synth_device saw stale frames)."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    assert torch.cuda.current_stream().cuda_stream == 0
    W, H, n = 3840, 2160, 48
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255)
    try:
        fr = torch.zeros((n, H, W, 3), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        op.synth_device(fr, W, H, 0xD1B5, 0)
        racy = fr[n - 1].to(torch.int64).sum()  # torch kernel right behind the library's
        torch.cuda.synchronize()
        assert int(racy) == int(fr[n - 1].to(torch.int64).sum())
        # the other way: a torch fill, then the series kernel reading it at once
        fr.fill_(3)
        fr[1:].fill_(200)
        ser = torch.full((n, 4), -1, dtype=torch.int64, device="cuda")
        op.run_device(fr, ser)
        torch.cuda.synchronize()
        assert int(ser[1, 0]) == W * H * 3 * 197 and int(ser[2, 0]) == 0
    finally:
        op.close()


@pytest.mark.parametrize("crosscheck", [False, True])
@pytest.mark.parametrize("c", [3, 4])
@pytest.mark.parametrize("mode", [0, 1])
def test_series_intensity_sum_forms_match_oracle(crosscheck, c, mode):
    """The two intensity-sum forms of series_v2 (ISI = 1, the integer sum
    with a threshold select, the default for tau >= 2^-5; ISI = 0, the exact
    f64 sum, DIPS_FLAG_CROSSCHECK) against the oracle for tau at and above
    2^-5 up to 1.0: synthetic and random clips, black / white frames (every
    pixel dI = 1: the largest per-lane sums), identical frames, a ragged shape
    and an offset (aligned-load) batch, with and without the map."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    bw = np.zeros((6, 32, 96, c), dtype=np.uint8)
    bw[1::2] = 255
    same = np.repeat(_frames(c, 96, 32, 1, 5, "random"), 4, axis=0)
    clips = [_frames(c, 256, 64, 9, 31, "synth"), _frames(c, 256, 64, 9, 32, "random"), bw, same,
             _frames(c, 1000, 37, 6, 33, "random")]
    below_one = float(np.nextafter(np.float32(1), np.float32(0)))
    for tau in (1 / 32, 8 / 255, 0.3, below_one, 1.0):
        for chroma in (0, 2):
            op = DiffSeriesOperator(PixelFormat(c), Mode(mode), tau, chroma, crosscheck=crosscheck)
            try:
                for fr in clips:
                    out4, si, dmap = oracle.series(fr, mode=mode, chroma=chroma, tau=tau, want_map=True)
                    got, gmap = op(fr, want_map=True)
                    _check(got, out4, si, gmap, dmap)
                    got, _ = op(fr)
                    _check(got, out4, si)
                # frames off a 4-byte boundary: the aligned-load form
                import torch
                for fr, off in ((clips[0], 1 if c == 3 else 3), (clips[2], 2)):
                    buf = torch.empty(fr.nbytes + 8, dtype=torch.uint8, device="cuda")
                    dev = buf[off:off + fr.nbytes].view(fr.shape)
                    dev.copy_(torch.from_numpy(fr))
                    ser = torch.zeros((fr.shape[0], 4), dtype=torch.int64, device="cuda")
                    op.run_device(dev, ser)
                    torch.cuda.synchronize()
                    out4, _, _ = oracle.series(fr, mode=mode, chroma=chroma, tau=tau)
                    assert np.array_equal(ser.cpu().numpy().view(np.uint64), out4), (crosscheck, tau, chroma, off)
            finally:
                op.close()


def _split_series(op, dev, parts, ref=None, map_out=None):
    """The series of `dev` as consecutive batches of < 256 frames each (the
    contiguous schedule; part_geometry applies from 256 frames), each against
    its own reference: 'overall' the given one, 'per-frame' the frame before
    the batch."""
    import torch
    from dips_amd import Mode
    n = dev.shape[0]
    out = torch.zeros((n, 4), dtype=torch.int64, device=dev.device)
    bounds = np.linspace(0, n, parts + 1).astype(int)
    for a, b in zip(bounds[:-1], bounds[1:]):
        assert b - a < 256
        r = ref if op.mode == Mode.Overall else (dev[a - 1] if a > 0 else None)
        op.run_device(dev[a:b], out[a:b], ref=r, map_out=None if map_out is None else map_out[a:b])
    return out


@pytest.mark.parametrize("mode", [0, 1])
def test_4k_forms_agree_and_match_oracle(mode):
    """At the bench's full frame size (4K), the forms of the two series
    kernels give the same series over a 48-frame batch (a size-independent
    property): GRAY8 auto = band table = pair table = f32 kernel, RGB8 ISI = 1
    (integer sum) = ISI = 0 (f64, DIPS_FLAG_CROSSCHECK); the first 4 frames of
    each against the oracle."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    w, h, n, tau = 3840, 2160, 48, 8 / 255
    for fmt, forms in ((PixelFormat.Gray8, GRAY_FORMS), (PixelFormat.RGB8, [dict(), dict(crosscheck=True)])):
        c = int(fmt)
        shape = (n, h, w) if c == 1 else (n, h, w, c)
        dev = torch.empty(shape, dtype=torch.uint8, device="cuda")
        got = []
        for k, form in enumerate(forms):
            op = DiffSeriesOperator(fmt, Mode(mode), tau, 0, **form)
            try:
                if k == 0:
                    op.synth_device(dev, w, h, 0xD1B5, 7)
                ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
                op.run_device(dev, ser)
                torch.cuda.synchronize()
                got.append(ser.cpu().numpy().view(np.uint64))
            finally:
                op.close()
        for k in range(1, len(forms)):
            assert np.array_equal(got[k], got[0]), (fmt, forms[k])
        head = dev[:4].cpu().numpy()
        out4, _, _ = oracle.series(head, mode=mode, tau=tau, nthreads=8)
        assert np.array_equal(got[0][:4], out4), fmt


@pytest.mark.parametrize("fmt_name,w,h,n", [("RGB8", 1920, 1080, 523), ("RGBA8", 1920, 1080, 525),
                                             ("Gray8", 2048, 1536, 1000)])
def test_part_major_schedule_matches_contiguous_and_oracle(fmt_name, w, h, n):
    """'Per-frame' batches of >= 256 frames run the part-major schedule
    (series_abi.hip part_geometry; series_v2.hip / series_gray.hip item loop).
    These shapes take it on a 256-CU MI355X: 1080p RGB8 4 parts of 131
    frames (the last 130), RGBA8 4 parts of 132 (the last 129), 2048x1536
    gray8 7 parts of 143 (the last 142), so items start mid-batch, segments
    end in 0- to 3-frame tails and the last part is short.  The series (and
    the |F - R| map for RGB8) must equal the contiguous schedule's -- the same
    frames as batches of < 256, each against the frame before it -- bit for
    bit, and every frame must match the oracle."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fmt = getattr(PixelFormat, fmt_name)
    c, tau = int(fmt), 8 / 255
    shape = (n, h, w) if c == 1 else (n, h, w, c)
    want_map = c == 3
    op = DiffSeriesOperator(fmt, Mode.PerFrame, tau, 0)
    try:
        dev = torch.empty(shape, dtype=torch.uint8, device="cuda")
        op.synth_device(dev, w, h, 0xA11CE, 3)
        ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        dmap = torch.empty_like(dev) if want_map else None
        op.run_device(dev, ser, map_out=dmap)
        cmap = torch.empty_like(dev) if want_map else None
        cser = _split_series(op, dev, 5 if n < 1000 else 8, map_out=cmap)
        torch.cuda.synchronize()
        got = ser.cpu().numpy().view(np.uint64)
        assert np.array_equal(got, cser.cpu().numpy().view(np.uint64))
        if want_map:
            assert torch.equal(dmap, cmap)
        frames = dev.cpu().numpy()
        out4, _, omap = oracle.series(frames, mode=1, tau=tau, want_map=want_map, nthreads=16)
        bad = np.nonzero(~np.all(got == out4, axis=1))[0]
        assert bad.size == 0, f"frames differing from the oracle: {bad[:10]}"
        if want_map:
            assert np.array_equal(dmap.cpu().numpy(), omap)
    finally:
        op.close()


@pytest.mark.parametrize("table", ["band", "pair", "auto"])
@pytest.mark.parametrize("mode", [0, 1])
def test_gray_auto_layout_branches_match_oracle(table, mode):
    """GRAY8 table layout 4 (the default): one kernel whose workgroups each
    take layout 5 (band clamp) or layout 2 from a sample of their own first
    items; DIPS_FLAG_GRAY_BAND_TABLE / _PAIR_TABLE pin one branch -- every
    branch against the oracle on synthetic, random, identical and ragged
    clips, tau 0 / 8/255 / 0.5, with and without the map, one-frame batches
    included."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    same = np.repeat(_frames(1, 256, 64, 1, 9, "random"), 5, axis=0)
    clips = [_frames(1, 256, 64, 9, 41, "synth"), _frames(1, 256, 64, 9, 42, "random"), same,
             _frames(1, 1000, 37, 6, 43, "random"), _frames(1, 512, 32, 1, 44, "synth")]
    for tau in (0.0, 8 / 255, 0.5):
        op = DiffSeriesOperator(PixelFormat.Gray8, Mode(mode), tau, 0, gray_table=table)
        try:
            for fr in clips:
                out4, si, dmap = oracle.series(fr, mode=mode, tau=tau, want_map=True)
                got, gmap = op(fr, want_map=True)
                _check(got, out4, si, gmap, dmap)
                got, _ = op(fr)
                _check(got, out4, si)
        finally:
            op.close()


@pytest.mark.parametrize("mode,n", [(0, 40), (1, 300)])
def test_gray_auto_mixed_content_per_workgroup(mode, n):
    """Layout 4 decides per workgroup, so one launch can run both tables: a
    2048 x 512 clip whose row bands are flat noise (128 +- 3: layout 2),
    slowly varying synthetic content and i.i.d. random bytes, 'overall' (40
    frames, contiguous ranges) and 'per-frame' (300 frames, the part-major
    schedule) -- every frame and the map equal to the oracle."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    rng = np.random.default_rng(77 + mode)
    w, h = 2048, 512
    fr = oracle.synth(1, w, h, 0xD1B5, 0, n)
    fr[:, :128] = (128 + rng.integers(-3, 4, (n, 128, w))).astype(np.uint8)
    fr[:, 384:] = rng.integers(0, 256, (n, 128, w), dtype=np.uint8)
    op = DiffSeriesOperator(PixelFormat.Gray8, Mode(mode), 8 / 255, 0)
    try:
        out4, si, dmap = oracle.series(fr, mode=mode, tau=8 / 255, want_map=True, nthreads=8)
        got, gmap = op(fr, want_map=True)
        _check(got, out4, si, gmap, dmap)
    finally:
        op.close()


@pytest.mark.parametrize("fmt_name,form", [("RGB8", {}), ("RGBA8", {}), ("Gray8", {}),
                                           ("Gray8", {"crosscheck": True}), ("RGB8", {"force_generic": True})])
def test_series_starts_from_zero_on_a_dirty_buffer(fmt_name, form):
    """The RGB(A) and GRAY8 table kernels clear the caller's series
    themselves (SeriesArgs::zero, no fill launch); the f32 GRAY8 kernel
    (DIPS_FLAG_CROSSCHECK) and the generic kernel after a fill.  A series
    tensor full of garbage, twice in a row, must come out equal to the oracle
    -- at 300 frames (part-major, the adaptive reduce grid) and 3 frames."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fmt = getattr(PixelFormat, fmt_name)
    c = int(fmt)
    for n, w, h in ((300, 256, 96), (3, 640, 480)):
        frames = _frames(c, w, h, n, 5 + n, "synth")
        want, _, _ = oracle.series(frames, mode=1, tau=8 / 255, nthreads=8)
        op = DiffSeriesOperator(fmt, Mode.PerFrame, 8 / 255, 0, **form)
        try:
            dev = torch.from_numpy(frames).cuda()
            ser = torch.full((n, 4), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
            for _ in range(2):
                op.run_device(dev, ser)
                torch.cuda.synchronize()
                assert np.array_equal(ser.cpu().numpy().view(np.uint64), want), (fmt_name, form, n)
                ser.fill_(-1)
        finally:
            op.close()


@pytest.mark.parametrize("fmt_name,n", [("RGB8", 1), ("RGB8", 3), ("Gray8", 2), ("RGBA8", 2)])
def test_reduce_grid_for_few_large_frames(fmt_name, n):
    """Few 8K frames: the reduce kernel takes 8 tiles per thread (one round of
    loads) over a grid of up to 4,050 groups in y (series_kernels.hip
    launch_series_reduce), the main kernel clears the series -- every frame
    equal to the oracle, both modes."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fmt = getattr(PixelFormat, fmt_name)
    c = int(fmt)
    frames = _frames(c, 7680, 4320, n, 90 + n, "synth")
    dev = torch.from_numpy(frames).cuda()
    for mode in (0, 1):
        want, _, _ = oracle.series(frames, mode=mode, tau=8 / 255, nthreads=8)
        op = DiffSeriesOperator(fmt, Mode(mode), 8 / 255, 0)
        try:
            ser = torch.full((n, 4), -1, dtype=torch.int64, device="cuda")
            op.run_device(dev, ser)
            torch.cuda.synchronize()
            assert np.array_equal(ser.cpu().numpy().view(np.uint64), want), (fmt_name, n, mode)
        finally:
            op.close()


@pytest.mark.parametrize("fmt_name,w,h,n", [("RGB8", 1920, 1080, 523), ("RGBA8", 1920, 1080, 525)])
def test_part_major_overall_matches_contiguous_and_oracle(fmt_name, w, h, n):
    """'Overall' batches on the part-major schedule (each item loads the
    fixed reference tile at its part's first frame) -- series and map equal
    to the contiguous schedule's (the same frames as batches of < 256 against
    the same reference) and every frame equal to the oracle."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fmt = getattr(PixelFormat, fmt_name)
    c, tau = int(fmt), 8 / 255
    op = DiffSeriesOperator(fmt, Mode.Overall, tau, 0)
    try:
        dev = torch.empty((n, h, w, c), dtype=torch.uint8, device="cuda")
        op.synth_device(dev, w, h, 0xB0B, 11)
        ref = dev[0].clone()
        ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        dmap = torch.empty_like(dev)
        op.run_device(dev, ser, ref=ref, map_out=dmap)
        cmap = torch.empty_like(dev)
        cser = _split_series(op, dev, 5, ref=ref, map_out=cmap)
        torch.cuda.synchronize()
        got = ser.cpu().numpy().view(np.uint64)
        assert np.array_equal(got, cser.cpu().numpy().view(np.uint64))
        assert torch.equal(dmap, cmap)
        out4, _, _ = oracle.series(dev.cpu().numpy(), mode=0, tau=tau, ref=ref.cpu().numpy(), nthreads=16)
        bad = np.nonzero(~np.all(got == out4, axis=1))[0]
        assert bad.size == 0, f"frames differing from the oracle: {bad[:10]}"
    finally:
        op.close()
