"""Seeded randomized parity test of the batch difference series (HIP, through
the C ABI) against the CPU oracle (oracle/dips_oracle.c).

The hand-listed tests in test_gpu_series.py pin each kernel form on chosen
shapes; this one draws the combinations instead -- pixel format, mode,
chroma, tau, frame shape, batch length, content kind, byte offsets of the
frames / reference / map, map on or off, host or device entry point -- so
that interactions between the kernel selections (fast / generic tail,
aligned-load RGB8, integer intensity sum for tau >= 2^-5, part-major
schedule for >= 256 frames, GRAY8 band table) are covered without being
enumerated.  tau is drawn from uniform f32 values and from the edges where
the selection or the threshold compare changes: 0, k/255 and its f32
neighbours (achievable gray differences), 2^-5 and its neighbours, 1.

Reference semantics: /root/reference/dips/src/gpu/shaders/dips_shader.wgsl
:64-82 (get_intensity), :185-240 (threshold, |F-R| map); the series itself
is the north star's per-frame statistic.  Bar: SAD, SJ,
count, SI_fixed and the map bit-exact; the host entry point's f64 SI within
1e-6 relative (test_gpu_series.SI_RTOL).  Run once with its fixed seed.
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

SEED = 0xD1F5
N_CASES = 400
SI_RTOL = 1e-6


def _f32(x):
    return float(np.float32(x))


def _draw_tau(rng):
    kind = rng.integers(0, 5)
    if kind == 0:
        return _f32(rng.random())
    if kind == 1:
        k = int(rng.integers(0, 256))
        t = np.float32(k / 255)
        return float(np.nextafter(t, np.float32(rng.choice([0, 2]))) if rng.random() < 0.5 else t)
    if kind == 2:
        t = np.float32(1 / 32)
        return float(rng.choice([t, np.nextafter(t, np.float32(0)), np.nextafter(t, np.float32(1))]))
    if kind == 3:
        return float(rng.choice([0.0, 1.0, _f32(8 / 255), _f32(1e-7)]))
    return _f32(rng.random() * 0.05)


def _draw_shape(rng):
    kind = rng.integers(0, 4)
    if kind == 0:  # whole vecs
        return int(rng.integers(1, 9)) * 16, int(rng.integers(1, 9))
    if kind == 1:  # ragged
        return int(rng.integers(1, 200)), int(rng.integers(1, 12))
    if kind == 2:  # single row / column
        return (int(rng.integers(1, 700)), 1) if rng.random() < 0.5 else (1, int(rng.integers(1, 300)))
    return int(rng.integers(60, 260)), int(rng.integers(20, 70))


def _content(rng, c, w, h, n):
    shape = (n, h, w) if c == 1 else (n, h, w, c)
    kind = rng.integers(0, 4)
    if kind == 0:
        return rng.integers(0, 256, shape, dtype=np.uint8)
    if kind == 1:
        return oracle.synth(c, w, h, int(rng.integers(0, 1 << 30)), int(rng.integers(0, 1000)), n)
    if kind == 2:  # a slowly varying clip: small temporal differences (band-dense for GRAY8)
        base = rng.integers(0, 256, shape[1:], dtype=np.int16)
        steps = rng.integers(-3, 4, shape, dtype=np.int16).cumsum(axis=0)
        return np.clip(base[None] + steps, 0, 255).astype(np.uint8)
    # sparse changes: repeated frames with a few pixels rewritten, extremes included
    f = np.repeat(rng.integers(0, 256, (1,) + shape[1:], dtype=np.uint8), n, axis=0)
    for t in range(1, n):
        m = rng.random(shape[1:]) < 0.05
        f[t][m] = rng.choice(np.array([0, 255, 1, 254, 128], dtype=np.uint8), size=int(m.sum()))
    return f


def test_random_series_cases_match_oracle():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat

    rng = np.random.default_rng(SEED)
    dev = torch.device("cuda")
    for case in range(N_CASES):
        c = int(rng.choice([1, 3, 4]))
        mode = int(rng.integers(0, 2))
        chroma = 0 if c == 1 else int(rng.integers(0, 4))
        tau = _draw_tau(rng)
        w, h = _draw_shape(rng)
        n = int(rng.integers(1, 12)) if rng.random() < 0.9 else int(rng.integers(250, 300))
        frames = _content(rng, c, w, h, n)
        explicit_ref = mode == 0 and rng.random() < 0.5
        ref = _content(rng, c, w, h, 1)[0] if explicit_ref else None
        with_map = bool(rng.random() < 0.5)
        host = bool(rng.random() < 0.3)
        offs = [int(x) for x in rng.integers(0, 4, 3)] if rng.random() < 0.5 else [0, 0, 0]
        what = dict(case=case, c=c, mode=mode, chroma=chroma, tau=tau, w=w, h=h, n=n,
                    explicit_ref=explicit_ref, with_map=with_map, host=host, offs=offs)

        out4, si, dmap = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, ref=ref, want_map=True)
        op = DiffSeriesOperator(PixelFormat(c), Mode(mode), tau, chroma)
        try:
            if host:
                got, gmap = op(frames, ref=ref, want_map=with_map)
                assert np.array_equal(got.as_array(), out4), what
                np.testing.assert_allclose(got.si, si, rtol=SI_RTOL, atol=1e-9, err_msg=str(what))
                if with_map:
                    assert np.array_equal(gmap, dmap), what
                continue
            fo, ro, mo = offs
            fb = frames[0].size
            nb = frames.nbytes
            fbuf = torch.zeros(nb + 8, dtype=torch.uint8, device=dev)
            fdev = fbuf[fo:fo + nb].view(frames.shape)
            fdev.copy_(torch.from_numpy(frames))
            rdev = None
            if ref is not None:
                rbuf = torch.zeros(fb + 8, dtype=torch.uint8, device=dev)
                rdev = rbuf[ro:ro + fb].view(ref.shape)
                rdev.copy_(torch.from_numpy(ref))
            mbuf = mdev = None
            if with_map:
                mbuf = torch.full((nb + 8,), 0xA5, dtype=torch.uint8, device=dev)
                mdev = mbuf[mo:mo + nb].view(frames.shape)
            series = torch.full((n, 4), -1, dtype=torch.int64, device=dev)
            op.run_device(fdev, series, ref=rdev, map_out=mdev)
            torch.cuda.synchronize()
            got = series.cpu().numpy().view(np.uint64)
            assert np.array_equal(got, out4), (what, got, out4)
            if with_map:
                m = mbuf.cpu().numpy()
                assert np.array_equal(m[mo:mo + nb].reshape(frames.shape), dmap), what
                assert (m[:mo] == 0xA5).all() and (m[mo + nb:] == 0xA5).all(), what
        finally:
            op.close()


def _alt_props(colorize, window, scalar, filt, chroma):
    from dips_amd.alt import ChromaFilter, DiPsProperties
    return DiPsProperties(colorize=colorize, window_size=window, sigmoid_horizontal_scalar=scalar,
                          filter_type=filt, chroma_filter=ChromaFilter(chroma))


def _alt_scalar(rng):
    kind = rng.integers(0, 4)
    if kind == 0:
        return _f32(rng.uniform(-20, 20))
    if kind == 1:
        return _f32(rng.uniform(0.01, 12))
    if kind == 2:
        return float(rng.choice([0.0, 5.0, 1.0, -1.0, 160.0, 161.0, 500.0, 1e-6]))
    return _f32(np.exp(rng.uniform(-8, 8)))


ALT_CASES = 150


def test_random_alt_runs_match_oracle():
    """dips_alt's loop (dips_alt/src/lib.rs:588-683 over
    dips_compute/mod.rs:498-646) on drawn parameters -- texture count,
    window, filter, colour, chroma, sigmoid scalar (the epilogue table and the
    arithmetic epilogue's |k| <= 160 range both crossed), frame shape,
    snapshot markers and the split of the clip into calls -- against the
    oracle's twin, RGBA8 outputs bit-exact."""
    from dips_amd.alt import DiPsRunner

    rng = np.random.default_rng(SEED + 1)
    for case in range(ALT_CASES):
        n_tex = int(rng.choice([1, 2, 2, 3, 4, 16]))
        window = int(rng.choice([1, 1, 1, 2, 3, 4, 5, 6]))
        filt = int(rng.choice([0, 1, 255]))
        colorize = bool(rng.random() < 0.5)
        chroma = int(rng.integers(0, 4))
        scalar = _alt_scalar(rng)
        w, h = int(rng.integers(1, 72)), int(rng.integers(1, 40))
        n = int(rng.integers(4, 28))
        shape = (n, h, w, 4)
        kind = rng.integers(0, 3)
        if kind == 0:
            frames = rng.integers(0, 256, shape, dtype=np.uint8)
        elif kind == 1:  # few distinct values: ties in every window
            frames = np.array([0, 1, 2, 128, 254, 255], dtype=np.uint8)[rng.integers(0, 6, shape)]
        else:  # slowly varying clip
            base = rng.integers(0, 256, shape[1:], dtype=np.int16)
            frames = np.clip(base[None] + rng.integers(-4, 5, shape, dtype=np.int16).cumsum(axis=0),
                             0, 255).astype(np.uint8)
        markers = sorted({int(x) for x in rng.integers(0, n, int(rng.integers(0, 4)))})
        cuts = sorted({int(x) for x in rng.integers(1, n, int(rng.integers(0, 3)))})
        pieces = np.diff([0] + cuts + [n]).tolist()
        what = dict(case=case, n_tex=n_tex, window=window, filt=filt, colorize=colorize, chroma=chroma,
                    scalar=scalar, w=w, h=h, n=n, markers=markers, pieces=pieces)
        want = oracle.AltCompute(n_tex, w, h, colorize, window, scalar, filt, chroma).run(frames, markers)
        r = DiPsRunner(h, w, _alt_props(colorize, window, scalar, filt, chroma), markers, num_textures=n_tex)
        try:
            outs, s = [], 0
            for k in pieces:
                outs.append(r(frames[s:s + k]))
                s += k
        finally:
            r.close()
        got = np.concatenate(outs)
        assert np.array_equal(got, want), (what, np.argwhere(got != want)[:4])


COMPAT_CASES = 60
COMPAT_OPS = 40


def test_random_compute_state_properties_match_oracle():
    """dips-compat ComputeState (dips/src/gpu/mod.rs:170-397, lib.rs:233-246)
    on drawn properties -- colour, window 1-6, sigmoid scalar, filter, chroma
    -- and frame shapes, each case a short random sequence of add_texture /
    dispatch / frame_callback / frame_callback_batch / start_texture against
    the oracle's ComputeState, every output bit-exact.  (The interleaving
    surface with streams and resume is test_gpu_sequence.py's, on fixed
    properties.)"""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback

    rng = np.random.default_rng(SEED + 2)
    for case in range(COMPAT_CASES):
        colorize = bool(rng.random() < 0.5)
        window = int(rng.choice([1, 1, 2, 3, 4, 5, 6]))
        scalar = _alt_scalar(rng)
        filt = int(rng.choice([0, 1, 255]))
        chroma = int(rng.integers(0, 4))
        w, h = int(rng.integers(1, 90)), int(rng.integers(1, 50))
        what = dict(case=case, colorize=colorize, window=window, scalar=scalar, filt=filt, chroma=chroma, w=w, h=h)
        gpu = ComputeState(colorize, window, scalar, DiPsFilter(filt), ChromaFilter(chroma))
        ora = oracle.ComputeState(colorize, window, scalar, filt, chroma)
        levels = rng.integers(0, 256, int(rng.integers(2, 7)), dtype=np.uint8) if rng.random() < 0.3 else None

        def frame():
            if levels is not None:  # few distinct bytes: ties in the temporal and spatial medians
                return levels[rng.integers(0, levels.size, (h, w, 4))]
            return rng.integers(0, 256, (h, w, 4), dtype=np.uint8)

        try:
            for i in range(COMPAT_OPS):
                op = rng.choice(["add", "dispatch", "callback", "batch", "start"], p=[0.3, 0.25, 0.2, 0.15, 0.1])
                where = (what, i, op)
                if op == "add":
                    f = frame()
                    gpu.add_texture(w, h, f)
                    ora.add_texture(w, h, f)
                elif op == "dispatch":
                    a, b = gpu.dispatch(), ora.dispatch()
                    assert (a is None) == (b is None), where
                    if b is not None:
                        assert np.array_equal(a, b), (where, np.argwhere(a != b)[:4])
                elif op == "callback":
                    f = frame()
                    a = frame_callback(w, h, f, gpu)
                    b = oracle.frame_callback(w, h, f, ora)
                    assert np.array_equal(a, b), (where, np.argwhere(a != b)[:4])
                elif op == "batch":
                    fr = np.stack([frame() for _ in range(int(rng.integers(1, 6)))])
                    a = gpu.frame_callback_batch(w, h, fr)
                    b = np.stack([oracle.frame_callback(w, h, f, ora) for f in fr])
                    assert np.array_equal(a, b), (where, np.argwhere(a != b)[:4])
                else:
                    a, b = gpu.start_texture(), ora.start_texture()
                    assert (a is None) == (b is None), where
                    if b is not None:
                        assert np.array_equal(a, b), where
        finally:
            gpu.close()
