"""CPU tests of the dips_alt operator: the oracle's C
and numpy restatements against each other and against known answers, the
host mirror of DiPsProperties / the command line, and the C-ABI entry points'
argument checks (no GPU compute)."""
import ctypes
import itertools

import numpy as np
import pytest

from dips_amd import _lib
from dips_amd.alt import (ChromaFilter, CliError, DiPsProperties, Encoding, Filter, FRAME_COUNT,
                          parse_args)
from oracle import np_restatement as nr
from oracle import oracle


def _frames(w, h, n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    if n > 5:
        f[5] = f[4]
    return f


# ---------------------------------------------------------------------------
# oracle
# ---------------------------------------------------------------------------

ALT_CASES = [(2, 1), (1, 1), (3, 1), (4, 1), (16, 1), (2, 2), (2, 3), (2, 5), (2, 7), (3, 3), (16, 3),
             (2, 11)]


@pytest.mark.parametrize("n_tex,window", ALT_CASES)
def test_alt_c_equals_numpy(n_tex, window):
    for filt, col, ch in itertools.product([0, 1, 255], [False, True], [0, 3]):
        frames = _frames(11, 7, 9, n_tex * 13 + window)
        a = oracle.AltCompute(n_tex, 11, 7, col, window, 2.5, filt, ch)
        b = nr.AltCompute(n_tex, 11, 7, col, window, 2.5, filt, ch)
        x, y = a.run(frames, [6]), b.run(frames, [6])
        assert np.array_equal(x, y), (filt, col, ch, np.argwhere(x != y)[:4])


def test_alt_temporal_known_answers():
    """A6: the 2-slot "median" is min(a, b); n = 1 gives 0;
    n = 16 is the plain upper median (index 16 clamped)."""
    assert oracle.alt_temporal([0.3, 0.1]) == np.float32(0.1)
    assert oracle.alt_temporal([0.7]) == 0.0
    assert oracle.alt_temporal([0.4, 0.2, 0.9]) == np.float32(0.2)  # sorted({0, .2, .4, .9})[1]
    assert oracle.alt_temporal([0.4, 0.2, 0.9, 0.6]) == np.float32(0.4)
    v = np.arange(16, dtype=np.float32)[::-1] / 16
    assert oracle.alt_temporal(v) == np.float32(0.5)


def test_alt_run_snapshot_schedule():
    """lib.rs:633-670: the snapshot is taken on the third frame and after each
    refresh marker two frames later; the snapshot frame's output is the gray
    min-intensity, every other output is the epilogue of snapshot - min."""
    w, h = 8, 4
    frames = _frames(w, h, 12, 3)
    a = oracle.AltCompute(FRAME_COUNT, w, h, False, 1, 5.0, 255, 0)
    out = a.run(frames, markers=[5])
    # frames 0 and 1: snapshot texture still zero, min(I_0, 0) = 0 -> gray 128
    assert (out[0][..., :3] == 128).all()
    # frame 2 (index == 2) and frame 7 (marker after the 5th frame, then two more)
    b = oracle.AltCompute(FRAME_COUNT, w, h, False, 1, 5.0, 255, 0)
    for t in range(12):
        o = b.send_frame(frames[t], snapshot=t in (2, 7))
        assert np.array_equal(o, out[t]), t


def test_alt_identical_frames_known_answer():
    """Identical frames: after the snapshot, snapshot - min = q(I)/255 - I is
    0 for gray pixels (128 out) and +-1/510 for an odd max+min."""
    w, h = 8, 8
    f = np.zeros((h, w, 4), np.uint8)
    f[..., 3] = 255
    f[0, 0, :3] = (10, 20, 31)  # I*255 = 20.5 -> RNE 20 -> snapshot below I
    f[0, 1, :3] = (77, 77, 77)
    a = oracle.AltCompute(2, w, h, False, 1, 5.0, 255, 0)
    outs = a.run(np.repeat(f[None], 6, axis=0))
    assert outs[2][0, 0, 0] == 20 and outs[2][0, 1, 0] == 77  # snapshot frame: q(min)
    for o in outs[3:]:
        assert o[0, 1, 0] == 128
        assert o[0, 0, 0] == 129  # 0.5 - 5 * 0.5 * (20/255 - 20.5/255) = 0.5049 -> 128.75 -> 129


# ---------------------------------------------------------------------------
# host mirror
# ---------------------------------------------------------------------------

def test_properties_defaults_and_setters():
    """DiPsProperties::default / set_* (dips_alt/src/dips_compute/mod.rs:176-234)."""
    p = DiPsProperties()
    assert (p.colorize, p.window_size, p.sigmoid_horizontal_scalar) == (True, 1, 5.0)
    assert p.filter_type == Filter.Sigmoid and p.chroma_filter == ChromaFilter.All
    p.set_sigmoid_horizontal_scalar(42.0)
    assert p.sigmoid_horizontal_scalar == 10.0
    p.set_sigmoid_horizontal_scalar(0.1)
    assert p.sigmoid_horizontal_scalar == 1.0
    for size, want in [(0, 1), (1, 1), (2, 1), (4, 3), (5, 5), (8, 7), (200, 7)]:
        p.set_window_size(size)
        assert p.window_size == want, size
    assert [int(f) for f in Filter] == [0, 1] and [int(c) for c in ChromaFilter] == [0, 1, 2, 3]
    assert FRAME_COUNT == 2


def test_encoding_fourcc():
    assert Encoding.Uncompressed.as_fourcc() == ord("R") | ord("G") << 8 | ord("B") << 16 | ord("A") << 24
    assert Encoding.H264.value == "H264" and Encoding.Huffman.value == "HFYU"


def test_parse_args_mirrors_main_rs():
    a = parse_args(["--input=in.avi", "--output=out.avi", "--encoding=H264", "--filter=inv_sig",
                    "--chroma=g", "--sig_scalar=20", "--win_size=4", "--colorize=false", "30", "90"])
    assert (a.input_path, a.output_path, a.encoding) == ("in.avi", "out.avi", Encoding.H264)
    p = a.properties
    assert (p.filter_type, p.chroma_filter, p.sigmoid_horizontal_scalar, p.window_size, p.colorize) == (
        Filter.InverseSigmoid, ChromaFilter.Green, 10.0, 3, False)
    assert a.refresh_markers == [30, 90]
    assert parse_args(["--input=a", "--output=b", "--encoding=XVID"]).encoding == Encoding.Uncompressed
    assert parse_args(["--help"]).help
    for bad, msg in [(["--input=a", "--output=b", "--filter=median"], "Invalide Filter Type"),
                     (["--input=a", "--output=b", "--chroma="], "Invalid Chroma Type"),
                     (["--output=b"], "Input file not specified"),
                     (["--input=a"], "Output file not specified"),
                     (["--input=a", "--output=b", "frame7"], "invalid digit"),
                     (["--input=a", "--output=b", "--win_size=-1"], "invalid u8")]:
        with pytest.raises(CliError, match=msg):
            parse_args(bad)


# ---------------------------------------------------------------------------
# C ABI (no compute)
# ---------------------------------------------------------------------------

def test_alt_params_default_matches_reference():
    p = _lib.DipsAltParams()
    assert _lib.load().dips_alt_params_default(ctypes.byref(p)) == 0
    assert (p.colorize, p.window_size, p.filter_type, p.chroma_filter, p.num_textures) == (1, 1, 0, 0, 2)
    assert abs(p.sigmoid_horizontal_scalar - 5.0) < 1e-7


@pytest.mark.parametrize("field,value", [("num_textures", 0), ("num_textures", 17), ("window_size", 0),
                                         ("window_size", 12), ("chroma_filter", 4),
                                         ("sigmoid_horizontal_scalar", float("inf"))])
def test_alt_create_rejects_bad_params(field, value):
    lib = _lib.load()
    p = _lib.DipsAltParams()
    lib.dips_alt_params_default(ctypes.byref(p))
    setattr(p, field, value)
    h = ctypes.c_void_p()
    assert lib.dips_alt_create(ctypes.byref(p), 8, 8, 0, ctypes.byref(h)) == _lib.DIPS_ERR_INVALID
    assert not h.value
    assert lib.dips_alt_last_error(None)


def test_alt_null_handle_calls_are_safe():
    lib = _lib.load()
    assert lib.dips_alt_send_frame(None, None, 0, 0, None, 0) == _lib.DIPS_ERR_INVALID
    assert lib.dips_alt_send_frames(None, None, 1, None, None) == _lib.DIPS_ERR_INVALID
    assert lib.dips_alt_run(None, None, 1, None, 0, None) == _lib.DIPS_ERR_INVALID
    h = ctypes.c_void_p()
    assert lib.dips_alt_create(None, 0, 8, 0, ctypes.byref(h)) == _lib.DIPS_ERR_INVALID
    lib.dips_alt_destroy(None)


def test_alt_lut_index_is_exact_and_injective():
    """The host-built two-level index of the dips_alt epilogue table
    (dips_amd/csrc/alt_lut.h, dips_alt_lut_index; no device): its value set
    is every f32 u(S) - (u(max) + u(min)) / 2, and every value reaches its own
    level-2 slot through the device's arithmetic -- cluster
    rint(510 * diff) from fma(diff, 510, 1.5 * 2^23) (exact rational
    arithmetic here), then ((bits(diff) >> sh) << 1) + x."""
    import ctypes
    from fractions import Fraction
    from dips_amd import _lib
    lib = _lib.load()
    n, l2 = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.dips_alt_lut_index(None, 0, None, None, 0, ctypes.byref(n), ctypes.byref(l2)) == 0
    l1 = np.zeros(2 * 1021, dtype=np.uint32)
    diffs = np.zeros(n.value, dtype=np.float32)
    slots = np.zeros(n.value, dtype=np.uint16)
    assert lib.dips_alt_lut_index(l1.ctypes.data, l1.size, diffs.ctypes.data, slots.ctypes.data, n.value,
                                  ctypes.byref(n), ctypes.byref(l2)) == 0
    # the value set, from the reference arithmetic
    F32 = np.float32
    u = (np.arange(256, dtype=np.float64) / 255.0).astype(F32)
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    iv = np.unique(((u[mx[keep]] + u[mn[keep]]) / F32(2)).astype(F32))
    want = np.unique((u[:, None] - iv[None, :]).astype(F32).ravel())
    assert len(want) == 2993
    assert np.array_equal(np.sort(diffs.view(np.uint32)), np.sort(want.view(np.uint32)))
    assert l2.value <= 5888  # kAltLutL2Max
    assert len(np.unique(slots)) == len(slots) and int(slots.max()) < l2.value
    bias = ((0x4B400000 - 510) << 3) & 0xFFFFFFFF
    for d, slot in zip(diffs.tolist(), slots.tolist()):
        # fma(d, 510, 1.5 * 2^23) rounded once to f32 (RNE), exactly
        exact = Fraction(d) * 510 + 12582912
        t = float(np.float32(float(exact)))  # the f64 of an exact rational, then f32
        # guard the double rounding: the f32 result must be the nearest to the exact value
        lo, hi = np.nextafter(F32(t), F32(-np.inf)), np.nextafter(F32(t), F32(np.inf))
        assert abs(Fraction(t) - exact) <= min(abs(Fraction(float(lo)) - exact), abs(Fraction(float(hi)) - exact))
        tb = int(np.array([t], dtype=np.float32).view(np.uint32)[0])
        a1 = ((tb << 3) - bias) & 0xFFFFFFFF
        assert a1 % 8 == 0 and a1 // 8 < 1021
        x, sh = int(l1[2 * (a1 // 8)]), int(l1[2 * (a1 // 8) + 1])
        db = int(np.array([d], dtype=np.float32).view(np.uint32)[0])
        a2 = (((db >> sh) << 1) + x) & 0xFFFFFFFF
        assert a2 == 2 * slot, (d, slot, a2)
