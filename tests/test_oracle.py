"""CPU tests of the oracle (test infrastructure): analytic known answers
(SURVEY.md s8c), the C restatement against the independent numpy
restatement, the committed golden fixtures, and the arithmetic identities
the HIP kernels rely on."""
import ctypes
import itertools
import json
import os

import numpy as np
import pytest

from oracle import np_restatement as nr
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_unorm_load_and_store_pins(oracle_lib):
    for c in range(256):
        u = oracle_lib.dips_oracle_u(c)
        assert np.float32(u) == np.float32(c) / np.float32(255.0)
        assert oracle_lib.dips_oracle_q(u) == c  # q(u(c)) round-trips
    # ties round half to even (SURVEY.md s8 "Canonical definitions")
    assert oracle_lib.dips_oracle_q(np.float32(20.5) / np.float32(255.0)) in (20,)
    assert oracle_lib.dips_oracle_q(float("nan")) == 0
    assert oracle_lib.dips_oracle_q(-1.0) == 0 and oracle_lib.dips_oracle_q(7.0) == 255


def test_upper_median_known_answer(oracle_lib):
    a = (ctypes.c_float * 4)(0.1, 0.4, 0.2, 0.3)
    assert abs(oracle_lib.dips_oracle_upper_median4(a) - 0.3) < 1e-7
    rng = np.random.default_rng(0)
    for _ in range(200):
        v = rng.random(4).astype(np.float32)
        a = (ctypes.c_float * 4)(*v)
        assert np.float32(oracle_lib.dips_oracle_upper_median4(a)) == np.sort(v)[2]


def test_unorm_fma_identity():
    """The HIP kernels compute u(c) = c/255 as fma(c, K_HI, c*K_LO)
    (dips_amd/csrc/series_kernels.hip unorm2): exact for every byte."""
    from fractions import Fraction
    k_hi = np.float32(float.fromhex("0x1.010102p-8"))
    k_lo = np.float32(float.fromhex("-0x1.fdfdfep-33"))

    def round_f32(x: Fraction) -> np.float32:
        cand = np.float32(float(x))
        best = cand
        for nb in (np.nextafter(cand, np.float32(-1)), np.nextafter(cand, np.float32(2))):
            if abs(Fraction(float(nb)) - x) < abs(Fraction(float(best)) - x):
                best = nb
        return best

    for c in range(256):
        lo = np.float32(np.float32(c) * k_lo)
        fma = round_f32(Fraction(c) * Fraction(float(k_hi)) + Fraction(float(lo)))
        assert fma == nr.U_LUT[c], c


def test_i2_pair_identity():
    """I2 = u(max) + u(min) equals 2 * get_intensity exactly, and the f32
    difference of I2 values is exactly twice the difference of I values."""
    a = np.arange(256, dtype=np.int64)
    mx, mn = np.meshgrid(a, a, indexing="ij")
    keep = mx >= mn
    mx, mn = mx[keep], mn[keep]
    i2 = (nr.U_LUT[mx] + nr.U_LUT[mn]).astype(np.float32)
    i = ((nr.U_LUT[mx] + nr.U_LUT[mn]).astype(np.float32) / np.float32(2.0)).astype(np.float32)
    assert np.array_equal(i2, (i * np.float32(2.0)).astype(np.float32))
    rng = np.random.default_rng(1)
    p, q = rng.integers(0, i.size, 200000), rng.integers(0, i.size, 200000)
    d2 = np.abs((i2[p] - i2[q]).astype(np.float32))
    d1 = np.abs((i[p] - i[q]).astype(np.float32))
    assert np.array_equal(d2, (d1 * np.float32(2.0)).astype(np.float32))
    # every |dI| is a multiple of 2^-32: dI * 2^32 is an exact integer
    assert np.all(np.ldexp(d1.astype(np.float64), 32) == np.floor(np.ldexp(d1.astype(np.float64), 32)))


def test_exp_log_close_to_libm(oracle_lib):
    xs = np.linspace(-30, 30, 20001).astype(np.float32)
    got = np.array([oracle_lib.dips_oracle_expf(float(x)) for x in xs])
    np.testing.assert_allclose(got, np.exp(xs.astype(np.float64)), rtol=5e-7)
    ys = np.geomspace(1e-30, 1e30, 20001).astype(np.float32)
    got = np.array([oracle_lib.dips_oracle_logf(float(y)) for y in ys])
    np.testing.assert_allclose(got, np.log(ys.astype(np.float64)), rtol=5e-7, atol=1e-7)


def test_exp_log_c_equals_numpy(oracle_lib):
    rng = np.random.default_rng(2)
    xs = np.concatenate([rng.uniform(-110, 95, 50000), rng.uniform(-3, 3, 50000),
                         [0.0, -0.0, np.inf, -np.inf]]).astype(np.float32)
    c = np.array([oracle_lib.dips_oracle_expf(float(x)) for x in xs], dtype=np.float32)
    assert np.array_equal(c.view(np.uint32), nr.expf(xs).view(np.uint32))
    ys = np.concatenate([rng.uniform(0, 4, 50000), 10.0 ** rng.uniform(-44, 38, 50000),
                         [0.0, np.inf]]).astype(np.float32)
    c = np.array([oracle_lib.dips_oracle_logf(float(y)) for y in ys], dtype=np.float32)
    assert np.array_equal(c.view(np.uint32), nr.logf(ys).view(np.uint32))


@pytest.mark.parametrize("c", [1, 3, 4])
def test_synth_c_equals_numpy(c):
    assert np.array_equal(oracle.synth(c, 37, 23, 5, 1000, 4), nr.synth(c, 37, 23, 5, 1000, 4))


@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
def test_series_c_equals_numpy(c, mode):
    for chroma, tau, seed in itertools.product([0, 1, 2, 3] if c != 1 else [0], [0.0, 8 / 255], [1, 2]):
        frames = oracle.synth(c, 29, 17, seed, 0, 5)
        ref = oracle.synth(c, 29, 17, seed + 100, 0, 1)[0]
        for r in (None, ref):
            a, sa, da = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, ref=r, want_map=True)
            b, sb, db = nr.series(frames, mode=mode, chroma=chroma, tau=tau, ref=r)
            assert np.array_equal(a, b)
            assert np.array_equal(da, db)
            np.testing.assert_allclose(sa, sb, rtol=1e-12)
            # the f64 sum agrees with the exact fixed-point sum
            np.testing.assert_allclose(sa, np.ldexp(a[:, 3].astype(np.float64), -32), rtol=1e-12)


def test_series_multithread_equals_single():
    frames = oracle.synth(3, 40, 30, 9, 0, 13)
    for mode in (0, 1):
        a, sa, _ = oracle.series(frames, mode=mode, tau=1 / 255)
        b, sb, _ = oracle.series(frames, mode=mode, tau=1 / 255, nthreads=4)
        assert np.array_equal(a, b) and np.array_equal(sa, sb)


def test_series_known_answers():
    # identical frames: everything zero
    f = np.repeat(oracle.synth(3, 16, 8, 1, 0, 1), 4, axis=0)
    out4, si, dmap = oracle.series(f, mode=0, want_map=True)
    assert not out4.any() and not si.any() and not dmap.any()
    # single pixel black -> white: SJ = 510, SI = 1.0, SAD = 765
    f = np.zeros((2, 8, 8, 3), np.uint8)
    f[1, 3, 4] = 255
    out4, si, _ = oracle.series(f)
    assert out4[1].tolist() == [765, 510, 1, 1 << 32] and si[1] == 1.0


def test_series_rejects_bad_args(oracle_lib):
    f = np.zeros((1, 2, 2, 3), np.uint8)
    with pytest.raises(ValueError):
        oracle.series(f, tau=-1.0)
    with pytest.raises(ValueError):
        oracle.series(f, chroma=4)


PARAMS = list(itertools.product([False, True], [1, 2, 3, 5, 11], [5.0, 0.7], [255, 0, 1], [0, 1, 3]))


@pytest.mark.parametrize("colorize,window,sens,filt,chroma", PARAMS[::3])
def test_compute_state_c_equals_numpy(colorize, window, sens, filt, chroma):
    rng = np.random.default_rng(window * 7 + filt)
    w, h = 19, 13
    frames = rng.integers(0, 256, (8, h, w, 4), dtype=np.uint8)
    frames[3] = frames[2]
    a = oracle.ComputeState(colorize, window, sens, filt, chroma)
    b = nr.ComputeState(colorize, window, sens, filt, chroma)
    for k in range(8):
        a.add_texture(w, h, frames[k])
        b.add_texture(w, h, frames[k])
        x, y = a.dispatch(), b.dispatch()
        assert (x is None) == (y is None)
        if x is not None:
            assert np.array_equal(x, y)


def test_compute_state_known_answers():
    """Identical frames: 128 for gray pixels; odd max+min (10,20,31) gives
    129 while unquantised slots decide the median (t = 3..5)."""
    w = h = 8
    f = np.zeros((h, w, 4), np.uint8)
    f[..., 3] = 255
    f[0, 0, :3] = (10, 20, 31)
    f[0, 1, :3] = (100, 101, 102)
    cs = oracle.ComputeState(False, 1, 5.0, 255, 0)
    outs = []
    for _ in range(8):
        cs.add_texture(w, h, f)
        outs.append(cs.dispatch())
    assert outs[0] is None and outs[1] is None and outs[2] is None
    assert [int(o[0, 0, 0]) for o in outs[3:]] == [129, 129, 129, 128, 128]
    assert all(int(o[0, 1, 0]) == 128 and int(o[4, 4, 0]) == 128 for o in outs[3:])
    # W = 3 spatial filter: the quirky median is always 0
    cs3 = oracle.ComputeState(False, 3, 5.0, 255, 0)
    for _ in range(4):
        cs3.add_texture(w, h, f)
    st = cs3.start_texture()
    assert not st[..., :3].any()


def _load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_golden_manifest_and_fixtures():
    """The committed fixtures (made by tests/golden/make_golden.py from the
    numpy restatement, cross-checked there against the C oracle) still match
    the oracle."""
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        manifest = json.load(f)
    assert manifest["pins"]["bounds_policy"] == "naga Restrict (Vulkan/DX12)"
    for case in manifest["series"]:
        z = _load_golden(case["file"])
        out4, si, dmap = oracle.series(z["frames"], mode=case["mode"], chroma=case["chroma"],
                                       tau=case["tau"], ref=z["ref"] if "ref" in z else None,
                                       want_map=True)
        assert np.array_equal(out4, z["out4"]), case["file"]
        assert np.array_equal(dmap, z["dmap"]), case["file"]
        np.testing.assert_allclose(si, z["si"], rtol=1e-12)
    for case in manifest["compute_state"]:
        z = _load_golden(case["file"])
        cs = oracle.ComputeState(*case["params"])
        outs = z["outputs"]
        for k, fr in enumerate(z["frames"]):
            cs.add_texture(fr.shape[1], fr.shape[0], fr)
            o = cs.dispatch()
            if k < 3:
                assert o is None
            else:
                assert np.array_equal(o, outs[k - 3]), (case["file"], k)
    for case in manifest["alt"]:
        z = _load_golden(case["file"])
        fr = z["frames"]
        got = oracle.AltCompute(case["num_textures"], fr.shape[2], fr.shape[1], case["colorize"], case["window"],
                                case["scalar"], case["filter"], case["chroma"]).run(fr, case["markers"])
        assert np.array_equal(got, z["outputs"]), case["file"]


def test_v2_intensity_identity():
    """series_v2 (dips_amd/csrc/series_v2.hip) computes 2*get_intensity
    without conversions: u(c) = c/255 rounds UP to c*65793*2^-24 +
    2^(msb(c)-31), hence u(max) + u(min) = RNE(J*65793*2^-24 + E*2^-31) with
    J = max+min and E = P(max)+P(min).  Exhaustive over every byte pair."""
    from fractions import Fraction
    for c in range(1, 256):
        p = 1 << (c.bit_length() - 1)
        assert Fraction(float(nr.U_LUT[c])) == Fraction(c * 65793, 1 << 24) + Fraction(p, 1 << 31), c
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    mx, mn = mx[keep], mn[keep]
    pw = lambda c: np.where(c > 0, np.left_shift(1, np.floor(np.log2(np.maximum(c, 1))).astype(np.int64)), 0)
    # exact in f64 (< 2^34 significant bits), then one rounding to f32
    i2s = ((mx + mn) * 65793 / 4.0 + (pw(mx) + pw(mn)) / 512.0).astype(np.float32)
    want = (nr.U_LUT[mx] + nr.U_LUT[mn]).astype(np.float32) * np.float32(2.0 ** 22)
    assert np.array_equal(i2s, want)


def test_v2_sj_from_intensity_difference():
    """series_v2 derives SJ = sum |dJ| from the intensity differences:
    |255 * |dI2| - |dJ|| < 1.1e-4 per pixel, EXHAUSTIVELY over every pair of
    (max, min) byte pairs (32896^2 pixel pairs), so the per-lane f32 sum
    rounds to the exact integer (next test)."""
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    mx, mn = mx[keep], mn[keep]
    i2 = (nr.U_LUT[mx] + nr.U_LUT[mn]).astype(np.float32)
    j = (mx + mn).astype(np.float64)
    # distinct I2 values decide the error; same I2 with different J cannot occur
    worst = 0.0
    for s in range(0, i2.size, 512):
        a = np.abs((i2[s:s + 512, None] - i2[None, :]).astype(np.float32)).astype(np.float64)
        err = np.abs(255.0 * a - np.abs(j[s:s + 512, None] - j[None, :]))
        worst = max(worst, float(err.max()))
    assert worst < 1.1e-4, worst


def test_v2_sj_lane_sum_rounds_exactly():
    """The kernel's per-lane SJ accumulation: sj = 0.5, then 20 fused
    sj = fma(|dI2s|, 255 * 2^-22, sj) (U = 5 vecs x 4 px per lane and frame,
    the RGB8 kernel; RGBA8's 4 vecs make 16);
    trunc(sj) must equal the lane's sum of |dJ|.  Lanes of worst-case pixels
    (largest per-pixel error, largest |dJ|) and random ones."""
    rng = np.random.default_rng(11)
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    mx, mn = mx[keep], mn[keep]
    i2s = ((nr.U_LUT[mx] + nr.U_LUT[mn]).astype(np.float32) * np.float32(2.0 ** 22)).astype(np.float32)
    j = (mx + mn).astype(np.int64)
    k_sj = np.float64(np.float32(255.0 / 4194304.0))
    n_lanes, px = 200_000, 20
    p = rng.integers(0, i2s.size, (n_lanes, px))
    q = rng.integers(0, i2s.size, (n_lanes, px))
    # append lanes of the extreme pixel pairs
    ext = np.array([0, i2s.size - 1, int(np.argmax(j)), int(np.argmin(j))])
    p = np.concatenate([p, np.repeat(ext[:, None], px, axis=1), np.repeat(ext[::-1, None], px, axis=1)])
    q = np.concatenate([q, np.repeat(ext[::-1, None], px, axis=1), np.repeat(ext[:, None], px, axis=1)])
    a = np.abs((i2s[p] - i2s[q]).astype(np.float32)).astype(np.float64)
    sj = np.full(p.shape[0], 0.5, dtype=np.float32)
    for k in range(px):
        # fma in f64 is exact here (a * k_sj has <= 32 significant bits, the
        # sum stays below 2^14), then one rounding to f32 = the fused result
        sj = (a[:, k] * k_sj + sj.astype(np.float64)).astype(np.float32)
    want = np.abs(j[p] - j[q]).sum(axis=1)
    assert np.array_equal(np.trunc(sj).astype(np.int64), want)


@pytest.mark.parametrize("tau", [0.03125, 8 / 255, 0.1, 0.5, 0.999, float(np.nextafter(np.float32(1), np.float32(0)))])
def test_v2_sadi_sums(tau):
    """series_v2 SADI (ISI = 2): per pixel x = trunc(|dI| * 2^28) (the
    intensities x32, I * 2^28), T = min(tau * 2^28, 2^28); per lane of 16
    pixels Sa = sum |x - T| (one u32), Sx_0 / Sx_1 = sum x over the two 8-pixel
    halves; the record carries Q = (Sa + Sx - 16 T) / 2 and
    u = (Sx_0 >> 8) + (Sx_1 >> 8); series_reduce adds 16 T count per frame and
    rounds SJ = (sum u * 510 + 2^19) >> 20 per 1024-pixel tile.  Checked:
    Q = sum_selected x - c T exactly and in [0, 2^32), the selected x exact
    (x * 2^-28 = |dI|), every u32 sum in range, and the per-tile SJ equal to
    sum |dJ| -- random tiles and tiles of the extreme pixel pairs (black
    against white: x = 2^28; equal pixels: x = 0).  SADI is used for
    2^-5 <= tau < 1 only: with tau = 1, T = 2^28 and 16 equal pixels would
    make Sa = 2^32."""
    rng = np.random.default_rng(23)
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    mx, mn = mx[keep], mn[keep]
    i28 = ((nr.U_LUT[mx] + nr.U_LUT[mn]).astype(np.float32) * np.float32(2.0 ** 27)).astype(np.float32)
    j = (mx + mn).astype(np.int64)
    tau32 = np.float32(tau)
    thr = np.float32(tau32 * np.float32(2.0 ** 28))
    T = int(min(float(thr), 2.0 ** 28))
    assert float(thr) == T and 2 ** 23 <= T < 2 ** 28
    n_tiles, lanes, px = 300, 64, 16
    p = rng.integers(0, i28.size, (n_tiles, lanes, px))
    q = rng.integers(0, i28.size, (n_tiles, lanes, px))
    ext = np.array([0, i28.size - 1, int(np.argmax(j)), int(np.argmin(j))])
    for a_, b_ in ((ext[0], ext[1]), (ext[1], ext[0]), (ext[2], ext[3]), (ext[0], ext[0]), (ext[1], ext[1])):
        p = np.concatenate([p, np.full((1, lanes, px), a_)])
        q = np.concatenate([q, np.full((1, lanes, px), b_)])
    d = np.abs((i28[p] - i28[q]).astype(np.float32))  # |dI| * 2^28, f32 (the kernel's d)
    x = np.trunc(d.astype(np.float64)).astype(np.int64)
    sel = d > thr
    assert np.all(x[sel] == d[sel].astype(np.float64)) and x.max() <= 2 ** 28
    sa = np.abs(x - T).sum(axis=2)
    sx0, sx1 = x[..., :8].sum(axis=2), x[..., 8:].sum(axis=2)
    assert sa.max() < 2 ** 32 and max(sx0.max(), sx1.max()) <= 2 ** 31
    q2 = sa + sx0 + sx1 - 16 * T
    assert np.all(q2 % 2 == 0) and q2.min() >= 0 and q2.max() < 2 ** 33
    qv = q2 // 2
    cnt = sel.sum(axis=2)
    assert np.array_equal(qv, np.where(sel, x, 0).sum(axis=2) - cnt * T)
    u = (sx0 >> 8) + (sx1 >> 8)
    assert u.max() <= 2 ** 24 and u.sum(axis=1).max() <= 2 ** 30
    sj_tile = (u.sum(axis=1) * 510 + (1 << 19)) >> 20
    assert np.array_equal(sj_tile, np.abs(j[p] - j[q]).sum(axis=(1, 2)))


def test_tau_boundary_fixtures_straddle_tau():
    """The *_tauedge fixtures hold pixels whose f32 |dI| is exactly f32(tau)
    and one ulp either side: moving tau down one ulp adds the 'equal' pixels
    to the count, moving it up one ulp drops the 'above' pixels -- so the
    fixtures pin the strict '>' of the threshold (series_v2.hip, the gray
    kernel and dips_oracle.c alike)."""
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        manifest = json.load(f)
    cases = [c for c in manifest["series"] if c.get("tau_boundary")]
    assert len(cases) == 14
    for case in cases:
        z = _load_golden(case["file"])
        t = np.float32(case["tau"])
        counts = []
        for tau in (np.nextafter(t, np.float32(0)), t, np.nextafter(t, np.float32(1))):
            out4, _, _ = oracle.series(z["frames"], mode=case["mode"], chroma=case["chroma"], tau=float(tau))
            counts.append(out4[1, 2])
        assert counts[0] > counts[1] > counts[2], (case["file"], counts)
        assert z["out4"][1, 2] == counts[1]


def test_gray_si_decomposition():
    """The identity behind series_gray_lut_kernel (dips_amd/csrc/series_gray.hip),
    exhaustively over all 65,536 gray byte pairs (a, b): with u(c) = c / 255
    correctly rounded, V = |RN(u(a) - u(b))| * 2^31 is an integer and
    V = 8421504 * |a - b| + corr with corr in {0, 1, 2, 4, ..., 128}, so a
    selected pixel's SI_fixed contribution 2 V is carried exactly by the two
    bytes (|a - b|, corr) of its table entry."""
    F32 = np.float32
    u = (np.arange(256, dtype=np.float64) / 255.0).astype(F32)
    a, b = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    di = np.abs((u[a] - u[b]).astype(F32)).astype(np.float64)
    v = di * 2.0 ** 31
    assert np.all(v == np.floor(v))
    v = v.astype(np.int64)
    d = np.abs(a - b)
    corr = v - 8421504 * d
    assert set(np.unique(corr).tolist()) <= {0, 1, 2, 4, 8, 16, 32, 64, 128}
    # the oracle's f32 dI is the same value: SI_fixed of a selected pixel = 2 V
    frames = np.stack([b.astype(np.uint8), a.astype(np.uint8)])  # reference b, then frame a
    out4, _, _ = oracle.series(frames, mode=1, tau=0.0)
    assert int(out4[1, 3]) == int(2 * v.sum())


def test_gray_alu_vec_identity():
    """The arithmetic vecs of series_gray_lut_kernel (series_gray.hip
    gray_alu_dword), exhaustively over the 65,536 byte pairs and several
    tau >= 2^-5: U'(c) = fma(c, 2^28 K_HI, c * 2^28 K_LO) = 2^28 u(c), the
    f32 difference D' = 2^28 RN(u(a) - u(b)), the pixel is selected exactly
    when dI > tau, a selected |D'| is an integer with 8 |D'| = V (the table's
    8421504 d + corr), and a per-lane sum S of 8 selected |D'| splits into
    sum d = S // 1052688 and sum corr = 8 (S mod 1052688)."""
    from fractions import Fraction
    F32 = np.float32
    k_hi = F32(float.fromhex("0x1.010102p20"))
    k_lo = F32(float.fromhex("-0x1.fdfdfep-5"))
    assert k_hi == F32(float.fromhex("0x1.010102p-8")) * F32(2.0 ** 28)
    assert k_lo == F32(float.fromhex("-0x1.fdfdfep-33")) * F32(2.0 ** 28)
    u28 = np.empty(256, F32)
    for c in range(256):
        lo = F32(F32(c) * k_lo)
        x = Fraction(c) * Fraction(float(k_hi)) + Fraction(float(lo))
        cand = F32(float(x))
        for nb in (np.nextafter(cand, F32(-1)), np.nextafter(cand, F32(2 ** 30))):
            if abs(Fraction(float(nb)) - x) < abs(Fraction(float(cand)) - x):
                cand = nb
        u28[c] = cand
    assert np.array_equal(u28.astype(np.float64), nr.U_LUT.astype(np.float64) * 2.0 ** 28)
    a, b = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    dp = np.abs((u28[a] - u28[b]).astype(F32))
    di = np.abs((nr.U_LUT[a] - nr.U_LUT[b]).astype(F32))
    assert np.array_equal(dp.astype(np.float64), di.astype(np.float64) * 2.0 ** 28)
    v = (di.astype(np.float64) * 2.0 ** 31).astype(np.int64)
    d = np.abs(a - b)
    rng = np.random.default_rng(5)
    for tau in (0.03125, 8.0 / 255.0, 0.05, 0.1, 0.5, 0.999, 1.0):
        tau = F32(tau)
        thr28 = F32(tau * F32(2.0 ** 28))
        assert float(thr28) == float(tau) * 2.0 ** 28 and float(thr28) == int(thr28)
        sel_alu = dp > thr28
        assert np.array_equal(sel_alu, di > tau)
        s = dp[sel_alu].astype(np.float64)
        assert np.all(s == np.floor(s)) and s.max(initial=0) <= 2.0 ** 28
        assert np.array_equal(8 * s.astype(np.int64), v[sel_alu])
        # random lanes of 8 selected pixels (worst case: 8 * 2^28 < 2^32)
        idx = np.flatnonzero(sel_alu.ravel())
        if idx.size == 0:
            continue
        lanes = rng.choice(idx, size=(4096, 8))
        S = dp.ravel()[lanes].astype(np.int64).sum(axis=1)
        assert S.max() < 2 ** 32
        sum_d, sum_corr = S // 1052688, 8 * (S % 1052688)
        assert np.array_equal(sum_d, d.ravel()[lanes].sum(axis=1))
        assert np.array_equal(8421504 * sum_d + sum_corr, v.ravel()[lanes].sum(axis=1))


@pytest.mark.parametrize("tau", [0.0, 1 / 255, 2 / 255, 7.5 / 255, 8 / 255, 15.9 / 255, 0.1, 0.5, 0.999, 1.0])
def test_gray_band_layout(tau):
    """Layout 3 of the GRAY8 table (series_gray.hip kGrayBandOffset): the
    entry of (a, b) at u16 index x * 256 + (a ^ sw(x)), x = a ^ b,
    sw(x) = (x << 1) & 0x7E, is a bijection of the 65,536 pairs; the band word
    (max of 256 - x over rows x holding a selected pair) gives
    K = 256 * 2^m - 1, m = floor(log2(first such row)), and every index
    <= K holds entry 0 -- so the kernel's clamp max(index, K) changes no
    entry, for any tau.  Also: the clamp is the whole near-diagonal band the
    bench's content lives in (|a - b| <= 7 at tau = 8/255 maps to K), and
    the bank of an index (bits 1-6) mixes a and x."""
    F32 = np.float32
    a, b = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    di = np.abs((nr.U_LUT[a] - nr.U_LUT[b]).astype(F32))
    sel = di > F32(tau)
    x = a ^ b
    pos = x * 256 + (a ^ ((x << 1) & 0x7E))
    assert np.array_equal(np.sort(pos.ravel()), np.arange(65536))
    entry = np.zeros(65536, dtype=np.int64)
    entry[pos.ravel()] = np.where(sel, 1 + np.abs(a - b), 0).ravel()  # nonzero exactly when selected
    rows = np.unique(x[sel])
    w = int(256 - rows.min()) if rows.size else 0
    first = 256 - min(w, 255)
    m = first.bit_length() - 1
    K = (256 << m) - 1
    assert K <= 65535 and not entry[: K + 1].any()
    # the kernel's view: max(index, K) reads the same entry as index
    assert np.array_equal(entry[np.maximum(pos, K)], entry[pos])
    # the band is as wide as tau allows: row `first` holds a selected pair
    if first < 256:
        assert entry[first * 256:(first + 1) * 256].any() and first < (2 << m)
    if abs(tau - 8 / 255) < 1e-9:
        assert K == 2047 and np.all(np.maximum(pos, K)[x < 8] == K)
    bank = (pos >> 1) & 63
    assert np.array_equal(bank, ((a >> 1) ^ x) & 63)


@pytest.mark.parametrize("filt", [0, 1, 255])
@pytest.mark.parametrize("colorize", [False, True])
def test_epilogue_table_encoding(filt, colorize):
    """The epilogue tables (compat_batch_lut_kernel, alt_lut.h) keep only
    R | G << 8 of each texel: B = min(R, G) and A = 255 must hold for every
    argument they are built from -- every diff u(S) - u(m) of the ComputeState
    table and every dips_alt diff u(S) - I -- for every filter, colour mode
    and sensitivities inside and far outside the usual range (inf / NaN
    texels of the inverse sigmoid included).  numpy restatement of the spec
    epilogue, exhaustive over the tables' domains."""
    F32 = np.float32
    u = (np.arange(256, dtype=np.float64) / 255.0).astype(F32)
    d_compat = (u[:, None] - u[None, :]).astype(F32).ravel()
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    iv = np.unique(((u[mx[keep]] + u[mn[keep]]) / F32(2)).astype(F32))
    d_alt = np.unique((u[:, None] - iv[None, :]).astype(F32).ravel())
    for k in (5.0, 1.0, 10.0, 0.0, -3.0, 200.0, 1e-30, 1e30):
        for d in (d_compat, d_alt):
            out = nr.epilogue(d, filt, k, colorize)
            assert np.all(out[:, 3] == 255)
            assert np.array_equal(out[:, 2], np.minimum(out[:, 0], out[:, 1])), (filt, colorize, k)
