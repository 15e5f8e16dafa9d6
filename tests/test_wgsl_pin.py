"""Parity of the oracle against the reference's own shader text (CPU).

oracle/wgsl_exec.py executes WGSL; oracle/wgsl_ref.py runs the reference's
shader files with the host side (ring, start texture, uniform index, the
dips_alt splice and run loop) restated from its Rust.  These tests:

* check the interpreter's WGSL semantics on small programs of our own
  (integer division / remainder, f32 %, abstract literals, loops with break /
  continue under divergent lanes, early return, switch, u32 wrap, both bounds
  policies);
* check the C oracle against every wgsl_* fixture (outputs of the executed
  reference shaders, tests/golden/make_wgsl_golden.py) -- no reference
  checkout needed;
* where the reference checkout is present (this container): the fixtures'
  shader hashes still match it and every fixture but the W = 11 one (25 s
  in the interpreter; generated under the same C-oracle assert) regenerates
  byte for byte; get_intensity from dips_shader.wgsl equals the restatement over all
  2^24 RGB triples and every channel value; fresh randomized ComputeState /
  dips_alt draws equal the C oracle; the Metal bounds policy reproduces
  SURVEY.md s8 A3's all-zero start texture; correctly rounded exp / log move
  an output byte by at most 1.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle
from oracle.wgsl_exec import Module, Pins, V, WgslError

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "wgsl_manifest.json")) as _f:
    WMAN = json.load(_f)

from oracle import wgsl_ref  # noqa: E402  (reads nothing at import)


@pytest.fixture
def ref():
    """Skip unless the reference checkout is present (it never is on a GPU
    box; these tests are CPU-only and only look for it when they run)."""
    if not wgsl_ref.available():
        pytest.skip("reference checkout not present")


needs_ref = pytest.mark.usefixtures("ref")

DISPATCH = -1


def _load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# -- interpreter semantics ---------------------------------------------------

_PROGRAM = """
const N: i32 = 4;
fn idiv(a: i32, b: i32) -> i32 { return a / b; }
fn irem(a: i32, b: i32) -> i32 { return a % b; }
fn udiv(a: u32, b: u32) -> u32 { return a / b; }
fn frem(a: f32, b: f32) -> f32 { return a % b; }
fn lit(x: f32) -> f32 { return x + 1 / 2 + 3 / 2.0; }
fn loopy(n: i32) -> i32 {
    var s = 0;
    for (var i = 0; i < 10; i++) {
        if (i == n) { break; }
        if (i % 2 == 1) { continue; }
        s += i;
    }
    return s;
}
fn early(x: f32) -> f32 {
    if (x < 0) { return -1.0; }
    var y = x * 2.0;
    y *= 3;
    return y;
}
fn arr(j: i32) -> f32 {
    var a: array<f32, N>;
    for (var i = 0; i < N; i++) { a[i] = f32(i + 1); }
    a[j] = 9.0;
    return a[j + 1];
}
fn sw(s: u32) -> i32 {
    switch s {
        case 0u: { return 10; }
        case 1u, 2u: { return 20; }
        default: { return 30; }
    }
}
fn wrap(a: u32) -> u32 { return a - 1u; }
fn conv(x: f32) -> i32 { return i32(x); }
fn vecs(x: f32) -> f32 {
    let v = vec3<f32>(x, 2.0 * x, 0.5) - vec3<f32>(1.0, 1.0, 1.0);
    return v.r + v.y * v.b + max(v.x, v.g);
}
@compute @workgroup_size(1)
fn main() {}
"""


def _call(fn, ty, values, pins=Pins()):
    pipe = Module(_PROGRAM).pipeline("main", {}, pins)
    return np.asarray(pipe.call(fn, [V(ty, np.asarray(v)) for v in values]).d)


def test_interpreter_integer_semantics():
    a = np.array([7, -7, 7, -7, 5, -2147483648], np.int32)
    b = np.array([2, 2, -2, -2, 0, -1], np.int32)
    # truncating division; x / 0 = x and INT_MIN / -1 = INT_MIN (WGSL)
    assert _call("idiv", "i32", [a, b]).tolist() == [3, -3, -3, 3, 5, -2147483648]
    assert _call("irem", "i32", [a, b]).tolist() == [1, -1, 1, -1, 0, 0]
    assert _call("udiv", "u32", [np.array([7, 9], np.uint32), np.array([2, 0], np.uint32)]).tolist() == [3, 9]
    assert _call("wrap", "u32", [np.array([0, 5], np.uint32)]).tolist() == [4294967295, 4]
    assert _call("conv", "f32", [np.array([2.9, -2.9, 3e9, np.nan], np.float32)]).tolist() == \
        [2, -2, 2147483520, 0]


def test_interpreter_float_and_abstract_semantics():
    # f32 %: e1 - e2 * trunc(e1 / e2)
    got = _call("frem", "f32", [np.array([5.5, -5.5, 2.0], np.float32), np.array([2.0, 2.0, 2.0], np.float32)])
    assert got.tolist() == [1.5, -1.5, 0.0]
    # 1 / 2 is abstract-int 0, 3 / 2.0 abstract-float 1.5
    assert _call("lit", "f32", [np.array([1.0], np.float32)]).tolist() == [2.5]
    x = np.array([3.0, 0.25], np.float32)
    want = (x - 1) + (2 * x - 1) * np.float32(-0.5) + np.maximum(x - 1, 2 * x - 1)
    assert np.array_equal(_call("vecs", "f32", [x]), want.astype(np.float32))


def test_interpreter_divergent_control_flow():
    n = np.arange(-1, 12, dtype=np.int32)
    want = [sum(i for i in range(10) if i % 2 == 0 and (k < 0 or i < k)) for k in n]
    assert _call("loopy", "i32", [n]).tolist() == want
    assert _call("early", "f32", [np.array([-2.0, 1.5], np.float32)]).tolist() == [-1.0, 9.0]
    assert _call("sw", "u32", [np.array([0, 1, 2, 3, 7], np.uint32)]).tolist() == [10, 20, 20, 30, 30]


def test_interpreter_bounds_policies():
    j = np.array([0, 2, 3, 4, -1], np.int32)
    # Restrict: every index clamped to the last element (a negative i32
    # index compares as a huge u32: a[-1] = 9.0 lands on a[3], a[0] is read)
    assert _call("arr", "i32", [j], Pins(bounds="restrict")).tolist() == [2.0, 4.0, 9.0, 9.0, 1.0]
    # ReadZeroSkipWrite: out-of-range reads give 0, writes are dropped
    assert _call("arr", "i32", [j], Pins(bounds="read_zero_skip_write")).tolist() == [2.0, 4.0, 0.0, 0.0, 1.0]


def test_interpreter_rejects_what_it_does_not_implement():
    with pytest.raises(WgslError):
        Module("fn f() -> i32 { loop { break; } return 1; } @compute @workgroup_size(1) fn main() {}")
    pipe = Module("fn f(a: f32) -> f32 { return frobnicate(a); } @compute @workgroup_size(1) fn main() {}"
                  ).pipeline("main")
    with pytest.raises(WgslError):
        pipe.call("f", [V("f32", np.zeros(2, np.float32))])


# -- the C oracle against the executed reference shaders --------------------

def _run_cs(cs, frames, ops, w, h):
    outs, some = [], []
    for op in ops:
        if op == DISPATCH:
            o = cs.dispatch()
            some.append(o is not None)
            if o is not None:
                outs.append(o)
        else:
            cs.add_texture(w, h, frames[op])
    return np.stack(outs) if outs else np.zeros((0, h, w, 4), np.uint8), np.array(some)


def test_wgsl_manifest_records_provenance():
    assert set(WMAN["shaders"]) == {"dips/src/gpu/shaders/dips_shader.wgsl",
                                    "dips/src/gpu/shaders/pre_compute_shader.wgsl",
                                    "dips_alt/src/dips_compute/shaders/pre_compute_shader.wgsl"}
    assert WMAN["pins"] == {"bounds": "restrict", "store_round": "half_even", "exp_log": "oracle"}
    windows = {c["params"][1] for c in WMAN["compute_state"]}
    assert windows >= set(range(1, 12))
    assert {c["params"][3] for c in WMAN["compute_state"]} == {0, 1, 255}
    assert {c["params"][4] for c in WMAN["compute_state"]} == {0, 1, 2, 3}
    assert {c["num_textures"] for c in WMAN["alt"]} >= {1, 2, 3, 16}
    assert {c["window"] for c in WMAN["alt"]} >= {1, 2, 3, 4, 5, 6, 7, 9, 11}


@pytest.mark.parametrize("case", WMAN["compute_state"], ids=lambda c: c["file"])
def test_c_oracle_reproduces_wgsl_compute_state(case):
    z = _load(case["file"])
    fr = z["frames"]
    outs, some = _run_cs(oracle.ComputeState(*case["params"]), fr, z["ops"].tolist(), fr.shape[2], fr.shape[1])
    assert np.array_equal(some, z["some"])
    assert np.array_equal(outs, z["outputs"]), case["file"]


@pytest.mark.parametrize("case", WMAN["alt"], ids=lambda c: c["file"])
def test_c_oracle_reproduces_wgsl_alt(case):
    z = _load(case["file"])
    fr = z["frames"]
    got = oracle.AltCompute(case["num_textures"], fr.shape[2], fr.shape[1], case["colorize"], case["window"],
                            case["scalar"], case["filter"], case["chroma"]).run(fr, case["markers"])
    assert np.array_equal(got, z["outputs"]), case["file"]


# -- with the reference checkout ---------------------------------------------

@needs_ref
def test_fixture_shader_hashes_match_the_reference():
    for rel, sha in WMAN["shaders"].items():
        assert wgsl_ref.shader_sha256(rel) == sha, f"{rel} changed: regenerate the wgsl_* fixtures"


@needs_ref
@pytest.mark.parametrize("case", [c for c in WMAN["compute_state"] if c["params"][1] <= 7], ids=lambda c: c["file"])
def test_wgsl_compute_state_fixture_regenerates(case):
    z = _load(case["file"])
    fr = z["frames"]
    outs, some = _run_cs(wgsl_ref.ComputeState(*case["params"]), fr, z["ops"].tolist(), fr.shape[2], fr.shape[1])
    assert np.array_equal(some, z["some"]) and np.array_equal(outs, z["outputs"]), case["file"]


@needs_ref
@pytest.mark.parametrize("case", [c for c in WMAN["alt"] if c["window"] <= 7], ids=lambda c: c["file"])
def test_wgsl_alt_fixture_regenerates(case):
    z = _load(case["file"])
    fr = z["frames"]
    got = wgsl_ref.AltCompute(case["num_textures"], fr.shape[2], fr.shape[1], case["colorize"], case["window"],
                              case["scalar"], case["filter"], case["chroma"]).run(fr, case["markers"])
    assert np.array_equal(got, z["outputs"]), case["file"]


@needs_ref
def test_get_intensity_exhaustive_against_the_shader():
    """dips_shader.wgsl:64-82 executed over all 2^24 RGB triples (chroma
    None) and every byte of the selected channel (chroma R / G / B) equals
    the restatement the series and the kernels are built on."""
    from oracle import np_restatement as nr
    r = np.arange(256, dtype=np.uint8)
    g, b = np.meshgrid(r, r, indexing="ij")
    for ri in range(0, 256, 32):
        rgba = np.empty((32, 256, 256, 4), np.uint8)
        rgba[..., 0] = (ri + np.arange(32, dtype=np.uint8))[:, None, None]
        rgba[..., 1] = g
        rgba[..., 2] = b
        rgba[..., 3] = 255
        flat = rgba.reshape(-1, 4)
        got = wgsl_ref.get_intensity(flat, 0)
        want = nr.intensity(flat[:, :3], 0, gray=False)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), ri
    rng = np.random.default_rng(5)
    for chroma in (1, 2, 3):
        px = rng.integers(0, 256, (256 * 64, 4), dtype=np.uint8)
        px[:, chroma - 1] = np.repeat(r, 64)
        got = wgsl_ref.get_intensity(px, chroma)
        assert np.array_equal(got.view(np.uint32), nr.intensity(px[:, :3], chroma, gray=False).view(np.uint32))


@needs_ref
@pytest.mark.parametrize("seed", range(6))
def test_random_compute_state_draws_equal_c_oracle(seed):
    rng = np.random.default_rng(1000 + seed)
    w, h = int(rng.integers(1, 26)), int(rng.integers(1, 20))
    params = (bool(rng.integers(0, 2)), int(rng.integers(1, 5)),
              float(rng.choice([5.0, 3.0, -2.0, 0.5, 40.0, float(rng.uniform(-10, 10))])),
              int(rng.choice([0, 1, 255])), int(rng.integers(0, 4)))
    frames = rng.integers(0, 256, (7, h, w, 4), dtype=np.uint8)
    if seed % 2:
        frames[..., :3] = (frames[..., :3] // 64) * 85  # few levels: ties and repeats
    # a random interleaving: add_texture without a dispatch, repeated
    # dispatches, dispatches before the ring is full
    ops, k = [], 0
    while k < 7:
        if rng.random() < 0.6:
            ops.append(k)
            k += 1
        else:
            ops.append(DISPATCH)
    ops.append(DISPATCH)
    a = _run_cs(wgsl_ref.ComputeState(*params), frames, ops, w, h)
    b = _run_cs(oracle.ComputeState(*params), frames, ops, w, h)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0]), params


@needs_ref
@pytest.mark.parametrize("seed", range(4))
def test_random_alt_draws_equal_c_oracle(seed):
    rng = np.random.default_rng(2000 + seed)
    w, h = int(rng.integers(1, 22)), int(rng.integers(1, 16))
    n_tex = int(rng.choice([1, 2, 3, 4, 6]))
    params = (n_tex, bool(rng.integers(0, 2)), int(rng.integers(1, 4)), float(rng.uniform(1.0, 10.0)),
              int(rng.integers(0, 2)), int(rng.integers(0, 4)))
    frames = rng.integers(0, 256, (9, h, w, 4), dtype=np.uint8)
    markers = sorted(set(int(x) for x in rng.integers(1, 9, 2)))
    a = wgsl_ref.AltCompute(n_tex, w, h, *params[1:]).run(frames, markers)
    b = oracle.AltCompute(n_tex, w, h, *params[1:]).run(frames, markers)
    assert np.array_equal(a, b), (params, markers)


@needs_ref
def test_metal_bounds_policy_zeroes_the_start_texture():
    """under naga's ReadZeroSkipWrite (Metal) the 4-slot
    bubble sort reads a 0 past the end and drops the write, so the upper
    median -- and the start texture -- is 0 wherever every intensity is
    positive; under Restrict it is the true upper median."""
    rng = np.random.default_rng(7)
    w, h = 12, 7
    frames = rng.integers(1, 256, (4, h, w, 4), dtype=np.uint8)
    cs = wgsl_ref.ComputeState(False, 1, 5.0, 255, 0, pins=Pins(bounds="read_zero_skip_write"))
    for f in frames:
        cs.add_texture(w, h, f)
    assert not cs.start_texture()[..., :3].any()
    cs = wgsl_ref.ComputeState(False, 1, 5.0, 255, 0)
    o = oracle.ComputeState(False, 1, 5.0, 255, 0)
    for f in frames:
        cs.add_texture(w, h, f)
        o.add_texture(w, h, f)
    assert np.array_equal(cs.start_texture(), o.start_texture())
    assert cs.start_texture()[..., :3].min() > 0


@needs_ref
@pytest.mark.parametrize("filt", [0, 1])
def test_correctly_rounded_exp_log_moves_bytes_by_at_most_one(filt):
    """WGSL bounds exp / log only by an error; the oracle's deterministic
    algorithms are one choice.  With the correctly rounded f32 results the
    executed shader's bytes differ from the pinned ones by at most 1."""
    rng = np.random.default_rng(11 + filt)
    w, h = 24, 16
    frames = rng.integers(0, 256, (8, h, w, 4), dtype=np.uint8)
    ops = sum(([k, DISPATCH] for k in range(8)), [])
    for k in (5.0, 0.7, 9.0):
        a = _run_cs(wgsl_ref.ComputeState(True, 1, k, filt, 0), frames, ops, w, h)[0]
        b = _run_cs(wgsl_ref.ComputeState(True, 1, k, filt, 0, pins=Pins(exp_log="nearest")), frames, ops, w, h)[0]
        d = np.abs(a.astype(int) - b.astype(int))
        assert d.max() <= 1, k


@needs_ref
def test_dips_opencv_runs_the_same_shaders():
    """dips_opencv's ComputeState (same signatures) compiles
    byte-identical shader files, so the fixtures pin it too."""
    for name in ("dips_shader.wgsl", "pre_compute_shader.wgsl"):
        assert wgsl_ref.shader_sha256("dips_opencv/src/gpu/shaders/" + name) == \
            WMAN["shaders"]["dips/src/gpu/shaders/" + name]
