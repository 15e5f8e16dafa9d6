"""The HIP path against the wgsl_* fixtures: outputs of the reference's own
shader files executed on the CPU (oracle/wgsl_exec.py, host side restated in
oracle/wgsl_ref.py, tests/golden/make_wgsl_golden.py), so the device output
is compared with the shader text's result, not with a restatement of it.

Every fixture runs through the C ABI in each form the product has:
ComputeState's add_texture / dispatch sequence (repeated dispatches and
add_texture without a dispatch included), the same with the plain kernels
(DIPS_FLAG_CROSSCHECK), and -- for the frame_callback sequences -- the
one-pass dips_frame_callback_batch; the dips_alt loop through dips_alt_run
(plain and crosscheck) and dips_alt_send_frames with run_dips_on_file's
snapshot flags."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "wgsl_manifest.json")) as _f:
    WMAN = json.load(_f)

DISPATCH = -1


def _load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _is_callback_sequence(ops):
    return ops == sum(([k, DISPATCH] for k in range(len(ops) // 2)), [])


@pytest.mark.gpu
@pytest.mark.parametrize("crosscheck", [False, True], ids=["default", "crosscheck"])
@pytest.mark.parametrize("case", WMAN["compute_state"], ids=lambda c: c["file"])
def test_compute_state_matches_executed_shaders(case, crosscheck):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    z = _load(case["file"])
    fr, ops = z["frames"], z["ops"].tolist()
    h, w = fr.shape[1], fr.shape[2]
    colorize, window, sens, filt, chroma = case["params"]
    cs = ComputeState(colorize, window, sens, DiPsFilter(filt), ChromaFilter(chroma), crosscheck=crosscheck)
    try:
        outs, some = [], []
        for op in ops:
            if op == DISPATCH:
                o = cs.dispatch()
                some.append(o is not None)
                if o is not None:
                    outs.append(o)
            else:
                cs.add_texture(w, h, fr[op])
    finally:
        cs.close()
    assert some == z["some"].tolist(), case["file"]
    got = np.stack(outs) if outs else np.zeros((0, h, w, 4), np.uint8)
    assert np.array_equal(got, z["outputs"]), (case["file"], np.argwhere(got != z["outputs"])[:4])


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in WMAN["compute_state"]], ids=lambda c: c["file"])
def test_frame_callback_batch_matches_executed_shaders(case):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    z = _load(case["file"])
    fr, ops = z["frames"], z["ops"].tolist()
    if not _is_callback_sequence(ops):
        pytest.skip("not a frame_callback sequence")
    h, w = fr.shape[1], fr.shape[2]
    colorize, window, sens, filt, chroma = case["params"]
    cs = ComputeState(colorize, window, sens, DiPsFilter(filt), ChromaFilter(chroma))
    try:
        got = cs.frame_callback_batch(w, h, fr)
    finally:
        cs.close()
    # frames 0..2 pass through (dips/src/lib.rs:241-245), then the dispatches
    assert np.array_equal(got[:3], fr[:3])
    assert np.array_equal(got[3:], z["outputs"]), (case["file"], np.argwhere(got[3:] != z["outputs"])[:4])


def _alt_props(case):
    from dips_amd.alt import ChromaFilter, DiPsProperties
    return DiPsProperties(colorize=case["colorize"], window_size=case["window"],
                          sigmoid_horizontal_scalar=case["scalar"], filter_type=case["filter"],
                          chroma_filter=ChromaFilter(case["chroma"]))


@pytest.mark.gpu
@pytest.mark.parametrize("crosscheck", [False, True], ids=["default", "crosscheck"])
@pytest.mark.parametrize("case", WMAN["alt"], ids=lambda c: c["file"])
def test_alt_run_matches_executed_shaders(case, crosscheck):
    from dips_amd.alt import DiPsRunner
    z = _load(case["file"])
    fr = z["frames"]
    r = DiPsRunner(fr.shape[1], fr.shape[2], _alt_props(case), case["markers"],
                   num_textures=case["num_textures"], crosscheck=crosscheck)
    try:
        got = r(fr)
    finally:
        r.close()
    assert np.array_equal(got, z["outputs"]), (case["file"], np.argwhere(got != z["outputs"])[:4])


@pytest.mark.gpu
@pytest.mark.parametrize("case", WMAN["alt"], ids=lambda c: c["file"])
def test_alt_send_frames_matches_executed_shaders(case):
    from dips_amd.alt import DiPsCompute, run_loop_flags
    z = _load(case["file"])
    fr = z["frames"]
    c = DiPsCompute(case["num_textures"], fr.shape[1], fr.shape[2], _alt_props(case))
    try:
        got = c.send_frames(fr, run_loop_flags(fr.shape[0], case["markers"]))
    finally:
        c.close()
    assert np.array_equal(got, z["outputs"]), (case["file"], np.argwhere(got != z["outputs"])[:4])
