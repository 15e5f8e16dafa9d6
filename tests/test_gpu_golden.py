"""The HIP path against the committed golden fixtures (tests/golden/, made by
make_golden.py from the numpy restatement and accepted only where the C
oracle agrees).  Every fixture runs through the C ABI: the difference series
(dips_diff_series, with and without a reference frame), the dips
ComputeState (add_texture / dispatch, dips/src/gpu/mod.rs:170-397) and the
dips_alt run loop (dips_alt/src/lib.rs:588-683)."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "manifest.json")) as _f:
    MANIFEST = json.load(_f)


def _load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST["series"], ids=lambda c: c["file"])
def test_series_fixture(case):
    from dips_amd import ChromaFilter, DiffSeriesOperator, Mode, PixelFormat
    z = _load(case["file"])
    fmt = {1: PixelFormat.Gray8, 3: PixelFormat.RGB8, 4: PixelFormat.RGBA8}[case["channels"]]
    # the shape picks the fast kernel (64x48) or the generic one (37x23);
    # force_generic runs the generic kernel on the fast shapes as well, and
    # the map / no-map launches are separate kernel instantiations
    for generic in (False, True):
        op = DiffSeriesOperator(fmt, Mode(case["mode"]), case["tau"], ChromaFilter(case["chroma"]),
                                force_generic=generic)
        try:
            got, dmap = op(z["frames"], ref=z.get("ref"), want_map=True)
            got_nomap, _ = op(z["frames"], ref=z.get("ref"))
        finally:
            op.close()
        for g in (got, got_nomap):
            assert np.array_equal(g.as_array(), z["out4"]), (case["file"], generic)
            np.testing.assert_allclose(g.si, z["si"], rtol=0, atol=1e-6)
        assert np.array_equal(dmap, z["dmap"]), (case["file"], generic)


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST["compute_state"], ids=lambda c: c["file"])
def test_compute_state_fixture(case):
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    z = _load(case["file"])
    colorize, window, sens, filt, chroma = case["params"]
    cs = ComputeState(colorize, window, sens, DiPsFilter(filt), ChromaFilter(chroma))
    try:
        outs = []
        for k, fr in enumerate(z["frames"]):
            cs.add_texture(fr.shape[1], fr.shape[0], fr)
            o = cs.dispatch()
            assert (o is None) == (k < 3)
            if o is not None:
                outs.append(o)
    finally:
        cs.close()
    assert np.array_equal(np.stack(outs), z["outputs"]), case["file"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST["alt"], ids=lambda c: c["file"])
def test_alt_fixture(case):
    from dips_amd.alt import ChromaFilter, DiPsProperties, DiPsRunner
    z = _load(case["file"])
    fr = z["frames"]
    props = DiPsProperties(colorize=case["colorize"], window_size=case["window"],
                           sigmoid_horizontal_scalar=case["scalar"], filter_type=case["filter"],
                           chroma_filter=ChromaFilter(case["chroma"]))
    r = DiPsRunner(fr.shape[1], fr.shape[2], props, case["markers"], num_textures=case["num_textures"])
    try:
        got = r(fr)
    finally:
        r.close()
    assert np.array_equal(got, z["outputs"]), (case["file"], np.argwhere(got != z["outputs"])[:4])
