"""CPU tests of the C-ABI boundary (no GPU compute): the library builds for
gfx950, loads, exports every function include/dips_hip.h declares, fills the
reference defaults and refuses bad parameters before touching a device."""
import ctypes
import os
import re
import subprocess

import pytest

from dips_amd import _lib
from dips_amd._lib import DipsParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_header_functions_exported():
    lib = _lib.load()
    names = _lib.header_functions()
    assert len(names) >= 18
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    hdr = open(os.path.join(ROOT, "include", "dips_hip.h")).read()
    want = int(re.search(r"#define DIPS_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.dips_abi_version() == want == _lib.ABI_VERSION  # the binding refuses any other library


def test_rust_crate_binds_every_entry_point():
    """The Rust crate's extern block (rust/dips-hip/src/ffi.rs) names every
    function the header declares; tests/test_rust_shim.py checks the types."""
    with open(os.path.join(ROOT, "rust", "dips-hip", "src", "ffi.rs")) as f:
        src = f.read()
    missing = [n for n in _lib.header_functions() if f"pub fn {n}(" not in src]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob  # the embedded code-object bundle


def test_params_default_matches_reference():
    """DiPsProperties::new() defaults, dips/src/lib.rs:74-86."""
    p = DipsParams()
    assert _lib.load().dips_params_default(ctypes.byref(p)) == 0
    assert p.colorize == 0
    assert p.spatial_window_size == 1
    assert abs(p.sensitivity - 5.0) < 1e-7
    assert p.filter_type == 255  # Unfiltered (lib.rs:36)
    assert p.chroma_filter == 0
    assert p.mode == 0 and p.format == 3 and p.tau == 0.0


@pytest.mark.parametrize("field,value", [("spatial_window_size", 0), ("spatial_window_size", 12),
                                         ("chroma_filter", 4), ("mode", 2), ("format", 2),
                                         ("tau", -1.0), ("tau", float("inf")), ("sensitivity", float("nan"))])
def test_create_rejects_bad_params(field, value):
    lib = _lib.load()
    p = DipsParams()
    lib.dips_params_default(ctypes.byref(p))
    setattr(p, field, value)
    h = ctypes.c_void_p()
    assert lib.dips_create(ctypes.byref(p), 0, ctypes.byref(h)) == _lib.DIPS_ERR_INVALID
    assert not h.value
    assert lib.dips_last_error(None)


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device error path")
def test_create_without_device_fails_cleanly():
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.dips_create(None, 0, ctypes.byref(h)) == _lib.DIPS_ERR_NODEVICE
    assert b"no HIP device" in lib.dips_last_error(None)
    from dips_amd import ComputeState, DiPsFilter, ChromaFilter, DipsError
    with pytest.raises(DipsError):
        ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)


def test_null_handle_calls_are_safe():
    lib = _lib.load()
    assert lib.dips_add_texture(None, 1, 1, None, 4) == _lib.DIPS_ERR_INVALID
    assert lib.dips_dispatch(None, None, 0) == _lib.DIPS_ERR_INVALID
    assert lib.dips_diff_series(None, 1, 1, None, 1, None, None, None) == _lib.DIPS_ERR_INVALID
    lib.dips_destroy(None)
    e = _lib.SeriesEntry(1, 2, 3, 1 << 32)
    assert lib.dips_series_si(ctypes.byref(e)) == 1.0


def test_header_cites_reference_interfaces():
    """Every entry point that replaces a reference interface names it."""
    text = open(os.path.join(ROOT, "include", "dips_hip.h")).read()
    for cite in ["dips/src/gpu/mod.rs:59", "dips/src/gpu/mod.rs:170", "dips/src/gpu/mod.rs:306",
                 "dips/src/lib.rs:233", "dips/src/lib.rs:23"]:
        assert cite.split(":")[0] in text
    assert re.search(r"ComputeState::new", text) and re.search(r"ComputeState::dispatch", text)


def test_product_has_no_oracle_dependency():
    """The product package must not import or link the oracle."""
    pkg = os.path.join(ROOT, "dips_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, fn)).read()
                assert "dips_oracle" not in src and "from oracle" not in src and "import oracle" not in src, fn
    ldd = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd
