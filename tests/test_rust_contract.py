"""The Rust crate's failure contract executed: cargo is
absent here, so tests/rust_contract.cpp restates every method of
rust/dips-hip/src/lib.rs -- the same FFI calls in the same order, the same
argument checks and status handling -- and runs it against the built
libdips_hip.so.  tests/test_rust_shim.py::test_crate_method_table maps each
crate method to its C entry point, its status handling and the rows below.

* CPU (no device): ComputeState::new, DiffSeries::new, DiPsCompute::new and
  Comm::loopback return Err(DIPS_ERR_NODEVICE) with the library's message.
* GPU: the warm-up gives Ok(None) (status 0) for frames 0..2; a negative
  status reaches the caller with dips_last_error set; a size change returns
  < 0 with the output untouched and makes the panicking frame_callback panic
  instead of passing the input through; add_texture swallows what
  try_add_texture reports; DiffSeries run / run_streamed / run_sharded
  (3 loopback ranks on threads) agree; the crate-side refusals fire before
  the library is called.
Reference: dips/src/gpu/mod.rs:59-65, :170-216, :306-397; dips/src/lib.rs:233-246."""
import os
import re
import subprocess

import pytest

from dips_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "rust_contract.cpp")


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def _build(tmp_path):
    exe = tmp_path / "rust_contract"
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-pthread", "-I", os.path.join(ROOT, "include"), SRC,
                    "-o", str(exe), "-L", libdir, "-ldips_hip", f"-Wl,-rpath,{libdir}",
                    "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    return exe


def _rows(out):
    return dict(re.findall(r"^ROW (\w+) (ok|FAIL.*)$", out, flags=re.M))


def contract_rows():
    """Every row name the harness can print."""
    return set(re.findall(r'row\("(\w+)"', open(SRC).read()))


@pytest.mark.skipif(_has_gpu(), reason="the no-device rows")
def test_contract_without_device(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    rows = _rows(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert set(rows) == {"check_abi", "new", "comm_loopback", "diff_series_new", "dips_compute_new"}, rows
    assert all(v == "ok" for v in rows.values()), rows


@pytest.mark.gpu
def test_contract_on_device(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([str(exe), "--device"], capture_output=True, text=True, timeout=300)
    rows = _rows(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert all(v == "ok" for v in rows.values()), rows
    # every row the harness defines ran
    assert set(rows) == contract_rows(), contract_rows() - set(rows)
