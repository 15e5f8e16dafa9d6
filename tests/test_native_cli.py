"""The native host program over the C ABI (dips_amd/bin/dips_raw, built by
__graft_entry__.build()): the perform_dips loop on raw RGBA8 files and the
difference series CSV, against the oracle (GPU tests) and its usage / error
behaviour (CPU tests)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "dips_amd", "bin", "dips_raw")


def _run(args, **kw):
    return subprocess.run([BIN] + [str(a) for a in args], capture_output=True, text=True, timeout=120, **kw)


def test_binary_built_and_usage():
    assert os.access(BIN, os.X_OK), "build() makes dips_amd/bin/dips_raw"
    r = _run([])
    assert r.returncode == 1 and "usage" in r.stderr
    r = _run(["series", "x", "0", "4", "rgb8"])
    assert r.returncode == 1  # zero width is a usage error


def test_missing_input_is_an_error(tmp_path):
    r = _run(["callback", tmp_path / "none.rgba", 8, 8, tmp_path / "o.rgba"])
    assert r.returncode == 1 and "cannot map" in r.stderr


def test_ragged_file_is_an_error(tmp_path):
    f = tmp_path / "ragged.rgba"
    f.write_bytes(b"\0" * (8 * 8 * 4 + 3))
    r = _run(["callback", f, 8, 8, tmp_path / "o.rgba"])
    assert r.returncode == 1 and "whole number" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 7])
@pytest.mark.parametrize("colorize,filt,chroma", [(False, "none", "none"), (True, "sigmoid", "green")])
def test_callback_file_matches_oracle(tmp_path, batch, colorize, filt, chroma):
    w, h, n = 64, 40, 23
    frames = np.random.default_rng(batch).integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    src, dst = tmp_path / "in.rgba", tmp_path / "out.rgba"
    frames.tofile(src)
    args = ["callback", src, w, h, dst, "--filter", filt, "--chroma", chroma, "--batch", batch]
    if colorize:
        args.append("--colorize")
    r = _run(args)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(dst, dtype=np.uint8).reshape(n, h, w, 4)
    codes = {"none": 255, "sigmoid": 0}
    chromas = {"none": 0, "green": 2}
    cs = oracle.ComputeState(colorize, 1, 5.0, codes[filt], chromas[chroma])
    want = np.stack([oracle.frame_callback(w, h, f, cs) for f in frames])
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,c", [("rgb8", 3), ("gray8", 1)])
@pytest.mark.parametrize("mode", ["overall", "per-frame"])
def test_series_csv_matches_oracle(tmp_path, fmt, c, mode):
    w, h, n = 96, 40, 17
    frames = oracle.synth(c, w, h, 3, 0, n)
    src = tmp_path / "in.raw"
    frames.tofile(src)
    r = _run(["series", src, w, h, fmt, "--mode", mode, "--tau", 8 / 255, "--chunk", 5])
    assert r.returncode == 0, r.stderr
    rows = [line.split(",") for line in r.stdout.strip().splitlines()[1:]]
    got = np.array([[int(x) for x in row[1:4]] for row in rows], dtype=np.uint64)
    out4, si, _ = oracle.series(frames, mode=0 if mode == "overall" else 1, tau=8 / 255)
    assert np.array_equal(got, out4[:, :3])
    np.testing.assert_allclose([float(row[4]) for row in rows], si, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,n", [(2, 17), (5, 23)])
@pytest.mark.parametrize("mode", ["overall", "per-frame"])
def test_sharded_csv_equals_series_csv(tmp_path, ranks, n, mode):
    """`dips_raw sharded`: N ranks (threads, one handle each) over a loopback
    communicator through dips_diff_series_sharded give the single-handle
    series of the whole file, and the oracle's."""
    w, h = 96, 40
    frames = oracle.synth(3, w, h, 5, 0, n)
    src = tmp_path / "in.raw"
    frames.tofile(src)
    r1 = _run(["series", src, w, h, "rgb8", "--mode", mode, "--tau", 8 / 255])
    rn = _run(["sharded", src, w, h, "rgb8", "--ranks", ranks, "--mode", mode, "--tau", 8 / 255])
    assert r1.returncode == 0 and rn.returncode == 0, r1.stderr + rn.stderr
    assert rn.stdout == r1.stdout
    rows = [line.split(",") for line in rn.stdout.strip().splitlines()[1:]]
    got = np.array([[int(x) for x in row[1:4]] for row in rows], dtype=np.uint64)
    out4, _, _ = oracle.series(frames, mode=0 if mode == "overall" else 1, tau=8 / 255)
    assert np.array_equal(got, out4[:, :3])


def test_sharded_usage():
    r = _run(["sharded", "x", "8", "4", "rgb8"])
    assert r.returncode == 1 and "usage" in r.stderr  # --ranks is required


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["overall", "per-frame"])
def test_sharded_csv_over_rccl_in_one_process(tmp_path, mode):
    """`dips_raw sharded --transport rccl`: the ranks of one process from
    dips_comm_create_all (ncclCommInitAll), rank r on device r -- one rank on
    the one-GPU box -- give the single-handle series."""
    w, h, n = 96, 40, 13
    frames = oracle.synth(3, w, h, 9, 0, n)
    src = tmp_path / "in.raw"
    frames.tofile(src)
    r1 = _run(["series", src, w, h, "rgb8", "--mode", mode])
    rn = _run(["sharded", src, w, h, "rgb8", "--ranks", 1, "--mode", mode, "--transport", "rccl"])
    assert r1.returncode == 0 and rn.returncode == 0, r1.stderr + rn.stderr
    assert rn.stdout == r1.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,transport", [(2, "loopback"), (3, "loopback"), (1, "rccl")])
def test_callback_ranks_equal_one_compute_state(tmp_path, ranks, transport):
    """`dips_raw callback --ranks N`: fresh ComputeStates per rank through
    dips_frame_callback_batch_sharded write the file one ComputeState writes
    (and the oracle's frame_callback)."""
    w, h, n = 48, 32, 23
    frames = np.random.default_rng(40 + ranks).integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    src, one, many = tmp_path / "in.rgba", tmp_path / "one.rgba", tmp_path / "many.rgba"
    frames.tofile(src)
    common = ["--colorize", "--filter", "sigmoid"]
    r1 = _run(["callback", src, w, h, one, "--batch", 5] + common)
    rn = _run(["callback", src, w, h, many, "--ranks", ranks, "--transport", transport] + common)
    assert r1.returncode == 0 and rn.returncode == 0, r1.stderr + rn.stderr
    assert one.read_bytes() == many.read_bytes()
    cs = oracle.ComputeState(True, 1, 5.0, 0, 0)
    want = np.stack([oracle.frame_callback(w, h, f, cs) for f in frames])
    assert np.array_equal(np.fromfile(many, dtype=np.uint8).reshape(n, h, w, 4), want)


@pytest.mark.gpu
def test_callback_ranks_layout_refused(tmp_path):
    w, h, n = 16, 8, 10  # 3 ranks start at 0, 3, 6: before frame 7
    src = tmp_path / "in.rgba"
    np.zeros((n, h, w, 4), dtype=np.uint8).tofile(src)
    r = _run(["callback", src, w, h, tmp_path / "o.rgba", "--ranks", 3])
    assert r.returncode == 2 and "< 7" in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,transport", [(0, None), (3, "loopback"), (8, "loopback"), (1, "rccl")])
def test_alt_file_matches_oracle(tmp_path, ranks, transport):
    """`dips_raw alt`: the dips_alt run_dips_on_file loop over a raw RGBA8
    file with refresh markers, on one handle or sharded over N ranks
    (dips_alt_run_sharded), equals the oracle's loop."""
    w, h, n, markers = 40, 24, 30, [4, 11, 12, 25]
    frames = np.random.default_rng(3).integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    src, dst = tmp_path / "in.rgba", tmp_path / "out.rgba"
    frames.tofile(src)
    args = ["alt", src, w, h, dst, "--markers", ",".join(map(str, markers))]
    if ranks:
        args += ["--ranks", ranks, "--transport", transport]
    r = _run(args)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(dst, dtype=np.uint8).reshape(n, h, w, 4)
    want = oracle.AltCompute(2, w, h, True, 1, 5.0, 0, 0).run(frames, markers)
    assert np.array_equal(got, want)


def test_alt_usage():
    for bad in (["alt", "x", "8", "4"], ["alt", "x", "8", "4", "o", "--markers", "1,,2"],
                ["alt", "x", "8", "4", "o", "--transport", "mpi"]):
        r = _run(bad)
        assert r.returncode == 1 and "usage" in r.stderr, bad
