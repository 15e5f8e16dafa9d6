"""bench.py's N > 1 path rehearsed on the one GPU of a test box: two ranks
on device 0 over gloo, RCCL itself refusing two ranks on one GPU.

The native path (the default): each step is one dips_diff_series_sharded
call per rank, the library's own sharding -- halo exchange, the series
launches, the gather of the series -- over the DIPS_COMM_HOST transport
backed by the gloo group (dips_amd.comm.TorchHostTransport); the driver's
run is the same call over an RCCL communicator.  The torch path
(DIPS_BENCH_SHARD=torch) is the older Python-level protocol of
dips_amd.shard with gloo moving device tensors.  Both run the configs[3] /
configs[4] legs and the self-check, exactly as the driver's run does.

2560x1440 RGB8, 300 frames per rank: rank 1's (F - 1)-frame launch beside
the halo runs the part-major schedule.  The gathered series is dumped and
compared with the CPU oracle on every shard-boundary frame and a seeded
sample; `--check` makes rank 0 compare the gather with one single-device
launch over all 600 frames too.  A damaged halo must make the run exit
non-zero with "equal": false in its line, on either path."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle
from _sched import library_schedule

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

W, H, F, WORLD = 2560, 1440, 300, 2
SEED = 0xD1B5  # bench.py SEED
TAU = 8.0 / 255.0


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(mode, corrupt, dump=None, frames=F, width=W, height=H, extra=(), env_extra=None, path="native",
         world=WORLD):
    env = dict(os.environ, DIPS_BENCH_BACKEND="gloo", DIPS_BENCH_ONE_DEVICE="1", DIPS_BENCH_SHARD=path,
               DIPS_BENCH_CORRUPT_HALO="1" if corrupt else "0", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--frames-per-gpu", str(frames),
           "--width", str(width), "--height", str(height), "--mode", mode,
           "--leg-steps", "1", "--no-cpu-baseline", "--no-pcie", "--no-map", "--no-per-frame-call",
           "--dist-timeout", "120", *extra]
    if dump:
        cmd += ["--dump-series", dump]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr[-4000:]


def _oracle_rows(picks, n_total, per_frame, w, h):
    """Oracle series rows of global frames `picks` of the bench's synthetic
    clip (oracle.synth is the shared generator): 'per-frame' row g from
    frames (g - 1, g) (row 0 against itself), 'overall' against frame 0."""
    rows = []
    f0 = oracle.synth(3, w, h, SEED, 0, 1)
    for g in picks:
        if per_frame:
            fr = f0 if g == 0 else oracle.synth(3, w, h, SEED, g - 1, 2)
            out4, _, _ = oracle.series(fr, mode=1, tau=TAU, nthreads=16)
        else:
            fr = oracle.synth(3, w, h, SEED, g, 1)
            out4, _, _ = oracle.series(fr, mode=0, tau=TAU, ref=f0[0], nthreads=16)
        rows.append(out4[-1])
    return np.stack(rows)


def _picks(n_total, world, n_random=6):
    from dips_amd import shard
    return shard.check_frames(n_total, world, n_random=n_random, seed=0xBEEF)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode,path", [("per-frame", "native"), ("overall", "native"), ("per-frame", "torch")])
def test_bench_two_ranks_rehearsal(mode, path, tmp_path):
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    if mode == "per-frame":
        # the schedule of rank 1's (F - 1)-frame launch: part-major, >= 2 parts
        op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, TAU)
        try:
            sch = library_schedule(op, W, H, F - 1)
        finally:
            op.close()
        assert sch is not None and sch[1] >= 2, sch
    dump = str(tmp_path / "series.npy")
    rc, line, err = _run(mode, corrupt=False, dump=dump, extra=("--check",), path=path)
    assert rc == 0, err
    assert line["n_gpus"] == WORLD and line["ranks"] == WORLD and len(line["devices"]) == WORLD, line
    assert "rehearsal" in line["config"]["parallelism"]
    assert line["shard_path"]["path"] == path, line["shard_path"]
    if path == "native":
        assert "dips_diff_series_sharded" in line["config"]["parallelism"]
        assert line["shard_path"]["transport"].startswith("host (gloo")
    assert "--check: gathered series" in err
    assert line["check"]["equal"] is True and line["check"]["frames_checked"] >= 12
    for key in ("configs3", "configs4"):
        assert "failed" not in line[key], line[key]
        assert line[key]["check"]["equal"] is True, line[key]
    # the gathered series against the oracle at every shard boundary
    got = np.load(dump)
    n_total = WORLD * F
    assert got.shape == (n_total, 4)
    picks = _picks(n_total, WORLD)
    want = _oracle_rows(picks, n_total, mode == "per-frame", W, H)
    bad = [g for g, a, b in zip(picks, got[picks], want) if not np.array_equal(a, b)]
    assert not bad, f"gathered rows differing from the oracle: {bad}"
    # configs[3]: the same ranks, 'overall' against the broadcast frame 0
    leg = np.load(str(tmp_path / "series_configs3.npy"))
    assert leg.shape == (n_total, 4)
    lp = _picks(n_total, WORLD, n_random=2)
    assert np.array_equal(leg[lp], _oracle_rows(lp, n_total, False, W, H))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("path", ["native", "torch"])
def test_bench_two_ranks_damaged_halo_fails(path):
    rc, line, err = _run("per-frame", corrupt=True, frames=24, width=640, height=360, path=path)
    assert rc != 0
    assert line is not None and line["check"]["equal"] is False, (line, err)
    assert line["shard_path"]["path"] == path


@pytest.mark.timeout(300)
def test_bench_rank_failure_exits_nonzero_with_device():
    """An exception on one rank (DIPS_BENCH_FAIL_RANK, injected right after
    the process group is up) ends the job with a non-zero status and a report
    naming the rank and its device's PCI bus id; the other rank, left in its
    first collective, fails at --dist-timeout instead of hanging."""
    rc, line, err = _run("per-frame", corrupt=False, frames=24, width=640, height=360,
                         extra=("--dist-timeout", "20"), env_extra={"DIPS_BENCH_FAIL_RANK": "1"})
    assert rc != 0
    assert line is None
    assert "FAILED on rank 1" in err and "PCI" in err, err


@pytest.mark.timeout(600)
def test_bench_three_ranks_native(tmp_path):
    """Three ranks: the middle one both receives and sends a halo; the
    gathered series against the oracle at both shard boundaries."""
    dump = str(tmp_path / "s3.npy")
    w, h, f = 640, 360, 40
    rc, line, err = _run("per-frame", corrupt=False, dump=dump, frames=f, width=w, height=h, world=3,
                         extra=("--check", "--no-legs"))
    assert rc == 0, err
    assert line["n_gpus"] == 3 and line["check"]["equal"] is True and line["shard_path"]["path"] == "native"
    got = np.load(dump)
    picks = _picks(3 * f, 3)
    assert np.array_equal(got[picks], _oracle_rows(picks, 3 * f, True, w, h))
