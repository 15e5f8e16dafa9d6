"""bench.py's N > 1 path rehearsed on the one GPU of a test box: two ranks
over gloo (which moves device tensors for every collective the step uses on
this torch build, tools/gloo_cuda_probe.py) on device 0 -- the halo
send/recv of device tensors beside the persistent series kernel under the
4-wave cap, the gather, the configs[3] / configs[4] legs and the
self-check, exactly as the driver's RCCL run executes them; RCCL itself
refuses two ranks on one GPU.  A damaged halo must make the run exit
non-zero with "equal": false in its line."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(mode, corrupt):
    env = dict(os.environ, DIPS_BENCH_BACKEND="gloo", DIPS_BENCH_ONE_DEVICE="1",
               DIPS_BENCH_CORRUPT_HALO="1" if corrupt else "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--frames-per-gpu", "24", "--mode", mode,
           "--leg-steps", "1", "--no-cpu-baseline", "--no-pcie", "--no-map", "--no-per-frame-call"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr[-3000:]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["per-frame", "overall"])
def test_bench_two_ranks_rehearsal(mode):
    rc, line, err = _run(mode, corrupt=False)
    assert rc == 0, err
    assert line["n_gpus"] == 2 and line["ranks"] == 2 and len(line["devices"]) == 2, line
    assert "rehearsal" in line["config"]["parallelism"]
    assert line["check"]["equal"] is True and line["check"]["frames_checked"] >= 12
    for key in ("configs3", "configs4"):
        assert "failed" not in line[key], line[key]
        assert line[key]["check"]["equal"] is True, line[key]


@pytest.mark.timeout(600)
def test_bench_two_ranks_damaged_halo_fails():
    rc, line, err = _run("per-frame", corrupt=True)
    assert rc != 0
    assert line is not None and line["check"]["equal"] is False, (line, err)
