"""RCCL on the hardware at world size 1 (tests/_rccl_world1.py in a child
process): init with device_id, broadcast of a uint8 frame, a uint8 halo by
send / recv to self, gather / all_gather of an int64 series, all_reduce,
all_gather_object, barrier -- every collective the N > 1 bench path issues,
on its dtypes.  RCCL refuses two ranks on one GPU, so this is as far as a
one-GPU box can take the RCCL leg; the multi-rank logic is covered by the
gloo tests (tests/test_dist_cpu.py, tests/test_gpu_bench_rehearsal.py)."""
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


def test_rccl_collectives_world1():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_rccl_world1.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=110)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    out = json.loads(lines[-1])
    assert out["ok"], out
