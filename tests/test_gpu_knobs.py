"""GPU parity of the non-default values of the library's environment knobs
that are read once per process (INTEGRATION.md "Environment knobs"):
DIPS_COPY_THREADS (1: no worker thread, the calling thread runs every copy
task; 3) and DIPS_POOL_SPIN_US (0: workers park at once).  Each runs in a
child process (the pool is built at its first use) over the per-frame call
paths the pool serves -- the zero-copy ComputeState frame_callback, the
deferred add_texture + dispatch, the host-fed batch and the dips_alt
send_frame -- and every output must equal the oracle's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle
from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
from dips_amd.alt import DiPsCompute, DiPsProperties
w, h = 256, 192  # 5 row stripes per frame
rng = np.random.default_rng(5)
frames = rng.integers(0, 256, (16, h, w, 4), dtype=np.uint8)
frames[6] = frames[5]
bad = 0
cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
ref = oracle.ComputeState(True, 1, 5.0, 0, 0)
threads = None
try:
    for k in range(10):
        bad += not np.array_equal(frame_callback(w, h, frames[k], cs), oracle.frame_callback(w, h, frames[k], ref))
        ph = cs.callback_phases()
        if ph:
            threads = int(ph["threads"])
    for k in range(10, 12):
        cs.add_texture(w, h, frames[k]); ref.add_texture(w, h, frames[k])
        bad += not np.array_equal(cs.dispatch(), ref.dispatch())
    got = cs.frame_callback_batch(w, h, frames[12:])
    want = np.stack([oracle.frame_callback(w, h, f, ref) for f in frames[12:]])
    bad += not np.array_equal(got, want)
finally:
    cs.close()
c = DiPsCompute(2, h, w, DiPsProperties())
aref = oracle.AltCompute(2, w, h)
try:
    for k in range(8):
        bad += not np.array_equal(c.send_frame(frames[k], True if k == 2 else None), aref.send_frame(frames[k], k == 2))
finally:
    c.close()
print(json.dumps({"bad": int(bad), "threads": threads}))
'''


@pytest.mark.parametrize("env", [{"DIPS_COPY_THREADS": "1"}, {"DIPS_COPY_THREADS": "3"},
                                 {"DIPS_POOL_SPIN_US": "0"}])
def test_copy_pool_knobs_match_oracle(env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, env=e, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["bad"] == 0, res
    if "DIPS_COPY_THREADS" in env:
        assert res["threads"] == int(env["DIPS_COPY_THREADS"]), res  # the pool the calls ran on
