"""bench.py's JSON line against the driver's contract, at N = 1 on a small
shape (the default shape is what the driver runs; this checks the line's
form, not its number): every required key with its type, value = frames /
step time, roofline.frac = achieved / peak with the guide's 8 TB/s HBM peak,
a cpu_baseline of kind "port" with its core count and sample, the self-check
passed, the batch's placement report, and one JSON line on stdout."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

W, H, F, STEPS = 1280, 720, 300, 3


def test_bench_line_keeps_the_contract():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        baseline = json.load(f)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(STEPS), "--warmup", "1",
           "--frames-per-gpu", str(F), "--width", str(W), "--height", str(H), "--cpu-seconds", "0.5",
           "--no-pcie", "--no-map", "--no-tau0", "--no-legs", "--no-per-frame-call"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["metric"] == baseline["metric"]
    assert d["unit"] == "frames/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["n_gpus"] == 1 and d["steps"] == STEPS and d["warmup"] == 1
    assert d["vs_baseline"] is None and not baseline["published"]
    assert d["dtype"] == "u8" and "synthetic" in d["data"]
    assert isinstance(d["config"], dict) and "workload" in d["config"] and "model" not in d["config"]
    assert d["value"] == pytest.approx(F / (d["ms_per_step"] / 1e3), rel=2e-3)
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-4)
    assert r["achieved"] == pytest.approx(F * W * H * 3 / (r["kernel_ms"] / 1e3) / 1e9, rel=2e-3)
    assert "traffic" in r and (r["traffic"] is None or r["traffic"] > 0)
    assert r["kernel_launches_timed"] == STEPS
    c = d["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["unit"] == "frames/s"
    assert isinstance(c["cores"], int) and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    assert c["series_matches_gpu"] is True
    assert d["check"]["equal"] is True
    # the batch's placement: both candidates timed alternately, the plain one
    # kept unless the other is faster by more than the threshold
    # (tools/placement.py), and the plain allocation's rate in the roofline
    from tools.placement import choose
    pl = d["placement"]
    assert isinstance(pl, list) and len(pl) == 1 and pl[0]["probe"] is True
    ms = pl[0]["candidate_kernel_ms"]
    assert len(ms) == 2 and pl[0]["kept"] == choose(ms[0], ms[1], pl[0]["threshold"])[0]
    assert r["plain_kernel_ms"] == pytest.approx(ms[0], abs=1e-4)
    assert r["plain_frac"] == pytest.approx(F * W * H * 3 / (ms[0] / 1e3) / 1e9 / 8000.0, rel=2e-3)
