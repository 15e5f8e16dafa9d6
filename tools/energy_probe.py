#!/usr/bin/env python3
"""energy_probe.py -- energy per wave64 VALU instruction by class (gfx950),
from build/ebench (tools/gen_ebench.py) and the amdsmi energy counter
(tools/power_probe.py's sampler; read-only queries).

Per class: average socket power over the class's window (the first 30 %
skipped as ramp), minus the idle power measured before, times the window,
over the wave64 instructions executed in it.  Prints one JSON line per class.
Run on the GPU box:  python tools/energy_probe.py [seconds_per_class]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from power_probe import Sampler  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    smp = Sampler()
    smp.start()
    t0 = time.monotonic()
    time.sleep(2.0)
    idle = smp.window(t0 + 0.5, time.monotonic())[0]
    p_idle = idle["avg_power_W_energy"]
    print(json.dumps({"phase": "idle", "gpu": idle}), flush=True)
    r = subprocess.run([os.path.join(ROOT, "build", "ebench"), str(secs)], capture_output=True, text=True,
                       timeout=60 + 40 * secs)
    smp.stop_ev.set()
    smp.join(timeout=2)
    for line in r.stdout.splitlines():
        if not line.startswith("class\t"):
            continue
        _, name, a, b, n = line.split("\t")
        a, b, n = float(a), float(b), float(n)
        dt = b - a
        w0 = a + 0.3 * dt
        g = smp.window(w0, b)[0]
        frac = (b - w0) / dt
        p = g["avg_power_W_energy"] if g else None
        row = {"class": name, "seconds": round(dt, 2), "wave_instr_per_s": n / dt, "gpu": g}
        if p is not None and p_idle is not None:
            row["pJ_per_wave64_instr_above_idle"] = round((p - p_idle) * (b - w0) / (n * frac) * 1e12, 1)
            row["pJ_per_lane_op_above_idle"] = round(row["pJ_per_wave64_instr_above_idle"] / 64.0, 2)
        print(json.dumps(row), flush=True)
    if r.returncode != 0:
        print(r.stderr[-2000:], file=sys.stderr)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
