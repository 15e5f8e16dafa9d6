#!/usr/bin/env python3
"""walk_energy.py -- runs build/walk_energy (tools/walk_energy.hip) while
tools/power_probe.py's sampler reads the amdsmi energy counter (read-only);
prints per run the rate, power, clock, PPT residency and energy per frame.
Run on the GPU box:  python tools/walk_energy.py [--bin build/<probe>] [args of the probe]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from power_probe import Sampler  # noqa: E402

FB = 3840 * 2160 * 3


def main():
    argv = sys.argv[1:]
    exe = os.path.join(ROOT, "build", "walk_energy")
    if argv[:1] == ["--bin"]:
        exe, argv = os.path.join(ROOT, argv[1]), argv[2:]
    args = argv or ["2000", "4", "2", "128"]
    smp = Sampler()
    smp.start()
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=600)
    smp.stop_ev.set()
    smp.join(timeout=2)
    for line in r.stdout.splitlines():
        p = line.split("\t")
        if p[0] != "run":
            continue
        rnd, name, t0, t1, med, frac, F = int(p[1]), p[2], float(p[3]), float(p[4]), float(p[5]), float(p[6]), int(p[7])
        dt = t1 - t0
        g = smp.window(t0 + 0.3 * dt, t1)[0]
        fps = F / (med / 1e3)
        row = {"round": rnd, "schedule": name, "kernel_ms_median": med, "frac_of_8TBps": frac, "frames_per_s": round(fps, 1),
               "gpu": g, "args": args}
        if g and g.get("avg_power_W_energy"):
            row["mJ_per_frame"] = round(g["avg_power_W_energy"] / fps * 1e3, 4)
        print(json.dumps(row), flush=True)
    if r.returncode != 0:
        print(r.stderr[-1000:], file=sys.stderr)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
