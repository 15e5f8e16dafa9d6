#!/usr/bin/env python3
"""policy_energy.py -- frames/s and energy per frame of the series kernel
for each frame-load cache policy (build/policy_<aux>, tools/policy_probe.hip),
run one after another in two alternated rounds while tools/power_probe.py's
sampler reads the energy counter (read-only).  One JSON line per run.
Run on the GPU box:  python tools/policy_energy.py [seconds] [aux,aux,...]
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

FB = 3840 * 2160 * 3


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
    auxes = (sys.argv[2] if len(sys.argv) > 2 else "2,0,1,3,16,18").split(",")
    smp = Sampler()
    smp.start()
    order = auxes + auxes[::-1]
    for k, aux in enumerate(order):
        exe = os.path.join(ROOT, "build", f"policy_{aux}")
        r = subprocess.run([exe, "2000", str(secs)], capture_output=True, text=True, timeout=120 + 2 * secs)
        line = [l for l in r.stdout.splitlines() if l.startswith("run\t")]
        if r.returncode != 0 or not line:
            print(json.dumps({"aux": aux, "rc": r.returncode, "err": r.stderr[-500:]}), flush=True)
            sys.exit(1)
        _, a, t0, t1, launches, frames, med, ck = line[0].split("\t")
        t0, t1 = float(t0), float(t1)
        dt = t1 - t0
        g = smp.window(t0 + 0.3 * dt, t1)[0]
        fps = 1000.0 * int(frames) / float(med)
        row = {"aux": int(a), "round": 1 + k // len(auxes), "kernel_ms_median": float(med),
               "frames_per_s": round(fps, 1), "frac_of_8TBps": round(fps * FB / 1e9 / 8000, 4),
               "series_checksum": ck, "gpu": g}
        if g and g.get("avg_power_W_energy"):
            row["mJ_per_frame"] = round(g["avg_power_W_energy"] / fps * 1e3, 4)
        print(json.dumps(row), flush=True)
        time.sleep(1.0)
    smp.stop_ev.set()
    smp.join(timeout=2)


if __name__ == "__main__":
    main()
