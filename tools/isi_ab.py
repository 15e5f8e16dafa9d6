#!/usr/bin/env python3
"""isi_ab.py -- variants of the RGB8 series kernel, named in argv[5]
(default "isi,f64"): the integer intensity sum (series_v2.hip ISI = 1, the
default for tau >= 2^-5), the f64 sum (ISI = 0, DIPS_FLAG_CROSSCHECK), and
"wN" = the default form with DIPS_SERIES_WAVES_PER_SIMD=N -- alternated in ONE
process over ONE resident buffer of the headline workload (5000 4K RGB8
frames, 'per-frame', tau 8/255): kernel time by the library's hipEvents,
socket energy and PPT residency from the SMU read right before and after
each variant's steps (tools/power_probe.py, no polling thread), series of
all variants compared.  One JSON line per (round, variant), then a summary.

Usage: python tools/isi_ab.py [frames] [steps] [rounds] [per-frame|overall] [variants] [WxH]"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    W, H = (int(v) for v in (sys.argv[6] if len(sys.argv) > 6 else "3840x2160").split("x"))
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    mode = Mode.PerFrame if (len(sys.argv) <= 4 or sys.argv[4] == "per-frame") else Mode.Overall
    names = (sys.argv[5] if len(sys.argv) > 5 else "isi,f64").split(",")
    ops = {k: DiffSeriesOperator(PixelFormat.RGB8, mode, 8 / 255, time_kernel=True, crosscheck=(k == "f64"))
           for k in names}
    frames = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
    ops[names[0]].synth_device(frames, W, H, 0xD1B5, 0)
    ref = frames[0].clone()
    series = {k: torch.zeros((F, 4), dtype=torch.int64, device="cuda") for k in names}
    torch.cuda.synchronize()
    smp = None
    try:
        from power_probe import Sampler
        smp = Sampler(pci_bus=torch.cuda.get_device_properties(0).pci_bus_id)
        if len(smp.handles) != 1:
            smp = None
    except Exception:
        smp = None
    res = {}
    for rnd in range(rounds):
        for name in (names if rnd % 2 == 0 else names[::-1]):
            os.environ.pop("DIPS_SERIES_WAVES_PER_SIMD", None)
            if name.startswith("w"):
                os.environ["DIPS_SERIES_WAVES_PER_SIMD"] = name[1:]
            op = ops[name]
            r = None if mode == Mode.PerFrame else ref
            op.run_device(frames, series[name], ref=r)  # warm
            torch.cuda.synchronize()
            op.kernel_time(reset=True)
            if smp:
                smp.sample()
            t0 = time.monotonic()
            for _ in range(steps):
                op.run_device(frames, series[name], ref=r)
            torch.cuda.synchronize()
            t1 = time.monotonic()
            if smp:
                smp.sample()
            kms = float(np.median(op.kernel_times()))
            rec = {"variant": name, "round": rnd, "steps": steps, "kernel_ms_median": round(kms, 4),
                   "frames_per_s": round(F / (kms / 1e3), 1),
                   "frac_of_8TBps": round(F * W * H * 3 / (kms / 1e3) / 8e12, 4),
                   "wall_frames_per_s": round(F * steps / (t1 - t0), 1)}
            if smp:
                g = smp.window(t0 - 0.5, t1 + 0.5)[0]
                if g and g.get("avg_power_W_energy"):
                    rec.update({"avg_W": g["avg_power_W_energy"], "ppt_frac": g.get("ppt_residency_frac"),
                                "mJ_per_frame": round(g["avg_power_W_energy"] / (F * steps / (t1 - t0)) * 1e3, 4),
                                "gfxclk_end_MHz": smp.rows[-1][4]})
            res.setdefault(name, []).append(rec)
            print(json.dumps(rec), flush=True)
    os.environ.pop("DIPS_SERIES_WAVES_PER_SIMD", None)
    same = all(bool(torch.equal(series[names[0]], series[k])) for k in names[1:])
    summ = {"summary": True, "size": f"{W}x{H}", "frames": F,
            "mode": "per-frame" if mode == Mode.PerFrame else "overall", "series_equal": same}
    for k, v in res.items():
        summ[k] = {"frac_median": float(np.median([r["frac_of_8TBps"] for r in v])),
                   "mJ_per_frame_median": float(np.median([r.get("mJ_per_frame", np.nan) for r in v])),
                   "wall_frames_per_s_median": float(np.median([r["wall_frames_per_s"] for r in v]))}
    print(json.dumps(summ), flush=True)
    for op in ops.values():
        op.close()


if __name__ == "__main__":
    main()
