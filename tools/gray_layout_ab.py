#!/usr/bin/env python3
"""gray_layout_ab.py -- the GRAY8 table kernel's layouts on several contents,
in one process over one resident batch per content (4K gray8, 3000 frames,
'per-frame', tau = 8/255): layout 2 (u16 table keyed by (a, b)), layout 3
(keyed by (a ^ b, a), band clamp, swizzled), layout 5 (the same unswizzled),
layout 4 (the default: 5 or 2 per workgroup from a sample of its own items),
as listed in LAYOUTS, alternated over ROUNDS rounds.
Contents: the bench's synthetic clip, i.i.d. uniform random frames, and the
smooth contents of tools/content_rate.py (flat, gradient, moving).  Kernel
time from the library's hipEvents (layout 4's in-kernel sample included); the
series of every layout must be equal.  One JSON line per (content, layout,
round).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

W, H = 3840, 2160


def main():
    import torch
    from content_rate import make
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    kinds = sys.argv[1].split(",") if len(sys.argv) > 1 else ["synthetic", "random", "flat", "gradient", "moving"]
    rounds = int(os.environ.get("ROUNDS", "3"))
    n = 3000
    op = DiffSeriesOperator(PixelFormat.Gray8, Mode.PerFrame, 8.0 / 255.0, time_kernel=True)
    try:
        for kind in kinds:
            if kind == "random":
                fr = torch.randint(0, 256, (n, H, W), dtype=torch.uint8, device="cuda")
            else:
                fr = make(torch, kind, n, 1, lambda d: op.synth_device(d, W, H, 0xD1B5, 0))
            ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            want = None
            for r in range(rounds):
                for lay in os.environ.get("LAYOUTS", "2,3,4").split(","):
                    os.environ["DIPS_GRAY_LUT"] = lay
                    op.run_device(fr, ser)  # warm (table build)
                    torch.cuda.synchronize()
                    op.kernel_time(reset=True)
                    for _ in range(3):
                        op.run_device(fr, ser)
                    torch.cuda.synchronize()
                    ms = float(np.median(op.kernel_times()))
                    got = ser.cpu().numpy()
                    if want is None:
                        want = got
                    gbs = n * W * H / (ms / 1e3) / 1e9
                    print(json.dumps({"content": kind, "layout": int(lay), "round": r, "frames": n,
                                      "kernel_ms": round(ms, 3), "GBps": round(gbs, 1),
                                      "frac_of_8TBps": round(gbs / 8000, 4),
                                      "series_equal": bool(np.array_equal(got, want))}), flush=True)
            os.environ.pop("DIPS_GRAY_LUT", None)
            del fr, ser
            torch.cuda.empty_cache()
    finally:
        op.close()


if __name__ == "__main__":
    main()
