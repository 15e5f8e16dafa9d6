#!/usr/bin/env python3
"""window_rate.py -- the spatial median (W in 1..11)
over HBM-resident 4K RGBA8 frames, frames/s by wall clock after a warm-up.
One JSON line per window size.

  python tools/window_rate.py [N]        dips ComputeState
      (frame_callback_batch_device; W > 1 through compat_filter_frames + the
      batch kernel)
  python tools/window_rate.py [N] alt    dips_alt DiPsCompute, N = 2
      (send_frames_device; W > 1 through alt_filter_frames + the batch
      kernel on f32 intensities; --generic: the per-frame kernel)"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    W, H = 3840, 2160
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 24
    alt = len(args) > 1 and args[1] == "alt"
    generic = "--generic" in sys.argv
    dev = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    out = torch.empty_like(dev)
    for win in range(1, 12):
        if alt:
            from dips_amd.alt import DiPsCompute, DiPsProperties
            cs = DiPsCompute(2, H, W, DiPsProperties(window_size=win), force_generic=generic)
            flags = [t == 2 for t in range(n)]
            cs.send_frames_device(dev[:8], out[:8], flags[:8])
            torch.cuda.synchronize()
            t = time.perf_counter()
            cs.send_frames_device(dev[8:], out[8:], flags[8:])
        else:
            cs = ComputeState(False, win, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
            cs.frame_callback_batch_device(dev[:8], out[:8])  # warm-up + start texture
            torch.cuda.synchronize()
            t = time.perf_counter()
            cs.frame_callback_batch_device(dev[8:], out[8:])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        cs.close()
        m = n - 8
        print(json.dumps({"operator": "dips_alt" + (" generic" if generic else "") if alt else "dips",
                          "window": win, "frames": m, "frames_per_s": round(m / dt, 1),
                          "ms_per_frame": round(dt / m * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
