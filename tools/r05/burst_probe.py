#!/usr/bin/env python3
"""burst_probe.py -- the series kernel in short bursts after the GPU idled,
against the same launches back to back: if the package power limit (not
the kernel) sets the sustained rate, a launch short enough to finish before
the limiter acts runs near the compute-free read rate.

The 4K RGB8 per-frame batch resident (placement-aware), then for N in
(100, 200, 400, 1000, 5000) frames: one launch over frames[:N] after 1.5 s
of idle (three times, the median) and five back-to-back launches (the
median of the last three); the compute-free read of the same bytes the
same two ways.  One JSON line per N.

Run on the GPU box: python tools/r05/burst_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

W, H, C, F = 3840, 2160, 3, 5000


def main():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from dips_amd.placement import resident_frames

    dev = torch.device("cuda", 0)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
    frames, placement = resident_frames(op, (F, H, W, C), dev, lambda t: op.synth_device(t, W, H, 0xD1B5, 0))
    series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
    fb = W * H * C

    def one(n):
        op.kernel_time(reset=True)
        op.run_device(frames[:n], series[:n])
        torch.cuda.synchronize()
        ms, k = op.kernel_time(reset=True)
        return ms / max(k, 1)

    print(json.dumps({"placement": placement}), flush=True)
    for n in (100, 200, 400, 1000, 5000):
        burst, burst_read = [], []
        for _ in range(3):
            time.sleep(1.5)
            burst.append(one(n))
            time.sleep(1.5)
            burst_read.append(op.read_ceiling_ms(frames[:n]))
        back = [one(n) for _ in range(5)][2:]
        back_read = [op.read_ceiling_ms(frames[:n]) for _ in range(5)][2:]
        rate = lambda ms: round(n * fb / (float(np.median(ms)) / 1e3) / 8e12, 4)  # noqa: E731
        print(json.dumps({"frames": n, "GB": round(n * fb / 1e9, 2),
                          "burst_ms": round(float(np.median(burst)), 4), "burst_frac": rate(burst),
                          "sustained_ms": round(float(np.median(back)), 4), "sustained_frac": rate(back),
                          "read_burst_frac": rate(burst_read), "read_sustained_frac": rate(back_read)}), flush=True)
    op.close()


if __name__ == "__main__":
    main()
