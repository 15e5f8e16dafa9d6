#!/usr/bin/env python3
"""fallback_rate.py -- throughput of the series path on shapes / pointers the
vectorised kernels do not take (VERDICT r1 "What's weak" #10): an odd pixel
count (1917x1079 RGB8), a frame batch that starts 1 byte past an aligned
address, and the same shapes forced onto the generic kernel, next to the
aligned fast path.  HBM-resident synthetic frames, kernel time from the
library's hipEvents, first frames checked against the oracle.  One JSON line
per case.

Run on the GPU box: python tools/fallback_rate.py [--frames 1000 --steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, width, height, channels, byte offset of the batch, force_generic)
CASES = [
    ("1920x1080 RGB8 aligned (fast kernel)", 1920, 1080, 3, 0, False),
    ("1917x1080 RGB8 aligned (W*H % 4 == 0: fast kernel)", 1917, 1080, 3, 0, False),
    ("1917x1079 RGB8 (odd pixel count)", 1917, 1079, 3, 0, False),
    ("1920x1080 RGB8 batch at +1 byte (unaligned frames)", 1920, 1080, 3, 1, False),
    ("1920x1080 RGB8 forced generic kernel", 1920, 1080, 3, 0, True),
    ("1920x1080 RGBA8 batch at +2 bytes", 1920, 1080, 4, 2, False),
    ("641x479 gray8 (odd pixel count)", 641, 479, 1, 0, False),
    ("640x480 gray8 aligned", 640, 480, 1, 0, False),
    ("1920x1080 RGBA8 aligned", 1920, 1080, 4, 0, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--mode", type=int, default=1)
    args = ap.parse_args()
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from oracle import oracle

    cases = []
    for name, W, H, C, off, generic in CASES:
        cases.append((name, W, H, C, off, generic, None))
        if C in (3, 4) and not generic and ((W * H * C) % 4 or off % 4):
            # the same unaligned batch with the byte-unaligned 12-/16-B loads (A/B)
            cases.append((name + " [DIPS_SERIES_ALIGN=0]", W, H, C, off, generic, "0"))
    for name, W, H, C, off, generic, align_env in cases:
        if align_env is None:
            os.environ.pop("DIPS_SERIES_ALIGN", None)
        else:
            os.environ["DIPS_SERIES_ALIGN"] = align_env
        F = args.frames if C != 1 else args.frames * 4
        fb = W * H * C
        flat = torch.empty(F * fb + 64, dtype=torch.uint8, device="cuda")
        shape = (F, H, W) if C == 1 else (F, H, W, C)
        frames = flat[off:off + F * fb].view(shape)
        op = DiffSeriesOperator(PixelFormat(C), Mode(args.mode), 8 / 255, time_kernel=True,
                                force_generic=generic)
        try:
            op.synth_device(frames, W, H, 0xD1B5, 0)
            series = torch.zeros((F, 4), dtype=torch.int64, device="cuda")
            op.run_device(frames, series)
            torch.cuda.synchronize()
            op.kernel_time(reset=True)
            t = time.perf_counter()
            for _ in range(args.steps):
                op.run_device(frames, series)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t) / args.steps
            kms, n = op.kernel_time()
            kms /= max(n, 1)
            try:
                waves, _, _ = op.geometry(W, H, F)
            except Exception:
                waves = 0
            host = frames[:3].cpu().numpy()
            want, _, _ = oracle.series(host, mode=args.mode, tau=8 / 255, nthreads=8)
            ok = bool(np.array_equal(series[:3].cpu().numpy().view(np.uint64), want))
        finally:
            op.close()
        ppv = 16 if C == 1 else 4
        kernel = "generic" if generic or not waves else (
            "vectorised + generic tail" if (W * H) % ppv else "vectorised")
        print(json.dumps({"case": name, "frames": F, "mode": args.mode,
                          "byte_offset": off, "frame_bytes_mod4": fb % 4, "kernel": kernel,
                          "frames_per_s": round(F / wall, 1), "kernel_ms": round(kms, 4),
                          "kernel_GBps": round(F * fb / (kms / 1e3) / 1e9, 1),
                          "frac_of_8TBps": round(F * fb / (kms / 1e3) / 8e12, 4),
                          "first_frames_match_oracle": ok}), flush=True)
        del flat, frames, series
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
