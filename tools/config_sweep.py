#!/usr/bin/env python3
"""config_sweep.py -- every BASELINE.json config on one MI355X (the per-GPU
slice of the multi-GPU ones), HBM-resident synthetic frames, timed with the
library's hipEvents around the series kernel.  One JSON line per config plus
a parity spot check of the first frames against the oracle.

Run on the GPU box: python tools/config_sweep.py [--steps 5]
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

# (name, width, height, channels, frames per GPU, mode, tau)
CONFIGS = [
    ("configs[0] 640x480 gray8, 300 frames, overall", 640, 480, 1, 300, 0, 0.0),
    ("configs[1] 1920x1080 RGB8, 1000 frames, overall", 1920, 1080, 3, 1000, 0, 8 / 255),
    ("configs[2] 3840x2160 RGB8, 5000 frames, per-frame", 3840, 2160, 3, 5000, 1, 8 / 255),
    ("configs[3] 3840x2160 RGB8, 40000/8 frames per GPU, overall", 3840, 2160, 3, 5000, 0, 8 / 255),
    ("configs[4] 7680x4320 RGB8, 10000/8 frames per GPU, f32 threshold", 7680, 4320, 3, 1250, 0, 8 / 255),
    ("extra: 3840x2160 RGBA8, 3750 frames, per-frame", 3840, 2160, 4, 3750, 1, 8 / 255),
    ("extra: 3840x2160 gray8, 15000 frames, per-frame", 3840, 2160, 1, 15000, 1, 8 / 255),
]

# GRAY8 kernel forms: the table kernel with its per-workgroup layout choice
# (the default), either table pinned (DIPS_FLAG_GRAY_*_TABLE), or the f32
# series_fast_kernel (DIPS_FLAG_CROSSCHECK)
_GRAY_FORMS = {"auto": {}, "band": {"gray_table": "band"}, "pair": {"gray_table": "pair"}, "f32": {"crosscheck": True}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--only", default="", help="run the configs whose name contains this string")
    ap.add_argument("--gray-kernel", choices=sorted(_GRAY_FORMS), default="auto",
                    help="GRAY8: the table kernel with its per-workgroup layout choice (auto, the library "
                         "default), the band-keyed or the pair-keyed table pinned, or the f32 kernel")
    ap.add_argument("--no-placement-probe", action="store_true",
                    help="one plain allocation per config (tools/placement.py resident_frames probe=False)")
    args = ap.parse_args()
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from tools.placement import resident_frames
    from oracle import oracle

    import bench  # the power legs: energy counter / PPT residency / gfx clock around a leg
    smp = bench._power_sampler(torch, 0)
    dev = torch.device("cuda", 0)
    for name, W, H, C, F, mode, tau in CONFIGS:
        if args.only and args.only not in name:
            continue
        shape = (F, H, W) if C == 1 else (F, H, W, C)
        op = DiffSeriesOperator(PixelFormat(C), Mode(mode), tau, time_kernel=True,
                                **(_GRAY_FORMS[args.gray_kernel] if C == 1 else {}))
        # the batch in the faster of two candidate placements, as bench.py
        frames, placement = resident_frames(op, shape, dev, lambda t: op.synth_device(t, W, H, 0xD1B5, 0),
                                            probe=not args.no_placement_probe)
        series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
        op.run_device(frames, series)
        torch.cuda.synchronize()
        op.kernel_time(reset=True)

        def timed():
            t = time.perf_counter()
            for _ in range(args.steps):
                op.run_device(frames, series)
            torch.cuda.synchronize()
            return (time.perf_counter() - t) / args.steps

        wall, power = bench._power_leg(smp, timed, F * args.steps, f"{args.steps} series launches")
        kms, n = op.kernel_time()
        kms /= max(n, 1)
        # the compute-free read of the same bytes, its own power reading
        reads, read_power = bench._power_leg(smp, lambda: [op.read_ceiling_ms(frames) for _ in range(args.steps)],
                                             F * args.steps, f"{args.steps} read_ceiling_kernel launches")
        read_ms = float(np.median(reads))
        host = frames[:3].cpu().numpy()
        want, _, _ = oracle.series(host, mode=mode, tau=tau, nthreads=8)
        ok = bool(np.array_equal(series[:3].cpu().numpy().view(np.uint64), want))
        fb = W * H * C
        print(json.dumps({"config": name, "steps": args.steps, "wall_ms": round(wall * 1e3, 4), **({"gray_kernel": args.gray_kernel} if C == 1 else {}),
                          "frames_per_s": round(F / wall, 1),
                          "kernel_ms": round(kms, 4), "kernel_GBps": round(F * fb / (kms / 1e3) / 1e9, 1),
                          "frac_of_8TBps": round(F * fb / (kms / 1e3) / 8e12, 4),
                          "power": power,
                          "read_ceiling": {"ms": round(read_ms, 4),
                                           "frac_of_8TBps": round(F * fb / (read_ms / 1e3) / 8e12, 4),
                                           "power": read_power},
                          "placement": placement,
                          "first_frames_match_oracle": ok}), flush=True)
        op.close()
        del frames, series
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
