#!/usr/bin/env python3
"""compat_variant_ab.py -- in-process A/B of the ComputeState table kernel's
(U, D) variants (DIPS_COMPAT_LUT_VARIANT, read per call): one frame batch,
variants alternated over rounds, kernel time by hipEvents, outputs compared
with the first variant's.  4K RGBA8, 1000 frames, colour + sigmoid.
Run on the GPU box: python tools/compat_variant_ab.py [rounds] [variants]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    variants = (sys.argv[2] if len(sys.argv) > 2 else "22,23,42,43").split(",")
    import torch
    from dips_amd import DiffSeriesOperator, PixelFormat
    from dips_amd.api import ChromaFilter, ComputeState, DiPsFilter
    W, H, n = 3840, 2160, 1000
    frames = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    syn = DiffSeriesOperator(PixelFormat.RGBA8)
    syn.synth_device(frames, W, H, 0xD1B5, 0)
    syn.close()
    out = torch.empty_like(frames)
    ref = None
    for r in range(rounds):
        for v in variants:
            os.environ["DIPS_COMPAT_LUT_VARIANT"] = v
            cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_, time_kernel=True)
            cs.frame_callback_batch_device(frames[:7], out[:7])
            cs.frame_callback_batch_device(frames, out)  # warm
            torch.cuda.synchronize()
            cs.kernel_time(reset=True)
            for _ in range(5):
                cs.frame_callback_batch_device(frames, out)
            torch.cuda.synchronize()
            ms, cnt = cs.kernel_time()
            ms /= max(cnt, 1)
            cs.close()
            h = out[::97].cpu().numpy()
            if ref is None:
                ref = h
            same = bool(np.array_equal(h, ref))
            gbs = 2 * n * W * H * 4 / (ms / 1e3) / 1e9
            print(json.dumps({"round": r, "variant": v, "kernel_ms": round(ms, 4), "GBps_read_write": round(gbs, 1),
                              "frac_of_8TBps": round(gbs / 8000, 4), "outputs_equal_first": same}), flush=True)


if __name__ == "__main__":
    main()
