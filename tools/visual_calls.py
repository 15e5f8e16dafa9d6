#!/usr/bin/env python3
"""visual_calls.py -- a few back-to-back batch calls of the two visual
operators (4K RGBA8, 1000 HBM-resident frames) for a rocprofv3 kernel /
copy trace: where the wall time of a call goes beyond its main kernel."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from dips_amd import DiffSeriesOperator, PixelFormat
    from dips_amd.api import ChromaFilter, ComputeState, DiPsFilter
    from dips_amd.alt import DiPsCompute
    W, H, n = 3840, 2160, 1000
    frames = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    syn = DiffSeriesOperator(PixelFormat.RGBA8)
    syn.synth_device(frames, W, H, 0xD1B5, 0)
    syn.close()
    out = torch.empty_like(frames)
    cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    cs.frame_callback_batch_device(frames[:7], out[:7])
    cs.frame_callback_batch_device(frames, out)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        cs.frame_callback_batch_device(frames, out)
    torch.cuda.synchronize()
    print("compat wall ms/call", (time.perf_counter() - t) / 5 * 1e3, flush=True)
    cs.close()
    flags = [k == 2 for k in range(n)]
    c = DiPsCompute(2, H, W)
    c.send_frames_device(frames, out, flags)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        c.send_frames_device(frames, out, flags)
    torch.cuda.synchronize()
    print("alt wall ms/call", (time.perf_counter() - t) / 5 * 1e3, flush=True)
    c.close()


if __name__ == "__main__":
    main()
