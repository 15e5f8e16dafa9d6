#!/usr/bin/env python3
"""content_rate.py -- throughput of the table kernels on different image
content (4K, HBM-resident, per-frame, tau = 8/255).

The GRAY8 series kernel and the ComputeState batch kernel look up a 2-D
table in LDS per pixel; an LDS read's bank follows from the table address,
so the speed depends on how the 64 lanes' (frame, reference) byte pairs
spread over the banks.  The bench's synthetic frames have an independent
random base per pixel (spread by construction); natural video has smooth
regions with a few levels of sensor noise.  Contents:
  synthetic  -- the bench generator (random base + moving disc + noise)
  flat       -- 128 + uniform noise in [-3, 3], independent per frame
  gradient   -- horizontal ramp 0..255 + noise in [-2, 2] (static scene)
  moving     -- the ramp shifted 3 px per frame + noise in [-2, 2]
Prints one JSON line per (kernel, content).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H = 3840, 2160


def make(torch, kind, n, c, op_synth):
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    shape = (n, H, W) if c == 1 else (n, H, W, c)
    if kind == "synthetic":
        fr = torch.empty(shape, dtype=torch.uint8, device="cuda")
        op_synth(fr)
        return fr
    out = torch.empty(shape, dtype=torch.uint8, device="cuda")
    ramp = (torch.arange(W, device="cuda", dtype=torch.float32) * (255.0 / (W - 1)))
    for t in range(n):
        if kind == "flat":
            base = torch.full((H, W), 128.0, device="cuda")
            amp = 3
        elif kind == "gradient":
            base = ramp.expand(H, W)
            amp = 2
        else:  # moving
            base = torch.roll(ramp, shifts=3 * t).expand(H, W)
            amp = 2
        noise = torch.randint(-amp, amp + 1, (H, W) if c == 1 else (H, W, c), device="cuda", generator=g)
        v = (base if c == 1 else base.unsqueeze(-1)) + noise
        out[t] = v.clamp_(0, 255).to(torch.uint8)
    return out


def main():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from dips_amd.api import ComputeState, DiPsFilter, ChromaFilter
    kinds = sys.argv[1].split(",") if len(sys.argv) > 1 else ["synthetic", "flat", "gradient", "moving"]
    reps = 5
    kern = os.environ.get("CONTENT_KERNELS", "gray,compat,alt")
    # GRAY8 series (table kernel)
    n = 3000
    op = DiffSeriesOperator(PixelFormat.Gray8, Mode.PerFrame, 8.0 / 255.0, time_kernel=True)
    for kind in (kinds if "gray" in kern else []):
        fr = make(torch, kind, n, 1, lambda d: op.synth_device(d, W, H, 0xD1B5, 0))
        ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        op.run_device(fr, ser)
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        for _ in range(reps):
            op.run_device(fr, ser)
        torch.cuda.synchronize()
        ms = float(np.median(op.kernel_times()))
        gbs = n * W * H / (ms / 1e3) / 1e9
        print(json.dumps({"kernel": "series_gray_lut_kernel", "content": kind, "frames": n, "kernel_ms": round(ms, 3),
                          "GBps": round(gbs, 1), "frac_of_8TBps": round(gbs / 8000, 4),
                          "selected_frac": round(float(ser[1:, 2].sum()) / ((n - 1) * W * H), 4)}), flush=True)
        del fr, ser
        torch.cuda.empty_cache()
    op.close()
    if "alt" in kern:
        # dips_alt run loop (RGBA8, N = 2, default colour + sigmoid: the
        # two-level diff table)
        from dips_amd.alt import DiPsCompute
        n = 1000
        syn = DiffSeriesOperator(PixelFormat.RGBA8, Mode.PerFrame, 0.0)
        for kind in kinds:
            fr = make(torch, kind, n, 4, lambda d: syn.synth_device(d, W, H, 0xD1B5, 0))
            if kind != "synthetic":
                fr[..., 3] = 255
            out = torch.empty_like(fr)
            flags = [t == 2 for t in range(n)]
            c = DiPsCompute(2, H, W, time_kernel=True)
            c.send_frames_device(fr, out, flags)
            torch.cuda.synchronize()
            c.kernel_time(reset=True)
            for _ in range(reps):
                c.send_frames_device(fr, out, flags)
            torch.cuda.synchronize()
            ms, cnt = c.kernel_time()
            ms /= max(cnt, 1)
            gbs = 2 * n * W * H * 4 / (ms / 1e3) / 1e9
            print(json.dumps({"kernel": "alt_batch_kernel LUT (colour + sigmoid)", "content": kind, "frames": n,
                              "kernel_ms": round(ms, 3), "launches": cnt, "GBps_read_write": round(gbs, 1),
                              "frac_of_8TBps": round(gbs / 8000, 4)}), flush=True)
            c.close()
            del fr, out
            torch.cuda.empty_cache()
        syn.close()
    if "compat" not in kern:
        return
    # ComputeState batch (RGBA8, colour + sigmoid: the (S, m) table kernel)
    n = 1000
    syn = DiffSeriesOperator(PixelFormat.RGBA8, Mode.PerFrame, 0.0)
    for kind in kinds:
        fr = make(torch, kind, n, 4, lambda d: syn.synth_device(d, W, H, 0xD1B5, 0))
        if kind != "synthetic":
            fr[..., 3] = 255
        cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_, time_kernel=True)
        out = torch.empty_like(fr)
        cs.frame_callback_batch_device(fr[:7], out[:7])  # the stream's first frames
        cs.frame_callback_batch_device(fr, out)          # warm
        torch.cuda.synchronize()
        cs.kernel_time(reset=True)
        for _ in range(reps):
            cs.frame_callback_batch_device(fr, out)
        torch.cuda.synchronize()
        ms, cnt = cs.kernel_time()
        ms /= max(cnt, 1)
        gbs = 2 * n * W * H * 4 / (ms / 1e3) / 1e9
        print(json.dumps({"kernel": "compat_batch_lut_kernel (colour + sigmoid)", "content": kind, "frames": n,
                          "kernel_ms": round(ms, 3), "launches": cnt, "GBps_read_write": round(gbs, 1),
                          "frac_of_8TBps": round(gbs / 8000, 4)}), flush=True)
        cs.close()
        del fr, out
        torch.cuda.empty_cache()
    syn.close()


if __name__ == "__main__":
    main()
