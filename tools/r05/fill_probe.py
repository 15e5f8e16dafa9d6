#!/usr/bin/env python3
"""fill_probe.py -- does the series kernel's rate follow the buffer (where it
was placed) or how its bytes were last written?  Two 124 GB buffers of one
process (A allocated first): A filled by the synthesis kernel and B by a
device-to-device copy of A, both measured; then the roles swap (B
synthesised, A copied from B) and both are measured again; then once more.
Same bytes in every buffer and pass (the series of every run is compared).
One JSON line per measurement.

Run on the GPU box: python tools/r05/fill_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

W, H, C, F = 3840, 2160, 3, 5000
SEED = 0xD1B5


def main():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat

    dev = torch.device("cuda", 0)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
    fb = W * H * C
    bufs = {"A": torch.empty(F * fb, dtype=torch.uint8, device=dev),
            "B": torch.empty(F * fb, dtype=torch.uint8, device=dev)}
    series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
    ref = None

    def measure(name, how, rnd):
        nonlocal ref
        frames = bufs[name].view(F, H, W, C)
        op.run_device(frames, series)
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        for _ in range(4):
            op.run_device(frames, series)
        torch.cuda.synchronize()
        ms, n = op.kernel_time()
        ms /= max(n, 1)
        got = series.cpu()
        if ref is None:
            ref = got
        print(json.dumps({"round": rnd, "buffer": name, "allocated": "first" if name == "A" else "second",
                          "filled_by": how, "series_ms": round(ms, 4),
                          "frac_of_8TBps": round(F * fb / (ms / 1e3) / 8e12, 4),
                          "series_equal": bool(torch.equal(got, ref))}), flush=True)

    for rnd, (syn, cop) in enumerate((("A", "B"), ("B", "A"), ("A", "B"))):
        op.synth_device(bufs[syn].view(F, H, W, C), W, H, SEED, 0)
        bufs[cop].copy_(bufs[syn])
        torch.cuda.synchronize()
        measure(syn, "synthesis kernel", rnd)
        measure(cop, "device copy", rnd)
    op.close()


if __name__ == "__main__":
    main()
