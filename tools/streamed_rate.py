#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-frame path (dips_diff_series_streamed):
frames start in pageable host memory, are staged through pinned buffers and
DMA'd on a side stream while the series kernel runs on the previous chunk.
Prints one JSON line; DESIGN.md quotes it next to the HBM-resident bench."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.init()
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from oracle import oracle  # test infra: parity of the streamed result only
    W, H, C = 3840, 2160, 3
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 240
    frames = oracle.synth(C, W, H, 0xD1B5, 0, 8)
    frames = np.concatenate([frames] * (n // 8))  # host batch (pageable)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8.0 / 255.0)
    res = {}
    for chunk in (8, 16, 32):
        op.streamed(frames[:2 * chunk], chunk_frames=chunk)  # warm (allocations)
        t = time.perf_counter()
        s = op.streamed(frames, chunk_frames=chunk)
        dt = time.perf_counter() - t
        res[chunk] = {"frames_per_s": round(n / dt, 1), "host_GB_per_s": round(frames.nbytes / dt / 1e9, 2)}
    ref = op(frames[:16])[0].as_array()
    ok = bool(np.array_equal(s.as_array()[:16], ref))
    print(json.dumps({"metric": "PCIe-inclusive series rate (host frames)", "frames": n,
                      "frame_bytes": W * H * C, "by_chunk_frames": res, "matches_device_path": ok}))


if __name__ == "__main__":
    main()
