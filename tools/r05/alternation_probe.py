#!/usr/bin/env python3
"""alternation_probe.py -- consecutive processes that each allocate one
124 GB frame buffer alternate between a fast and a slow rate
(profiles/r05/ab_u5/).  Is the slow one the process that starts while the
previous process's memory is still being released?  Prints, at start, the
device's free memory (hipMemGetInfo) a few times over a second, then the
frame buffer's device address and the series kernel's rate.  Run several
times in a row: tools/r05/alternation.sh.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

W, H, C, F = 3840, 2160, 3, 5000


def main():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat

    wait = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
    dev = torch.device("cuda", 0)
    t0 = time.time()
    free = []
    for _ in range(5):
        f, total = torch.cuda.mem_get_info(dev)
        free.append(round(f / 2 ** 30, 1))
        time.sleep(0.2)
    if wait > 0:  # wait until (nearly) all of the device's memory is free, at most `wait` s
        while time.time() - t0 < wait:
            f, total = torch.cuda.mem_get_info(dev)
            if f > total - (4 << 30):
                break
            time.sleep(0.1)
    f_alloc, total = torch.cuda.mem_get_info(dev)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
    frames = torch.empty((F, H, W, C), dtype=torch.uint8, device=dev)
    op.synth_device(frames, W, H, 0xD1B5, 0)
    series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
    op.run_device(frames, series)
    torch.cuda.synchronize()
    op.kernel_time(reset=True)
    for _ in range(4):
        op.run_device(frames, series)
    torch.cuda.synchronize()
    ms, n = op.kernel_time()
    ms /= max(n, 1)
    print(json.dumps({"free_GiB_at_start": free, "free_GiB_at_alloc": round(f_alloc / 2 ** 30, 1),
                      "total_GiB": round(total / 2 ** 30, 1), "waited_s": round(time.time() - t0, 2),
                      "frames_address_GiB": round(frames.data_ptr() / 2 ** 30, 2), "series_ms": round(ms, 4),
                      "frac_of_8TBps": round(F * W * H * C / (ms / 1e3) / 8e12, 4)}), flush=True)
    op.close()


if __name__ == "__main__":
    main()
