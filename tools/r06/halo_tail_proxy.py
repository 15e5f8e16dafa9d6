"""What the halo's RCCL kernel costs the series launch at N > 1, by proxy on
one GPU.  Over xGMI the halo (one 4K RGB8 frame, 24.9 MB) takes ~0.3 ms, and
the RCCL p2p kernel holds its wave slots that long; the series launch is a
persistent grid with a fixed share per wave, so a displaced wave should
start -- and finish -- that much later.  The proxy: `blocks` one-wave spin
kernels (torch.cuda._sleep, no memory traffic) posted on side streams for
`us` microseconds before the series launch over F resident frames; the
launch's hipEvent time against the launch alone.  One JSON line per variant
(median of `reps`), the expectation being +us per launch, independent of the
number of displaced waves."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dips_amd import DiffSeriesOperator, Mode, PixelFormat  # noqa: E402

W, H = 3840, 2160
F = int(os.environ.get("F", "2000"))
REPS = int(os.environ.get("REPS", "7"))
torch.cuda.init()

op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
frames = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
op.synth_device(frames, W, H, 0xD1B5, 0)
series = torch.zeros((F, 4), dtype=torch.int64, device="cuda")
main = torch.cuda.current_stream()
sides = [torch.cuda.Stream() for _ in range(8)]


def sleep_cycles_per_us():
    """torch.cuda._sleep's clock, calibrated with events."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cyc = 20_000_000
    torch.cuda._sleep(cyc // 10)  # warm
    torch.cuda.synchronize()
    e0.record()
    torch.cuda._sleep(cyc)
    e1.record()
    torch.cuda.synchronize()
    return cyc / (e0.elapsed_time(e1) * 1e3)


def launch_ms(us, blocks, cpu):
    """Median hipEvent time of the series launch with `blocks` spin kernels
    of `us` microseconds posted first."""
    out = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        for b in range(blocks):
            with torch.cuda.stream(sides[b]):
                torch.cuda._sleep(int(us * cpu))
        op.run_device(frames, series)
        torch.cuda.synchronize()
        out.append(op.kernel_times()[-1])
    return float(np.median(out))


cpu = sleep_cycles_per_us()
op.run_device(frames, series)  # warm
torch.cuda.synchronize()
base = launch_ms(0, 0, cpu)
print(json.dumps({"variant": "series alone", "frames": F, "launch_ms": round(base, 4), "sleep_cycles_per_us": cpu}),
      flush=True)
for us in (100, 330, 1000):
    for blocks in (1, 8):
        ms = launch_ms(us, blocks, cpu)
        print(json.dumps({"variant": f"{blocks} spin kernel(s) of {us} us posted first", "frames": F,
                          "launch_ms": round(ms, 4), "extra_ms": round(ms - base, 4),
                          "extra_over_spin": round((ms - base) / (us / 1e3), 3)}), flush=True)
