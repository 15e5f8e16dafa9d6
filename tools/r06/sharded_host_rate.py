"""Host-pointer calls of the series at one rank: the sharded call over an
RCCL communicator (world size 1) against the streamed feed and the plain
staged call, on the same 96 4K RGB8 frames in pageable host memory; frames/s
and host->device GB/s of each, series equal.  One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dips_amd import DiffSeriesOperator, Mode, PixelFormat  # noqa: E402
from dips_amd.comm import Comm  # noqa: E402

W, H, N, REPS = 3840, 2160, 96, 3
op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255)
comm = Comm.rccl(Comm.unique_id(), 1, 0, 0)
try:
    dev = torch.empty((N, H, W, 3), dtype=torch.uint8, device="cuda")
    op.synth_device(dev, W, H, 0xD1B5, 0)
    torch.cuda.synchronize()
    host = dev.cpu().numpy()
    del dev

    def timed(fn):
        fn()  # warm (pinned / ring allocations)
        out, ts = None, []
        for _ in range(REPS):
            t = time.perf_counter()
            out = fn()
            ts.append(time.perf_counter() - t)
        return out, float(np.median(ts))

    s_sh, t_sh = timed(lambda: op.sharded(comm, host, N)[1].as_array())
    s_st, t_st = timed(lambda: op.streamed(host).as_array())
    s_pl, t_pl = timed(lambda: op(host)[0].as_array())
    fb = W * H * 3
    rec = {"frames": N, "sharded_world1": {"frames_per_s": round(N / t_sh, 1), "GBps": round(N * fb / t_sh / 1e9, 2)},
           "streamed": {"frames_per_s": round(N / t_st, 1), "GBps": round(N * fb / t_st / 1e9, 2)},
           "staged": {"frames_per_s": round(N / t_pl, 1), "GBps": round(N * fb / t_pl / 1e9, 2)},
           "series_equal": bool(np.array_equal(s_sh, s_st) and np.array_equal(s_st, s_pl))}
    print(json.dumps(rec), flush=True)
finally:
    op.close()
    comm.close()
