"""Does the halo exchange of the sharded 'per-frame' call hide behind the
series launch?  At world size 1 on one GPU: an RCCL self send/recv of one 4K
RGB8 frame (ncclSend + ncclRecv to rank 0 in one group -- the same p2p
kernel a rank-to-rank halo launches) on a side stream, concurrently with the
series launch over F resident frames on the main stream, with the series
grid at its full occupancy (4 waves per SIMD) and at one slot per SIMD left
free (DIPS_SERIES_WAVES_PER_SIMD=3, what shard_abi.hip's reserve gives).
Prints one JSON line per variant (median of `reps` repetitions, ms)."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dips_amd import DiffSeriesOperator, Mode, PixelFormat  # noqa: E402

W, H = 3840, 2160
F = int(os.environ.get("F", "2000"))
REPS = int(os.environ.get("REPS", "7"))
torch.cuda.init()
rccl = ctypes.CDLL("librccl.so.1")


class UID(ctypes.Structure):
    _fields_ = [("b", ctypes.c_char * 128)]


uid = UID()
assert rccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
comm = ctypes.c_void_p()
assert rccl.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0

op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
frames = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
op.synth_device(frames, W, H, 0xD1B5, 0)
series = torch.zeros((F, 4), dtype=torch.int64, device="cuda")
halo = torch.empty_like(frames[0])
nbytes = frames[0].numel()
side = torch.cuda.Stream()
main = torch.cuda.current_stream()


def exchange():
    s = ctypes.c_void_p(side.cuda_stream)
    assert rccl.ncclGroupStart() == 0
    assert rccl.ncclSend(ctypes.c_void_p(frames[-1].data_ptr()), ctypes.c_size_t(nbytes), 1, 0, comm, s) == 0
    assert rccl.ncclRecv(ctypes.c_void_p(halo.data_ptr()), ctypes.c_size_t(nbytes), 1, 0, comm, s) == 0
    assert rccl.ncclGroupEnd() == 0


def timed(fn):
    out = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t) * 1e3)
    return float(np.median(out))


def series_only():
    op.run_device(frames, series)


def both(order):
    def fn():
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        if order == "exchange_first":
            exchange()
            op.run_device(frames, series)
        else:
            op.run_device(frames, series)
            exchange()
    return fn


series_only()
exchange()
torch.cuda.synchronize()
rows = []
for cap in (None, "3"):
    if cap:
        os.environ["DIPS_SERIES_WAVES_PER_SIMD"] = cap
    else:
        os.environ.pop("DIPS_SERIES_WAVES_PER_SIMD", None)
    waves = op.geometry(W, H, F)[0]
    r = {"cap": cap or "none", "waves": waves, "frames": F,
         "series_ms": timed(series_only), "exchange_ms": timed(exchange),
         "both_exchange_first_ms": timed(both("exchange_first")),
         "both_series_first_ms": timed(both("series_first"))}
    r["hidden_exchange_first"] = round(r["series_ms"] + r["exchange_ms"] - r["both_exchange_first_ms"], 4)
    rows.append(r)
    print(json.dumps(r), flush=True)
rccl.ncclCommDestroy(comm)
op.close()
