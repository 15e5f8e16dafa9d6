#!/usr/bin/env python3
"""halo_overlap.py -- does RCCL's send / recv kernel find wave slots while the
persistent series kernel holds the GPU?  (The N > 1 'per-frame' step posts
the halo frame's send / recv, then launches frames 1..F-1; frame 0 waits for
the halo, dips_amd/shard.py per_frame_overlapped.)

World size 1 on cuda:0 (RCCL refuses two ranks on one GPU): a send / recv of
one 4K RGB8 frame to self, posted from a side stream right before the
4,999-frame series launch under DIPS_SERIES_WAVES_PER_SIMD=4 (as bench.py
sets it for N > 1).  hipEvents on the side stream (after the RCCL work) and
on the launch stream give when each finished, from a common start event;
the same transfer alone gives its own duration.  One JSON line per trial.

Run on the GPU box: RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \\
    python tools/r05/halo_overlap.py [--trials 3]
"""
import argparse
import json
import os
import sys
from datetime import timedelta

os.environ.setdefault("DIPS_SERIES_WAVES_PER_SIMD", "4")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

W, H, C, F = 3840, 2160, 3, 5000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=60))
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
    frames = torch.empty((F, H, W, C), dtype=torch.uint8, device=dev)
    op.synth_device(frames, W, H, 0xD1B5, 0)
    series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
    halo = torch.empty((H, W, C), dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()

    def post(dst):
        ops = [dist.P2POp(dist.isend, frames[-1], 0), dist.P2POp(dist.irecv, dst, 0)]
        return dist.batch_isend_irecv(ops)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    # warm: RCCL's first p2p sets up its connection
    for w in post(halo):
        w.wait()
    op.run_device(frames[1:], series[1:], ref=frames[0])
    torch.cuda.synchronize()
    for trial in range(args.trials):
        # the transfer alone
        e0, e1 = ev(), ev()
        with torch.cuda.stream(side):
            e0.record(side)
            for w in post(halo):
                w.wait()
            e1.record(side)
        torch.cuda.synchronize()
        alone = e0.elapsed_time(e1)
        # the transfer posted right before the series launch
        halo.zero_()
        torch.cuda.synchronize()
        s0, r1, k1 = ev(), ev(), ev()
        s0.record(main_s)
        side.wait_event(s0)
        with torch.cuda.stream(side):
            works = post(halo)
            for w in works:
                w.wait()
            r1.record(side)
        op.run_device(frames[1:], series[1:], ref=frames[0])
        k1.record(main_s)
        torch.cuda.synchronize()
        rec = {"trial": trial, "transfer_alone_ms": round(alone, 4),
               "transfer_done_ms": round(s0.elapsed_time(r1), 4),
               "series_done_ms": round(s0.elapsed_time(k1), 4),
               "halo_equal": bool(torch.equal(halo, frames[-1])),
               "waves_per_simd_cap": os.environ["DIPS_SERIES_WAVES_PER_SIMD"]}
        rec["overlapped"] = rec["transfer_done_ms"] < 0.5 * rec["series_done_ms"]
        print(json.dumps(rec), flush=True)
    dist.destroy_process_group()
    op.close()


if __name__ == "__main__":
    main()
