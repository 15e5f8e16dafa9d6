"""Placement-aware allocation of a resident frame batch.

Where the driver places a 124 GB frame buffer moves the series kernel by 2-3
points of 8 TB/s: the kernel is bound by the package power limit, and one of
the two placements a process can get costs more energy per byte (more
address-translation misses for the same HBM requests; DESIGN.md "Open items
after round 5", profiles/r05/placement/).  Which placement an allocation gets
alternates between consecutive processes (profiles/r05/placement/alternation/)
and is not controlled by the allocation API, the alignment or the schedule.

`resident_frames` therefore allocates two candidate buffers when the device
has room for both, fills each with the same frames, times a few launches of
the caller's series operator on each and keeps the faster one; the other is
released before the function returns.  The choice and both candidates'
timings are returned so that callers (bench.py) report them.  With
probe=False, or without room for two buffers, it is one plain allocation.
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple


def resident_frames(op, shape: Tuple[int, ...], device, fill: Callable, probe: bool = True,
                    launches: int = 2, ref_of: Callable = None, margin_bytes: int = 8 << 30):
    """Allocate a uint8 tensor of `shape` on `device`, filled by fill(tensor).

    op: a DiffSeriesOperator (its run_device is the probe; its kernel timer
    is reset afterwards).  ref_of(tensor) gives the probe launch's reference
    frame ('overall' operators), or None.  Returns (tensor, report)."""
    import torch

    nbytes = 1
    for s in shape:
        nbytes *= int(s)
    free, _ = torch.cuda.mem_get_info(device)
    report: Dict = {"probe": False}
    if not probe or 2 * nbytes + margin_bytes > free or shape[0] == 0:
        t = torch.empty(shape, dtype=torch.uint8, device=device)
        fill(t)
        report["reason"] = "disabled" if not probe else ("empty batch" if shape[0] == 0 else
                                                          "no room for two candidates")
        return t, report
    cands = [torch.empty(shape, dtype=torch.uint8, device=device)]
    try:
        cands.append(torch.empty(shape, dtype=torch.uint8, device=device))
    except torch.cuda.OutOfMemoryError:  # reported free, not allocatable: one plain buffer
        torch.cuda.empty_cache()
        fill(cands[0])
        report["reason"] = "second candidate not allocatable"
        return cands[0], report
    series = torch.empty((shape[0], 4), dtype=torch.int64, device=device)
    ms = []
    for c in cands:
        fill(c)
        ref = ref_of(c) if ref_of else None
        op.run_device(c, series, ref=ref)  # warm
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        for _ in range(launches):
            op.run_device(c, series, ref=ref)
        torch.cuda.synchronize()
        k, n = op.kernel_time(reset=True)
        ms.append(k / max(n, 1))
    keep = 0 if ms[0] <= ms[1] else 1
    t = cands[keep]
    del cands, series
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # the other candidate back to the driver
    report.update({"probe": True, "candidate_kernel_ms": [round(x, 4) for x in ms], "kept": keep,
                   "launches_each": launches})
    return t, report
