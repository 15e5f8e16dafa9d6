#!/usr/bin/env python3
"""pfc_threads_ab.py -- the per_frame_call leg (4K RGBA8 dips_frame_callback
from pageable host memory, DiPsProperties defaults) under copy-pool variants:
the pool's thread count (DIPS_COPY_THREADS, read once per process) and its
NUMA pinning (DIPS_COPY_AFFINITY=1: workers on the GPU's node).  Each variant
runs in its own process, the variants alternated over --rounds rounds; every
run prints one JSON line with frames/s and the per-phase medians of
dips_callback_phases.  Outputs are checked against the device batch path.

  python tools/pfc_threads_ab.py [--rounds 2] [--calls 200] [--variants 8:0,16:0,8:1,16:1]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bind_node(node: str) -> None:
    """PFC_BIND_NODE=n: run this process (every thread it starts, and so the
    first touch of its buffers) on NUMA node n's CPUs."""
    cpus = set()
    try:
        with open(f"/sys/devices/system/node/node{int(node)}/cpulist") as f:
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
    except (OSError, ValueError):
        return
    cpus &= os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)


def worker(calls: int, warm: int = 8):
    if os.environ.get("PFC_BIND_NODE"):
        _bind_node(os.environ["PFC_BIND_NODE"])
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    W, H = 3840, 2160
    n = warm + calls
    gen = DiffSeriesOperator(PixelFormat.RGBA8)
    dev = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    gen.synth_device(dev, W, H, 0xD1B5 ^ 0x4A, 0)
    gen.close()
    host = dev.cpu().numpy()
    b = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    od = torch.empty_like(dev)
    b.frame_callback_batch_device(dev, od)
    torch.cuda.synchronize()
    want = od.cpu().numpy()
    b.close()
    del dev, od
    torch.cuda.empty_cache()
    outs = np.empty_like(host)
    outs.fill(0)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    times, ph = [], []

    def cpu_stat():
        try:
            with open("/sys/fs/cgroup/cpu.stat") as f:
                return {k: int(v) for k, v in (l.split() for l in f if len(l.split()) == 2)}
        except (OSError, ValueError):
            return {}
    c0 = t00 = None
    for t in range(n):
        if t == warm:
            c0, t00 = cpu_stat(), time.perf_counter()
        t0 = time.perf_counter()
        hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                         outs[t].ctypes.data, outs[t].nbytes))
        dt = time.perf_counter() - t0
        if t >= warm:
            times.append(dt)
            ph.append(cs.callback_phases())
    c1, t11 = cpu_stat(), time.perf_counter()
    cs.close()
    cg = ({"cpus_busy_avg": round((c1["usage_usec"] - c0["usage_usec"]) / 1e6 / (t11 - t00), 2),
           "throttled_ms": round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 2)}
          if c0 and c1 and "usage_usec" in c0 else None)
    med = {k: round(float(np.median([p[k] for p in ph])) / 1e3, 4) for k in ph[0]
           if k not in ("threads", "stripes")}
    return {"frames_per_s": round(calls / sum(times), 1), "median_ms": round(float(np.median(times)) * 1e3, 4),
            "p90_ms": round(float(np.percentile(times, 90)) * 1e3, 4), "phases_ms_median": med,
            "threads": int(ph[0]["threads"]), "stripes": int(ph[0]["stripes"]),
            "equal": bool(np.array_equal(outs, want)), "cgroup_cpu": cg}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="8:0:1,12:0:1,16:0:1,8:1:1,16:1:1",
                    help="comma list of threads:affinity[:DIPS_CALLBACK_DIRECT[:DIPS_CB_BLOCKING[:PFC_BIND_NODE]]]")
    ap.add_argument("--env-variants", default=None,
                    help="instead of --variants: '|'-separated variants of 'KEY=VAL,KEY=VAL' environment settings")
    args = ap.parse_args()
    if args.worker:
        print(json.dumps(worker(args.calls)), flush=True)
        return
    if args.env_variants is not None:
        for r in range(args.rounds):
            for v in args.env_variants.split("|"):
                kv = dict(x.split("=", 1) for x in v.split(",") if x)
                p = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", "--calls", str(args.calls)],
                                   env=dict(os.environ, **kv), capture_output=True, text=True, timeout=300)
                line = [l for l in p.stdout.splitlines() if l.startswith("{")]
                rec = json.loads(line[-1]) if line else {"failed": p.stderr[-800:]}
                rec.update({"round": r, "env": kv})
                print(json.dumps(rec), flush=True)
        return
    for r in range(args.rounds):
        for v in args.variants.split(","):
            th, aff, *rest = v.split(":")
            direct = rest[0] if rest else "1"
            blocking = rest[1] if len(rest) > 1 else "0"
            node = rest[2] if len(rest) > 2 else ""
            env = dict(os.environ, DIPS_COPY_THREADS=th, DIPS_COPY_AFFINITY=aff, DIPS_CALLBACK_DIRECT=direct,
                       DIPS_CB_BLOCKING=blocking, PFC_BIND_NODE=node)
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", "--calls", str(args.calls)],
                               env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("{")]
            rec = json.loads(line[-1]) if line else {"failed": p.stderr[-800:]}
            rec.update({"round": r, "DIPS_COPY_THREADS": int(th), "DIPS_COPY_AFFINITY": int(aff),
                        "DIPS_CALLBACK_DIRECT": int(direct), "DIPS_CB_BLOCKING": int(blocking),
                        "PFC_BIND_NODE": node})
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
