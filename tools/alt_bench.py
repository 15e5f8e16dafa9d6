#!/usr/bin/env python3
"""alt_bench.py -- measurement of the dips_alt operator.

Workload: 3840x2160 RGBA8 synthetic frames resident in HBM (the dips_alt
front-end converts every decoded frame to RGBA, dips_alt/src/lib.rs:621-631),
the run_dips_on_file loop with FRAME_COUNT = 2 textures and the default
DiPsProperties (colorize, window 1, sigmoid, scalar 5; mod.rs:176-186), one
snapshot on the third frame.  A step = one dips_alt_send_frames pass over the
batch (alt_batch_kernel).  Algorithmic HBM bytes per frame = W*H*4 read +
W*H*4 written; roofline = those bytes / the kernel's hipEvent time.
cpu_baseline = the oracle's DiPsCompute (oracle/dips_oracle.c) on a few of
the same frames, one thread.

Prints one JSON line.  Run on the GPU box: python tools/alt_bench.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-frames", type=int, default=10)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "alt_pmc_traffic.json"),
                    help="HBM traffic per launch measured by profiles/collect_alt_pmc.sh")
    ap.add_argument("--kernel", choices=["lut", "arith"], default="lut",
                    help="lut: alt_batch_kernel with the epilogue table (default); arith: per-pixel epilogue")
    args = ap.parse_args()

    import torch
    from dips_amd import DiffSeriesOperator, PixelFormat
    from dips_amd.alt import DiPsCompute

    W, H, F = args.width, args.height, args.frames
    dev = torch.device("cuda", 0)
    frames = torch.empty((F, H, W, 4), dtype=torch.uint8, device=dev)
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(frames, W, H, 0xD1B5, 0)
    op.close()
    out = torch.empty_like(frames)
    flags = [t == 2 for t in range(F)]
    c = DiPsCompute(2, H, W, time_kernel=True, crosscheck=args.kernel == "arith")
    for _ in range(args.warmup):
        c.send_frames_device(frames, out, flags)
    torch.cuda.synchronize()
    c.kernel_time(reset=True)
    t = time.perf_counter()
    for _ in range(args.steps):
        c.send_frames_device(frames, out, flags)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t
    kms, launches = c.kernel_time()
    kernel_ms = kms / max(launches, 1)

    # parity spot check + CPU baseline on the first frames (fresh state)
    from oracle import oracle
    n_cpu = max(3, args.cpu_frames)
    host = frames[:n_cpu].cpu().numpy()
    ref = oracle.AltCompute(2, W, H, True, 1, 5.0, 0, 0)
    t0 = time.perf_counter()
    want = np.stack([ref.send_frame(host[k], k == 2) for k in range(n_cpu)])
    cpu_s = time.perf_counter() - t0
    c2 = DiPsCompute(2, H, W)
    o2 = torch.empty_like(frames[:n_cpu])
    c2.send_frames_device(frames[:n_cpu], o2, flags[:n_cpu])
    torch.cuda.synchronize()
    match = bool(np.array_equal(o2.cpu().numpy(), want))
    c2.close()
    c.close()

    algo = F * W * H * 8
    achieved = algo / (kernel_ms / 1e3) / 1e9
    traffic, traffic_src = None, None
    if os.path.exists(args.pmc_json):
        import hashlib
        from dips_amd import _lib as L
        with open(L.LIB_PATH, "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()
        with open(args.pmc_json) as f:
            pmc = json.load(f)
        # only a measurement of this very library build and workload counts
        if (pmc.get("width"), pmc.get("height"), pmc.get("frames")) == (W, H, F) and pmc.get("lib_sha256") == sha \
                and args.kernel == "lut":
            traffic, traffic_src = pmc.get("hbm_bytes_per_launch"), pmc.get("source")
        else:
            traffic_src = "traffic null: the PMC file is of another library build, workload or kernel form"
    print(json.dumps({
        "metric": "dips_alt frames/s + achieved HBM GB/s, 4K RGBA8",
        "value": round(F * args.steps / elapsed, 2), "unit": "frames/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "dtype": "u8/f32", "data": "synthetic (shared integer-hash generator, frames generated in HBM)",
        "config": {"workload": f"{W}x{H} RGBA8, {F} frames, dips_alt run loop, FRAME_COUNT=2, default "
                               "DiPsProperties (colorize, window 1, sigmoid, scalar 5)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     **({"traffic_source": traffic_src} if traffic_src else {}),
                     "kernel": ("alt_batch_kernel<0,0,0,true,2,LUT=true> (epilogue table in LDS)"
                                if args.kernel == "lut" else "alt_batch_kernel<0,0,1,true,2> (arithmetic epilogue)"),
                     "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": algo},
        "cpu_baseline": {"value": round(n_cpu / cpu_s, 4), "unit": "frames/s", "cores": 1, "kind": "port",
                         "sample": f"first {n_cpu} frames, oracle/dips_oracle.c DiPsCompute, {cpu_s:.2f} s",
                         "matches_gpu": match},
    }), flush=True)


if __name__ == "__main__":
    main()
