#!/usr/bin/env python3
"""sweep_summary.py -- per BASELINE.json config, the series kernel's dispatches
under rocprofv3 (tools/r05/sweep_prof.sh): median duration from the kernel
trace, HBM bytes per dispatch from FETCH_SIZE (x2, the gfx950 wide-stream
correction) + WRITE_SIZE, and both against the config's algorithmic bytes
(W * H * C * frames read once).

The sweep runs the configs in order, one series-kernel launch shape per
config; dispatches are grouped by (kernel, grid size) in order of first
appearance and the largest group of each config's shape is taken (the parity
spot check launches smaller grids).
Usage: python tools/r05/sweep_summary.py <dir with kt/, FETCH_SIZE/, WRITE_SIZE/>
"""
import collections
import csv
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from tools.config_sweep import CONFIGS  # noqa: E402

SERIES = ("series_v2_kernel", "series_fast_kernel", "series_gray")


def groups_from(path, value_col=None, counter=None):
    """Consecutive runs of series dispatches with one (kernel, grid), in
    dispatch order: [(key, [values])]."""
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not any(s in name for s in SERIES) or (counter and r["Counter_Name"] != counter):
            continue
        key = (name.replace("(anonymous namespace)::", "").split("(")[0], int(r["Grid_Size"]) if "Grid_Size" in r else int(r["Grid_Size_X"]))
        v = float(r[value_col]) if value_col else (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        rows.append((int(r["Dispatch_Id"]), key, v))
    out = []
    for _, key, v in sorted(rows):
        if not out or out[-1][0] != key:
            out.append((key, []))
        out[-1][1].append(v)
    return out


def main():
    d = sys.argv[1]
    kt = groups_from(os.path.join(d, "kt", "run_kernel_trace.csv"))
    fe = groups_from(os.path.join(d, "FETCH_SIZE", "run_counter_collection.csv"), "Counter_Value", "FETCH_SIZE")
    wr = groups_from(os.path.join(d, "WRITE_SIZE", "run_counter_collection.csv"), "Counter_Value", "WRITE_SIZE")
    print(f"{'config':64s} {'kernel':44s} {'grid':>7s} {'n':>2s} {'ms':>7s} {'alg GB':>7s} {'HBM GB':>7s} "
          f"{'HBM/alg':>7s} {'%8TB/s':>6s}")
    # the i-th config's group: the i-th run whose duration fits the config's
    # bytes at >= 30 % of 8 TB/s (the parity spot checks are small launches)
    big = [i for i, (k, v) in enumerate(kt) if k[1] > 1024]
    gi = 0
    for name, W, H, C, F, mode, tau in CONFIGS:
        alg = W * H * C * F
        while gi < len(big) and alg / (statistics.median(kt[big[gi]][1]) / 1e3) / 8e12 < 0.3:
            gi += 1
        if gi >= len(big):
            print(f"{name[:64]:64s} (no matching dispatch group)")
            continue
        i = big[gi]
        gi += 1
        (kname, grid), durs = kt[i]
        ms = statistics.median(durs)
        # the counter passes run the same sequence: the run with the same
        # position among the runs of this (kernel, grid)
        nth = sum(1 for k, _ in kt[:i] if k == (kname, grid))

        def pick(groups):
            same = [v for k, v in groups if k == (kname, grid)]
            return statistics.median(same[nth]) if nth < len(same) else float("nan")
        hbm = pick(fe) * 1024 * 2 + pick(wr) * 1024
        print(f"{name[:64]:64s} {kname[-44:]:44s} {grid:7d} {len(durs):2d} {ms:7.3f} {alg / 1e9:7.2f} "
              f"{hbm / 1e9:7.2f} {hbm / alg:7.4f} {alg / (ms / 1e3) / 8e12 * 100:6.1f}")


if __name__ == "__main__":
    main()
