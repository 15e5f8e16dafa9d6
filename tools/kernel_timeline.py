#!/usr/bin/env python3
"""kernel_timeline.py -- from a rocprofv3 --kernel-trace CSV: the dispatches of
one kernel grouped into calls (a gap of more than GAP us starts a new call),
per call the start / end of each dispatch in us from the call's first start,
and the busy span.  Usage: kernel_timeline.py DIR KERNEL_SUBSTRING [GAP_US]"""
import csv
import glob
import os
import sys


def main():
    d, kern = sys.argv[1], sys.argv[2]
    gap = float(sys.argv[3]) if len(sys.argv) > 3 else 300.0
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    calls, cur = [], []
    for s, e in rows:
        if cur and (s - cur[-1][1]) / 1e3 > gap:
            calls.append(cur)
            cur = []
        cur.append((s, e))
    if cur:
        calls.append(cur)
    for c in calls[-8:]:
        t0 = c[0][0]
        parts = " ".join(f"[{(s - t0) / 1e3:.0f} {(e - t0) / 1e3:.0f}]" for s, e in c)
        span = (max(e for _, e in c) - t0) / 1e3
        busy = sum(e - s for s, e in c) / 1e3
        print(f"{len(c)} dispatches, span {span:.0f} us, summed {busy:.0f} us: {parts}")


if __name__ == "__main__":
    main()
