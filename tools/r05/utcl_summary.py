#!/usr/bin/env python3
"""utcl_summary.py -- medians of the rocprofv3 counters per run of
build/alloc_policy_ab under --pmc (tools/r05/tlb_pmc.sh, wg16_ab.sh): one
line per consecutive group of series dispatches (S0 = the contiguous
schedule, P = part-major, P16 / Px = the probe variants), in dispatch order,
which is the order of the tool's runs (buffer #0 first).
Usage: python tools/r05/utcl_summary.py <run_counter_collection.csv> ...
"""
import collections
import csv
import statistics
import sys


def main():
    for path in sys.argv[1:]:
        by = collections.OrderedDict()
        for r in csv.DictReader(open(path)):
            d = by.setdefault(int(r["Dispatch_Id"]), {
                "name": r["Kernel_Name"], "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
        groups = []
        for v in by.values():
            n = v["name"]
            tag = ("S0" if "series_v2" in n else "P16" if "wg16" in n else "Px" if "xcd" in n
                   else "P" if "parts_isi" in n else None)
            if tag is None:
                continue
            if not groups or groups[-1][0] != tag:
                groups.append((tag, []))
            groups[-1][1].append(v)
        print(path)
        for tag, vs in groups:
            keys = [k for k in vs[0] if k != "name"]
            med = {k.replace("TCP_UTCL1_", ""): round(statistics.median(v[k] for v in vs), 3 if k == "ms" else None)
                   for k in keys}
            print(f"  {tag:4s} n={len(vs):2d} " + " ".join(f"{k}={x}" for k, x in med.items()))


if __name__ == "__main__":
    main()
