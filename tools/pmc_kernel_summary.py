#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (one directory per pass under ROOT) for
the dispatches of one kernel: per counter, the value of the longest dispatch
(the full-batch launch) and derived LDS figures (bank-conflict cycles per LDS
instruction, LDS-active share of the kernel's cycles).
Usage: pmc_kernel_summary.py ROOT KERNEL_SUBSTRING"""
import csv
import glob
import json
import os
import sys


def main():
    root, kern = sys.argv[1], sys.argv[2]
    vals, dur = {}, None
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(d):
            continue
        rows = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    rows.setdefault(int(r["Dispatch_Id"]), []).append(r)
        if not rows:
            continue
        # the longest dispatch of the pass: the full-batch launch
        did = max(rows, key=lambda k: int(rows[k][0]["End_Timestamp"]) - int(rows[k][0]["Start_Timestamp"]))
        r0 = rows[did][0]
        dur = (int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])) * 1e-9
        for r in rows[did]:
            vals[r["Counter_Name"]] = float(r["Counter_Value"])
    out = {"kernel": kern, "duration_s_profiled": dur, "counters": vals}
    lds = vals.get("SQ_INSTS_LDS")
    if lds:
        if "SQ_LDS_BANK_CONFLICT" in vals:
            out["bank_conflict_cycles_per_lds_inst"] = round(vals["SQ_LDS_BANK_CONFLICT"] / lds, 3)
        if "SQ_LDS_IDX_ACTIVE" in vals:
            out["lds_idx_active_cycles_per_lds_inst"] = round(vals["SQ_LDS_IDX_ACTIVE"] / lds, 3)
    if "SQ_LDS_BANK_CONFLICT" in vals and "SQ_LDS_IDX_ACTIVE" in vals and vals["SQ_LDS_IDX_ACTIVE"]:
        out["conflict_share_of_lds_active"] = round(vals["SQ_LDS_BANK_CONFLICT"] / vals["SQ_LDS_IDX_ACTIVE"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
